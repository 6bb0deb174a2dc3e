"""CPU: the oracle (our C restatement) against the golden fixtures.

The fixtures' expected outputs were computed with the reference's OWN
compiled operator functions (oracle/gen_golden.py); this pins the oracle's
operators bit-for-bit. When the reference tree is present, the fixtures are
also regenerated and compared, so they cannot drift from the reference.
"""
import json
import os

import numpy as np
import pytest

import oracle
from _compare import assert_match

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load_cases(op, dtype):
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        man = json.load(f)
    cases = man["cases"][f"{op}_{dtype}"]
    z = np.load(os.path.join(GOLDEN, f"golden_{op}_{dtype}.npz"))
    return [(c["npes"], z[f"in_{k}"], z[f"out_{k}"]) for k, c in enumerate(cases)]


def test_manifest_covers_all_44_pairs():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        man = json.load(f)
    assert sorted(man["cases"]) == sorted(f"{op}_{t}" for op, t in oracle.PAIRS)
    assert len(man["cases"]) == 44


@pytest.mark.parametrize("op,dtype", oracle.PAIRS)
def test_oracle_matches_golden(op, dtype):
    for npes, ins, outs in load_cases(op, dtype):
        srcs = [ins[i] for i in range(npes)]
        for me in range(npes):
            got = oracle.reduce_pe(op, dtype, srcs, me)
            # the oracle is compiled by the same gcc: every bit, NaNs included
            assert (oracle.as_value_bytes(got, dtype) == oracle.as_value_bytes(outs[me], dtype)).all(), \
                (op, dtype, npes, me)


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (no /root/reference)")
@pytest.mark.parametrize("op,dtype", oracle.PAIRS)
def test_golden_matches_reference_ops(op, dtype):
    for npes, ins, outs in load_cases(op, dtype):
        srcs = [ins[i] for i in range(npes)]
        for me in range(npes):
            ref = oracle.ref_reduce_pe(op, dtype, srcs, me)
            assert (oracle.as_value_bytes(ref, dtype) == oracle.as_value_bytes(outs[me], dtype)).all()


def test_fp_order_matters_between_pes():
    """The reference's PEs disagree in the last bits for FP sums:
    the fixtures must contain such cases, or they could not catch a wrong order."""
    differing = 0
    for npes, ins, outs in load_cases("sum", "double"):
        for me in range(1, npes):
            differing += int((outs[me].view(np.uint64) != outs[0].view(np.uint64)).sum())
    assert differing > 0


def test_integer_wraps_like_gcc():
    a = np.array([2**31 - 1, -2**31], dtype=np.int32)
    b = np.array([1, -1], dtype=np.int32)
    assert list(oracle.reduce_pe("sum", "int", [a, b], 0)) == [-2**31, 2**31 - 1]
    s = np.array([300], dtype=np.int16)
    assert list(oracle.reduce_pe("prod", "short", [s, s], 0)) == [np.int16(90000 - 65536 * 1)]


def test_minmax_is_a_select_not_ieee_minnum():
    """a < b ? a : b returns b when either is NaN, and the later operand on +-0 ties."""
    nan = np.float64("nan")
    a = np.array([nan, 1.0, 0.0, -0.0], dtype=np.float64)
    b = np.array([1.0, nan, -0.0, 0.0], dtype=np.float64)
    got = oracle.reduce_pe("min", "double", [a, b], 0)
    assert got[0] == 1.0 and np.isnan(got[1])
    assert np.signbit(got[2]) and not np.signbit(got[3])


# ---------------------------------------------------------------------------
# NaN payloads (golden_nan_*): which NaN comes out of the reference's float,
# double and complex sum/prod
# ---------------------------------------------------------------------------
def load_nan_cases(op, dtype):
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        man = json.load(f)
    cases = man["nan_cases"][f"{op}_{dtype}"]
    z = np.load(os.path.join(GOLDEN, f"golden_nan_{op}_{dtype}.npz"))
    return [(c["npes"], z[f"in_{k}"], z[f"out_{k}"]) for k, c in enumerate(cases)]


NAN_PAIRS = [(op, t) for op in ("sum", "prod") for t in ("float", "double", "complexf", "complexd")]


@pytest.mark.parametrize("op,dtype", NAN_PAIRS)
def test_oracle_matches_nan_golden(op, dtype):
    for npes, ins, outs in load_nan_cases(op, dtype):
        srcs = [ins[i] for i in range(npes)]
        for me in range(npes):
            got = oracle.reduce_pe(op, dtype, srcs, me)
            assert (oracle.as_value_bytes(got, dtype) == oracle.as_value_bytes(outs[me], dtype)).all(), \
                (op, dtype, npes, me)


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (no /root/reference)")
@pytest.mark.parametrize("op,dtype", NAN_PAIRS)
def test_nan_golden_matches_reference_ops(op, dtype):
    for npes, ins, outs in load_nan_cases(op, dtype):
        srcs = [ins[i] for i in range(npes)]
        for me in range(npes):
            ref = oracle.ref_reduce_pe(op, dtype, srcs, me)
            assert (oracle.as_value_bytes(ref, dtype) == oracle.as_value_bytes(outs[me], dtype)).all()


def test_nan_golden_is_payload_rich():
    """The families must hold results whose NaNs differ in sign and payload,
    and invalid-operation NaNs, or they could not pin the rule below."""
    for op in ("sum", "prod"):
        outs = np.concatenate([o.ravel() for _, _, o in load_nan_cases(op, "double")])
        nans = outs.view(np.uint64)[np.isnan(outs)]
        assert len(np.unique(nans)) > 100, op
        assert (nans == np.uint64(0xFFF8000000000000)).any(), op      # SSE's "indefinite"
        assert ((nans >> np.uint64(63)) == 0).any(), op                # positive NaNs too


# The rule the GPU kernels restate (osss-gasnet_amd/csrc/ops.h x86_result,
# cmul), restated once more in numpy and checked here against the reference's
# compiled code, so the GPU tests check an algorithm already pinned on the CPU.
_NANBITS = {np.float32: (np.uint32, 0x00400000, 0xFFC00000), np.float64: (np.uint64, 0x0008000000000000,
                                                                           0xFFF8000000000000)}


def x86_result(r, a, b):
    """SSE: a NaN result is the first NaN operand, quieted; else (an invalid
    operation) the negative 'indefinite' QNaN."""
    u_t, quiet, indef = _NANBITS[r.dtype.type]
    ua, ub = a.view(u_t) | u_t(quiet), b.view(u_t) | u_t(quiet)
    pick = np.where(np.isnan(a), ua, np.where(np.isnan(b), ub, u_t(indef)))
    return np.where(np.isnan(r), pick.view(r.dtype), r)


def x86_cmul(a, b, c, d):
    """libgcc __muldc3/__mulsc3 as compiled in this image (ops.h cmul)."""
    with np.errstate(all="ignore"):
        ac, bd = x86_result(a * c, a, c), x86_result(b * d, b, d)
        ad, bc = x86_result(a * d, a, d), x86_result(c * b, c, b)
        x, y = x86_result(ac - bd, ac, bd), x86_result(ad + bc, ad, bc)
        t = a.dtype.type
        _, _, indef = _NANBITS[t]
        for i in np.nonzero(np.isnan(x) & np.isnan(y))[0]:
            A, B, C, D = a[i], b[i], c[i], d[i]
            recalc = False
            if np.isinf(A) or np.isinf(B):
                A, B = np.copysign(t(1 if np.isinf(A) else 0), A), np.copysign(t(1 if np.isinf(B) else 0), B)
                C = np.copysign(t(0), C) if np.isnan(C) else C
                D = np.copysign(t(0), D) if np.isnan(D) else D
                recalc = True
            if np.isinf(C) or np.isinf(D):
                C, D = np.copysign(t(1 if np.isinf(C) else 0), C), np.copysign(t(1 if np.isinf(D) else 0), D)
                A = np.copysign(t(0), A) if np.isnan(A) else A
                B = np.copysign(t(0), B) if np.isnan(B) else B
                recalc = True
            if not recalc and (np.isinf(ac[i]) or np.isinf(bd[i]) or np.isinf(ad[i]) or np.isinf(bc[i])):
                A, B, C, D = [np.copysign(t(0), v) if np.isnan(v) else v for v in (A, B, C, D)]
                recalc = True
            if recalc:
                xi, yi = t(np.inf) * (A * C - B * D), t(np.inf) * (A * D + B * C)
                x[i] = np.array(indef, dtype=_NANBITS[t][0]).view(t) if np.isnan(xi) else xi
                y[i] = np.array(indef, dtype=_NANBITS[t][0]).view(t) if np.isnan(yi) else yi
    return x, y


def restated_op(op, dtype, acc, src):
    with np.errstate(all="ignore"):
        if dtype in ("float", "double"):
            return x86_result(acc + src if op == "sum" else acc * src, acc, src)
        a, b, c, d = acc.real.copy(), acc.imag.copy(), src.real.copy(), src.imag.copy()
        out = np.empty_like(acc)
        if op == "sum":
            out.real = x86_result(a + c, a, c)
            # gcc's float complex add takes the incoming imaginary part first
            out.imag = x86_result(d + b, d, b) if dtype == "complexf" else x86_result(b + d, b, d)
        else:
            out.real, out.imag = x86_cmul(a, b, c, d)
        return out


@pytest.mark.parametrize("op,dtype", NAN_PAIRS)
def test_restated_x86_rule_matches_nan_golden(op, dtype):
    for npes, ins, outs in load_nan_cases(op, dtype):
        for me in range(npes):
            order = [me] + [i for i in range(npes) if i != me]
            acc = ins[order[0]].copy()
            for i in order[1:]:
                acc = restated_op(op, dtype, acc, ins[i])
            bad = np.nonzero((oracle.as_value_bytes(acc, dtype) != oracle.as_value_bytes(outs[me], dtype)).any(axis=1))[0]
            assert len(bad) == 0, (op, dtype, npes, me, len(bad), acc[bad[:3]], outs[me][bad[:3]])
