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
