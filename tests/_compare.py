"""Bit comparison helpers shared by the parity tests (test infrastructure)."""
import os

import numpy as np

import oracle

# Every value bit must match, NaN payloads and signs included: the kernels
# restate SSE's NaN rule and libgcc's complex-multiply operand order
# (osss-gasnet_amd/csrc/ops.h; pinned on the CPU by tests/test_oracle_golden.py
# against the reference's compiled operators). SHMEM_TEST_RELAXED_NAN=1 lets
# two NaNs match whatever their payloads (the pre-round-5 latitude), for
# comparing with an older build.
FP = {"float", "double", "complexf", "complexd"}
RELAXED_NAN = os.environ.get("SHMEM_TEST_RELAXED_NAN") == "1"


def mismatches(got, want, op, dtype, strict=False):
    """Indices where got != want (every value bit; see above)."""
    got = np.ascontiguousarray(got, dtype=oracle.NP[dtype])
    want = np.ascontiguousarray(want, dtype=oracle.NP[dtype])
    assert got.shape == want.shape, (got.shape, want.shape)
    if got.size == 0:
        return np.zeros(0, dtype=np.int64)
    eq = (oracle.as_value_bytes(got, dtype) == oracle.as_value_bytes(want, dtype)).all(axis=1)
    if dtype in FP and op in ("sum", "prod") and RELAXED_NAN and not strict:
        if dtype.startswith("complex"):
            def part_ok(g, w):
                g, w = np.ascontiguousarray(g), np.ascontiguousarray(w)
                return (np.isnan(g) & np.isnan(w)) | (g.view(np.uint8).reshape(len(g), g.itemsize) ==
                                                      w.view(np.uint8).reshape(len(w), w.itemsize)).all(axis=1)
            nan_ok = part_ok(got.real, want.real) & part_ok(got.imag, want.imag)
        else:
            nan_ok = np.isnan(got) & np.isnan(want)
        eq = eq | nan_ok
    return np.nonzero(~eq)[0]


def assert_match(got, want, op, dtype, ctx="", strict=False):
    bad = mismatches(got, want, op, dtype, strict)
    if len(bad):
        i = bad[0]
        g = np.ascontiguousarray(got, dtype=oracle.NP[dtype])
        w = np.ascontiguousarray(want, dtype=oracle.NP[dtype])
        raise AssertionError(f"{ctx} {op}/{dtype}: {len(bad)} of {len(got)} elements differ; "
                             f"first at {i}: got {g[i]!r} ({g[i:i + 1].view(np.uint8).tobytes().hex()}) "
                             f"want {w[i]!r} ({w[i:i + 1].view(np.uint8).tobytes().hex()})")
