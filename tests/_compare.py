"""Bit comparison helpers shared by the parity tests (test infrastructure)."""
import os

import numpy as np

import oracle

# long double is x87 arithmetic restated in software (x80.h), NaN rule
# included, so its NaN payloads must match too; the hardware float types
# follow the IEEE-754 latitude below unless SHMEM_TEST_STRICT_NAN=1
FP = {"float", "double", "complexf", "complexd"}
STRICT_NAN = os.environ.get("SHMEM_TEST_STRICT_NAN") == "1"


def mismatches(got, want, op, dtype):
    """Indices where got != want. Integer/logical, min/max and long double:
    every value bit must match. float/double (and complex) sum/prod: bits must
    match, except that two NaNs match (IEEE 754 leaves NaN payload propagation
    open; the x86 host and gfx950 differ) -- unless SHMEM_TEST_STRICT_NAN=1."""
    got = np.ascontiguousarray(got, dtype=oracle.NP[dtype])
    want = np.ascontiguousarray(want, dtype=oracle.NP[dtype])
    assert got.shape == want.shape, (got.shape, want.shape)
    if got.size == 0:
        return np.zeros(0, dtype=np.int64)
    eq = (oracle.as_value_bytes(got, dtype) == oracle.as_value_bytes(want, dtype)).all(axis=1)
    if dtype in FP and op in ("sum", "prod") and not STRICT_NAN:
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


def assert_match(got, want, op, dtype, ctx=""):
    bad = mismatches(got, want, op, dtype)
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{ctx} {op}/{dtype}: {len(bad)} of {len(got)} elements differ; "
                             f"first at {i}: got {got[i]!r} want {want[i]!r}")
