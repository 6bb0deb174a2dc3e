"""BASELINE.json configs as parity cases, with SURVEY.md §8(d)'s input recipes.

  c1   shmem_int_sum_to_all, 2 PEs, n = 1024: src_p[i] = (int)(i*7 + p*1000003)
  c3   shmem_double_sum_to_all, 8 PEs, n = 2^25 (256 MiB):
       src_p[i] = U(-1,1) * (1 + U*2^-40) * 2^k, k in [0,7], seed 1234+p
  c4f  shmem_float_max_to_all, 8 PEs, n = 2^24 (64 MiB): the same recipe in float
  c4l  shmem_longlong_and_to_all, 8 PEs, n = 2^23 (64 MiB): random words whose
       bits are 1 with probability 0.9, seed 99+p
  c5   shmem_double_sum_to_all, 8 PEs, 64 KiB per call, back to back

Shared by the GPU workers (each makes its own source) and the checking side
(which makes every PE's source and runs the oracle on them).
"""
import hashlib

import numpy as np

CONFIGS = {
    "c1": ("sum", "int"),
    "c3": ("sum", "double"),
    "c4f": ("max", "float"),
    "c4l": ("and", "longlong"),
    "c5": ("sum", "double"),
}


def _fp(seed, n, dtype):
    rng = np.random.default_rng(seed)
    u1 = rng.uniform(-1.0, 1.0, n)
    u2 = rng.uniform(0.0, 1.0, n)
    k = rng.integers(0, 8, n)
    return (u1 * (1.0 + u2 * 2.0**-40) * np.exp2(k)).astype(dtype)


def _bits09(seed, n):
    rng = np.random.default_rng(seed)
    out = np.empty(n, dtype=np.uint64)
    chunk = 1 << 18
    for lo in range(0, n, chunk):
        m = min(chunk, n - lo)
        bits = rng.integers(0, 10, (m, 64), dtype=np.uint8) != 0      # P(1) = 0.9
        out[lo:lo + m] = np.packbits(bits, axis=1, bitorder="little").view("<u8").ravel()
    return out.view(np.int64)


def source(config, n, pe, slot=0):
    """PE pe's source for a config (slot: which of several inputs, for c5)."""
    if config == "c1":
        i = np.arange(n, dtype=np.int64)
        return ((i * 7 + pe * 1000003 + slot) & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    if config in ("c3", "c5"):
        return _fp(1234 + pe + 7919 * slot, n, np.float64)
    if config == "c4f":
        return _fp(1234 + pe, n, np.float32)
    if config == "c4l":
        return _bits09(99 + pe, n)
    raise ValueError(config)


def digest(a):
    """SHA-256 of the array's bytes, plus a strided sample for diagnostics."""
    a = np.ascontiguousarray(a)
    step = max(1, len(a) // 4096)
    return hashlib.sha256(a.tobytes()).hexdigest(), a[::step].copy()
