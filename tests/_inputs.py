"""Seeded inputs shared by the GPU workers and the checking side."""
import numpy as np

import gen_golden


def source(op, dtype, n, seed, pe):
    rng = np.random.default_rng(seed * 1009 + pe)
    if n == 0:
        import oracle
        return np.zeros(0, dtype=oracle.NP[dtype])
    return gen_golden.values(rng, op, dtype, n)
