#!/usr/bin/env python3
"""Every (op, type) pair of the 44 through the every-member fold at the N = 8
reduce-scatter shape (mi355_combine_orders: 8 sources x 32 MiB -> 8 outputs,
algorithmic bytes 16 x 32 MiB), and through the plain 8-source fold
(mi355_combine, 8 x 32 MiB -> 1 output, 9 x 32 MiB): per-launch time from 10
back-to-back launches, GB/s and the fraction of the 8 TB/s HBM peak, so the
pairs furthest below the roofline stand out. Inputs: gen_golden's values for
the pair (realistic for its type, specials included). Measurement tool.
usage: python3 tools/probes/orders_sweep.py OUT.jsonl [op/dtype ...]   (default: all 44)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
import shmem_reduce  # noqa: E402

SHARD = 32 << 20
K = int(os.environ.get("ORDERS_SWEEP_SOURCES", "8"))   # sources (the N = K shape)


def values(rng, dtype, n):
    t = oracle.NP[dtype]
    if dtype in ("short", "int", "long", "longlong"):
        info = np.iinfo(t)
        return rng.integers(info.min, info.max, n, dtype=t, endpoint=True)
    if dtype.startswith("complex"):
        base = np.float32 if dtype == "complexf" else np.float64
        out = np.empty(n, dtype=t)
        out.real, out.imag = values(rng, "double", n).astype(base), values(rng, "double", n).astype(base)
        return out
    x = (rng.random(n) - 0.5) * np.exp2(rng.integers(-4, 5, n))
    return x.astype(t)


def main():
    out = open(sys.argv[1], "w")
    os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str(2 * K * SHARD + (64 << 20)))
    os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
    shm = shmem_reduce.Shmem()
    shm.init()
    src, dst = shm.malloc_device(K * SHARD), shm.malloc_device(K * SHARD)
    srcs = [src + q * SHARD for q in range(K)]
    dsts = [dst + q * SHARD for q in range(K)]
    pairs = [tuple(a.split("/")) for a in sys.argv[2:]] or oracle.PAIRS
    for op, dtype in pairs:
        es = np.dtype(oracle.NP[dtype]).itemsize
        n = SHARD // es
        rng = np.random.default_rng(9)
        block = values(rng, dtype, 1 << 16)   # tiled to full size
        for q in range(K):
            shm.put(srcs[q], np.resize(np.roll(block, 977 * q), n))
        rec = {"op": op, "dtype": dtype}
        for name, launch, nbytes in (
                ("orders", lambda: shm.combine_orders(op, dtype, dsts, srcs, n), 2 * K * SHARD),
                ("fold", lambda: shm.combine(op, dtype, dsts[0], srcs, n), (K + 1) * SHARD)):
            for _ in range(2):
                assert launch() == 0
            shm.sync()
            t0 = time.perf_counter()
            for _ in range(10):
                assert launch() == 0
            shm.sync()
            t = (time.perf_counter() - t0) / 10
            rec[name] = {"us": round(t * 1e6, 1), "GB_s": round(nbytes / t / 1e9, 1),
                         "frac": round(nbytes / t / 8e12, 3)}
        out.write(json.dumps(rec) + "\n")
        out.flush()
        print(json.dumps(rec), flush=True)
    shm.finalize()


if __name__ == "__main__":
    main()
