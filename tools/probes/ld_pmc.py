#!/usr/bin/env python3
"""Launch the every-member folds of one N = 8 reduce-scatter shape (8 sources
x 32 MiB, 8 outputs) for long double and double sum, five times each, for a
rocprofv3 --pmc pass (is the x87 software sum VALU-bound?). Measurement tool.
usage: rocprofv3 --pmc <counters> -- python3 tools/probes/ld_pmc.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "osss-gasnet_amd"))
import shmem_reduce  # noqa: E402

S = 256 << 20
os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str(2 * S + (64 << 20)))
os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
os.environ.setdefault("SHMEM_DEVICE_ORDER_SIZE", "1M")
shm = shmem_reduce.Shmem()
shm.init()
src, out = shm.malloc_device(S), shm.malloc_device(S)
k, shard = 8, S // 8
for dtype, es in (("longdouble", 16), ("double", 8)):
    x = (np.random.default_rng(3).random(S // 16) - 0.5)
    shm.put(src, x.astype(np.longdouble) if dtype == "longdouble" else np.concatenate([x, x]))
    n = shard // es
    srcs = [src + q * shard for q in range(k)]
    dsts = [out + q * shard for q in range(k)]
    for _ in range(5):
        assert shm.combine_orders("sum", dtype, dsts, srcs, n) == 0
    shm.sync()
shm.finalize()
print("ok")
