#!/usr/bin/env python3
"""Every-member-order fold (mi355_combine_orders) against the plain fold
(mi355_combine) on one GPU, per element type, at the per-GPU reduce-scatter
shape of an N-PE call on 256 MiB per PE (N sources of 256/N MiB; orders
writes N outputs, the fold one). Kernel time from HIP event stamps (median of
reps). Measurement tool: prints one JSON line per (type, N).

usage: orders_bench.py [reps] [dtype,dtype,...]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "osss-gasnet_amd"))
import shmem_reduce  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
S = 256 << 20
os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str(2 * S + (64 << 20)))
os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
os.environ.setdefault("SHMEM_DEVICE_ORDER_SIZE", "1M")
shm = shmem_reduce.Shmem()
shm.init()
L = shm.lib
L.mi355_time_next_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
src_arena, out_arena = shm.malloc_device(S), shm.malloc_device(S)
rand = np.random.default_rng(3).random(S // 8) - 0.5
shm.put(out_arena, np.zeros(S // 8))


def fill(dtype):
    """source values of the type (long double: normal x87 values, not double bit patterns)"""
    if dtype == "longdouble":
        shm.put(src_arena, rand[:S // 16].astype(np.longdouble))
    else:
        shm.put(src_arena, rand)
e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
L.hipEventCreate(ctypes.byref(e0))
L.hipEventCreate(ctypes.byref(e1))


def timed(launch):
    for _ in range(3):
        assert launch() == 0
    shm.sync()
    ts = []
    for _ in range(reps):
        L.mi355_time_next_launch(e0, e1)
        assert launch() == 0
        L.hipEventSynchronize(e1)
        ms = ctypes.c_float()
        L.hipEventElapsedTime(ctypes.byref(ms), e0, e1)
        ts.append(ms.value * 1e-3)
    return float(np.median(ts))


for op, dtype in [("sum", "double"), ("sum", "float"), ("max", "float"), ("min", "double"), ("prod", "complexd"),
                  ("sum", "complexf"), ("sum", "longdouble"), ("prod", "longdouble"), ("max", "longdouble")]:
    if only and dtype not in only:
        continue
    es = np.dtype(shmem_reduce.NP[dtype]).itemsize
    fill(dtype)
    for npes in (2, 4, 8):
        shard = S // npes
        n = shard // es
        srcs = [src_arena + k * shard for k in range(npes)]
        outs = [out_arena + k * shard for k in range(npes)]
        t_fold = timed(lambda: shm.combine(op, dtype, outs[0], srcs, n))
        t_ord = timed(lambda: shm.combine_orders(op, dtype, outs, srcs, n))
        print(json.dumps({"op": op, "dtype": dtype, "npes": npes, "shard_MiB": shard >> 20,
                          "fold_us": round(t_fold * 1e6, 1), "fold_TB_s": round((npes + 1) * shard / t_fold / 1e12, 2),
                          "orders_us": round(t_ord * 1e6, 1),
                          "orders_TB_s": round(2 * npes * shard / t_ord / 1e12, 2),
                          "orders_over_fold": round(t_ord / t_fold, 2)}), flush=True)
shm.finalize()
