#!/usr/bin/env python3
"""k-source combine microbench on one GPU (tuning/measurement tool).

Simulates the reduce-scatter leg's fold of k PEs' buffers with k local
buffers: dst = src0 (+) src1 (+) ... (+) src(k-1), 256 MiB each, for several
ops/types. Algorithmic bytes (k+1)*S per launch. Kernel time from HIP event
stamps on the library stream (median of reps).
usage: fold_bench.py [MiB] [reps]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "osss-gasnet_amd"))
import shmem_reduce  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
S = mib << 20
os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str(10 * S + (64 << 20)))
os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
shm = shmem_reduce.Shmem()
shm.init()
bufs = [shm.malloc_device(S) for _ in range(9)]
rng = np.random.default_rng(1)
for b in bufs:
    shm.put(b, rng.standard_normal(S // 8))
out = []
for op, dtype in [("sum", "double"), ("sum", "float"), ("xor", "longlong"), ("max", "float"), ("sum", "short"),
                  ("prod", "complexd"), ("sum", "longdouble")]:
    es = np.dtype(shmem_reduce.NP[dtype]).itemsize
    n = S // es
    for k in (1, 2, 3, 4, 8):
        srcs = bufs[1:1 + k]
        for _ in range(3):
            shm.combine(op, dtype, bufs[0], srcs, n)
        shm.sync()
        ts = []
        import ctypes
        shm.lib.mi355_time_next_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        hip = ctypes.CDLL("libamdhip64.so")
        e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
        hip.hipEventCreate(ctypes.byref(e0)); hip.hipEventCreate(ctypes.byref(e1))
        for _ in range(reps):
            shm.lib.mi355_time_next_launch(e0, e1)
            rc = shm.combine(op, dtype, bufs[0], srcs, n)
            assert rc == 0, rc
            hip.hipEventSynchronize(e1)
            ms = ctypes.c_float()
            hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1)
            ts.append(ms.value)
        t = float(np.median(ts)) * 1e-3
        gbs = (k + 1) * S / t / 1e9
        out.append({"op": op, "dtype": dtype, "k": k, "us": round(t * 1e6, 1), "GB_s": round(gbs, 1),
                    "frac_8TBs": round(gbs / 8000, 3)})
        print(json.dumps(out[-1]), flush=True)
shm.finalize()
