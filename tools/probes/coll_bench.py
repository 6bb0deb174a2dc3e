#!/usr/bin/env python3
"""Bandwidth of put/get, broadcast and fcollect, one
process per PE (run under tools/oshrun or torch.distributed.run). Prints one
JSON line per op from PE 0. usage: coll_bench.py [MiB per PE] [reps]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "osss-gasnet_amd"))
import shmem_reduce  # noqa: E402

mib = float(sys.argv[1]) if len(sys.argv) > 1 else 64.0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
S = int(mib * (1 << 20)) // 256 * 256
shm = shmem_reduce.Shmem()
npes_env = int(os.environ.get("SHMEM_NPES", os.environ.get("WORLD_SIZE", "1")))
os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str((npes_env + 2) * S + (64 << 20)))
os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "24M")
shm.init()
me, npes = shm.my_pe(), shm.n_pes()
L = shm.lib
vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
src = shm.malloc_device(S)
dst = shm.malloc_device(npes * S)
shm.put(src, np.random.default_rng(me).integers(0, 2**62, S // 8, dtype=np.int64))
ps = shm._psync_ptr
for name, fn, args in [
    ("broadcast64", "shmem_broadcast64", lambda: (dst, src, S // 8, 0, 0, 0, npes, ps)),
    ("fcollect64", "shmem_fcollect64", lambda: (dst, src, S // 8, 0, 0, npes, ps)),
    ("get64 from next PE", "shmem_get64", lambda: (dst, src, S // 8, (me + 1) % npes)),
    ("put64 to next PE", "shmem_put64", lambda: (dst, src, S // 8, (me + 1) % npes)),
]:
    f = getattr(L, fn)
    a = args()
    f.argtypes = [vp if isinstance(x, int) and x > 2**31 else (sz if k == 2 else i) for k, x in enumerate(a)] \
        if False else None
    if fn.startswith("shmem_broadcast"):
        f.argtypes = [vp, vp, sz, i, i, i, i, vp]
    elif fn.startswith("shmem_fcollect"):
        f.argtypes = [vp, vp, sz, i, i, i, vp]
    else:
        f.argtypes = [vp, vp, sz, i]
    for _ in range(2):
        f(*a)
    shm.barrier_all()
    t0 = time.perf_counter()
    for _ in range(reps):
        f(*a)
    shm.barrier_all()
    t = (time.perf_counter() - t0) / reps
    moved = {"broadcast64": S, "fcollect64": npes * S}.get(name, S)  # bytes landing in this PE's target
    if me == 0:
        print(json.dumps({"op": name, "npes": npes, "bytes_per_pe": S, "us_per_call": round(t * 1e6, 1),
                          "GB_s_into_each_pe": round(moved / t / 1e9, 1)}), flush=True)
shm.free_device(dst)
shm.free_device(src)
shm.finalize()
