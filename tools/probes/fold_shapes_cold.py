#!/usr/bin/env python3
"""Launch shapes of the plain 8-source fold from HBM (round 6 probe).

The order-free operators' P2P shard at N = 8 is a plain 8-source fold with one
output (BASELINE config 4's longlong and: 8 x 8 MiB -> 1; bench.py leg
rs_shard_n8_longlong_and). Its shape (combine_kernels.h Shape<8>: 4 vectors
per lane, 8 blocks per CU) was tuned at 256 MiB per source. This times the
library's launch (mi355_combine) and the shapes of a tools/peer_shapes.hip
build (SHAPES_LIB, default tools/probes/liborderswindow.so) on bench.py's
staggered layout, warm and cold (>= 2.25 GiB of disjoint sets), and checks
every variant's output against the library's. One JSON line per (size, shape).

run from the repo root on the GPU box: python3 tools/probes/fold_shapes_cold.py
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "osss-gasnet_amd"))
import shmem_reduce  # noqa: E402

STAGGER = 4352
FOOT = 2304 << 20
PEAK = 8000.0


def main():
    os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", "64M")
    os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
    shm = shmem_reduce.Shmem()
    shm.init()
    L, vp = shm.lib, ctypes.c_void_p
    P = ctypes.CDLL(os.environ.get("SHAPES_LIB", os.path.join(ROOT, "tools", "probes", "liborderswindow.so")))
    P.peer_shapes_fold_long_and.argtypes = [ctypes.c_int, vp, ctypes.POINTER(vp), ctypes.c_size_t, vp, vp, vp]
    L.mi355_time_next_launch.argtypes = [vp, vp]
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    reps = 40
    ev = [vp() for _ in range(2 * reps)]
    for e in ev:
        L.hipEventCreate(ctypes.byref(e))
    u, b = ctypes.c_int(), ctypes.c_int()
    for mib in [int(x) for x in os.environ.get("FOLD_MIB", "8,32").split(",")]:
        nb = mib << 20
        n = nb // 8
        span = nb + STAGGER
        set_bytes = 9 * span
        sets = max(2, -(-FOOT // set_bytes))
        pool = vp()
        assert L.hipMalloc(ctypes.byref(pool), ctypes.c_size_t(sets * set_bytes)) == 0
        base = pool.value
        rng = np.random.default_rng(9)
        xs = [rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64) | rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
              for _ in range(8)]
        for j in range(sets):
            for q in range(8):
                shm.put(base + j * set_bytes + q * span, xs[q])

        def bufs(j):
            s = [base + j * set_bytes + q * span for q in range(8)]
            return base + j * set_bytes + 8 * span, s, (vp * 8)(*s)

        def launcher(v):
            if v < 0:
                return lambda j, e0, e1: (L.mi355_time_next_launch(e0, e1) if e0 else None,
                                          shm.combine("and", "longlong", bufs(j)[0], bufs(j)[1], n))[1]
            return lambda j, e0, e1: P.peer_shapes_fold_long_and(v, bufs(j)[0], bufs(j)[2], n, e0, e1, None)

        def timed(f, cold):
            for j in range(sets):
                assert f(j, None, None) == 0
            shm.sync()
            for r in range(reps):
                assert f(r % sets if cold else 0, ev[2 * r], ev[2 * r + 1]) == 0
            shm.sync()
            ts = []
            for r in range(reps):
                ms = ctypes.c_float()
                L.hipEventElapsedTime(ctypes.byref(ms), ev[2 * r], ev[2 * r + 1])
                ts.append(ms.value * 1e3)
            return float(np.mean(ts))

        alg = 9 * nb
        ref = None
        for v in [-1] + [v for v in range(P.peer_shapes_count()) if P.peer_shapes_pipe(v) == 0]:
            f = launcher(v)
            w, c = timed(f, False), timed(f, True)
            h = hashlib.sha256(shm.get(bufs(0)[0], n, "longlong").view(np.uint8)).hexdigest()
            ref = ref or h
            if v >= 0:
                P.peer_shapes_describe(v, ctypes.byref(u), ctypes.byref(b))
                shape = f"{u.value} vectors/lane, {b.value} blocks/CU"
            else:
                shape = "library"
            print(json.dumps({"kernel": "combine_vec<and,longlong,8>", "bytes_per_source": nb, "shape": shape,
                              "warm_us": round(w, 2), "warm_frac": round(alg / w / 1e3 / PEAK, 4),
                              "cold_us": round(c, 2), "cold_frac": round(alg / c / 1e3 / PEAK, 4), "sets": sets,
                              "same_output": h == ref}), flush=True)
        L.hipFree(pool)
    shm.finalize()


if __name__ == "__main__":
    main()
