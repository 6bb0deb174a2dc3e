#!/usr/bin/env python3
"""Launch shapes of the every-member fold from HBM (round 6 probe).

The library's every-member fold (combine_kernels.h combine_orders_vec) of
BASELINE config 4's float max runs at one vector per lane and 8 blocks per
CU (OrdersShape: min/max chains), measured in round 2 on buffers a power of
two apart; the double sum at 4 vectors per lane. With the round-5 buffer
stagger, bench.py's kernel legs put the float max at 8 x 8 MiB at 0.64 of
the HBM peak cold against 0.69-0.70 for the double sum at the same bytes.
This probe times the library's launch (mi355_combine_orders) and the shapes
of tools/libpeershapes.so (the same kernel template) on bench.py's layout
(buffers LEG_STAGGER bytes further apart than their size), warm (the same
buffers every launch) and cold (disjoint copies taken in turn, >= 2.25 GiB),
HIP event pair per launch, and checks every variant's outputs against the
library's. One JSON line per (kernel, size, shape).

run from the repo root on the GPU box: python3 tools/probes/orders_shapes_cold.py
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
    # SHAPES_LIB: another build of tools/peer_shapes.hip with its own shape list
    P = ctypes.CDLL(os.environ.get("SHAPES_LIB", os.path.join(ROOT, "tools", "libpeershapes.so")))
    for f in (P.peer_shapes_orders_float_max,):
        f.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.c_size_t, vp, vp, vp]
    P.peer_shapes_orders_double_sum.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                                ctypes.c_size_t, vp, vp, vp]
    L.mi355_time_next_launch.argtypes = [vp, vp]
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    reps = 40
    ev = [vp() for _ in range(2 * reps)]
    for e in ev:
        L.hipEventCreate(ctypes.byref(e))
    u, b = ctypes.c_int(), ctypes.c_int()
    # SHAPES_CASES: op:dtype:MiB,... (default: the three below)
    cases = [(c.split(":")[0], c.split(":")[1], int(c.split(":")[2]) << 20)
             for c in os.environ.get("SHAPES_CASES", "max:float:8,max:float:32,sum:double:8").split(",")]
    for op, dtype, nb in cases:
        es = 4 if dtype in ("float", "int") else 8
        n = nb // es
        span = nb + STAGGER
        set_bytes = 16 * span
        sets = max(2, -(-FOOT // set_bytes))
        pool = vp()
        assert L.hipMalloc(ctypes.byref(pool), ctypes.c_size_t(sets * set_bytes)) == 0
        base = pool.value
        x = np.random.default_rng(5).random(n * 8) - 0.5
        xs = x.astype(np.float32) if dtype == "float" else (x * 2**31).astype(np.int32) if dtype == "int" else x
        if op == "prod":
            xs = (1.0 + x * 1e-3).astype(xs.dtype)
        if dtype == "float" and os.environ.get("SHAPES_DATA") == "doublebytes":
            xs = x.view(np.float32)[:n * 8]   # bench.py's kernel legs: doubles' bytes read as floats (NaNs, zeros)
        for j in range(sets):
            for q in range(8):
                shm.put(base + j * set_bytes + q * span, xs[q * n:(q + 1) * n])

        def bufs(j):
            s = [base + j * set_bytes + q * span for q in range(8)]
            d = [base + j * set_bytes + (8 + q) * span for q in range(8)]
            return (vp * 8)(*d), (vp * 8)(*s), d, s

        def launcher(v):
            if v < 0:
                return lambda j, e0, e1: (L.mi355_time_next_launch(e0, e1) if e0 else None,
                                          shm.combine_orders(op, dtype, bufs(j)[2], bufs(j)[3], n))[1]
            if (op, dtype) == ("sum", "double"):
                return lambda j, e0, e1: P.peer_shapes_orders_double_sum(v, 8, bufs(j)[0], bufs(j)[1], n, e0, e1, None)
            f = getattr(P, f"peer_shapes_orders_{dtype}_{op}")
            f.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.c_size_t, vp, vp, vp]
            return lambda j, e0, e1: f(v, bufs(j)[0], bufs(j)[1], n, e0, e1, None)

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

        def outhash():
            h = hashlib.sha256()
            for d in bufs(0)[2]:
                h.update(shm.get(d, n, dtype).view(np.uint8))
            return h.hexdigest()

        alg = 16 * nb
        ref = None
        for v in [-1] + list(range(P.peer_shapes_count())):
            f = launcher(v)
            w, c = timed(f, False), timed(f, True)
            h = outhash()
            ref = ref or h
            if v >= 0:
                P.peer_shapes_describe(v, ctypes.byref(u), ctypes.byref(b))
                shape = f"{u.value} vectors/lane, {b.value} blocks/CU"
                if hasattr(P, "peer_shapes_pipe") and P.peer_shapes_pipe(v) == 1:
                    shape += ", pipelined"
            else:
                shape = "library"
            print(json.dumps({"kernel": f"combine_orders_vec<{op},{dtype},8>", "bytes_per_source": nb, "shape": shape,
                              "warm_us": round(w, 2), "warm_frac": round(alg / w / 1e3 / PEAK, 4),
                              "cold_us": round(c, 2), "cold_frac": round(alg / c / 1e3 / PEAK, 4), "sets": sets,
                              "same_outputs": h == ref}), flush=True)
        L.hipFree(pool)
    shm.finalize()


if __name__ == "__main__":
    main()
