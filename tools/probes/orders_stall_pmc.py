#!/usr/bin/env python3
"""Where the every-member fold's cold launches wait (round 6 probe, for PMC passes).

Launches the library's every-member fold (mi355_combine_orders) of config 4's
float max and, for comparison, the double sum, both at 8 sources x 8 MiB ->
8 outputs, cold: disjoint buffer sets (>= 2.25 GiB) taken in turn, on
bench.py's staggered layout (tools/probes/orders_shapes_cold.py); and, as
the reference point, the headline's 1-PE call (copy_segments, 256 MiB double
sum over 5 disjoint pairs, bench.py's headline_rotating). Prints the mean
HIP-event time per launch; run under `rocprofv3 --pmc ...
--kernel-include-regex 'combine_orders|copy_segments'` for the counters of
the same launches.

run from the repo root on the GPU box: python3 tools/probes/orders_stall_pmc.py
"""
import ctypes
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
    os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", "2600M")
    os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
    shm = shmem_reduce.Shmem()
    shm.init()
    L, vp = shm.lib, ctypes.c_void_p
    L.mi355_time_next_launch.argtypes = [vp, vp]
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    reps = int(os.environ.get("STALL_REPS", "40"))
    ev = [vp() for _ in range(2 * reps)]
    for e in ev:
        L.hipEventCreate(ctypes.byref(e))
    for op, dtype in (("max", "float"), ("sum", "double")):
        nb = 8 << 20
        es = 4 if dtype == "float" else 8
        n = nb // es
        span = nb + STAGGER
        set_bytes = 16 * span
        sets = max(2, -(-FOOT // set_bytes))
        pool = vp()
        assert L.hipMalloc(ctypes.byref(pool), ctypes.c_size_t(sets * set_bytes)) == 0
        base = pool.value
        x = np.random.default_rng(5).random(n * 8) - 0.5
        xs = x.astype(np.float32) if dtype == "float" else x
        for j in range(sets):
            for q in range(8):
                shm.put(base + j * set_bytes + q * span, xs[q * n:(q + 1) * n])
        srcs = [[base + j * set_bytes + q * span for q in range(8)] for j in range(sets)]
        dsts = [[base + j * set_bytes + (8 + q) * span for q in range(8)] for j in range(sets)]
        for j in range(sets):
            shm.combine_orders(op, dtype, dsts[j], srcs[j], n)
        shm.sync()
        for r in range(reps):
            j = r % sets
            L.mi355_time_next_launch(ev[2 * r], ev[2 * r + 1])
            shm.combine_orders(op, dtype, dsts[j], srcs[j], n)
        shm.sync()
        ts = []
        for r in range(reps):
            ms = ctypes.c_float()
            L.hipEventElapsedTime(ctypes.byref(ms), ev[2 * r], ev[2 * r + 1])
            ts.append(ms.value * 1e3)
        us = float(np.mean(ts))
        print(json.dumps({"kernel": f"combine_orders_vec<{op},{dtype},8>", "bytes_per_source": nb, "cold_us": round(us, 2),
                          "cold_frac": round(16 * nb / us / 1e3 / PEAK, 4), "sets": sets, "reps": reps}), flush=True)
        L.hipFree(pool)
    # the headline call, HBM-only: 5 disjoint 256 MiB pairs in turn
    nb = 256 << 20
    pairs = [(shm.malloc_device(nb), shm.malloc_device(nb)) for _ in range(5)]
    x = np.random.default_rng(6).random(nb // 8)
    for s_, _ in pairs:
        shm.put(s_, x)
    for j in range(5):
        shm.to_all("sum", "double", pairs[j][1], pairs[j][0], nb // 8)
    shm.sync()
    for r in range(reps):
        j = r % 5
        L.mi355_time_next_launch(ev[2 * r], ev[2 * r + 1])
        shm.to_all("sum", "double", pairs[j][1], pairs[j][0], nb // 8)
    shm.sync()
    ts = []
    for r in range(reps):
        ms = ctypes.c_float()
        L.hipEventElapsedTime(ctypes.byref(ms), ev[2 * r], ev[2 * r + 1])
        ts.append(ms.value * 1e3)
    us = float(np.mean(ts))
    assert np.array_equal(shm.get(pairs[0][1], nb // 8, "double"), x)
    print(json.dumps({"kernel": "copy_segments (1-PE double sum)", "bytes": nb, "cold_us": round(us, 2),
                      "cold_frac": round(2 * nb / us / 1e3 / PEAK, 4), "pairs": 5, "reps": reps}), flush=True)
    shm.finalize()


if __name__ == "__main__":
    main()
