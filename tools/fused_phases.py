#!/usr/bin/env python3
"""Where a fused call's time goes: the phase stamps of the probe build of the
fused kernel (csrc/Makefile `probe`: fused.hip with MI355_FUSED_PHASES), one
PE process of a job whose PEs share this GPU. Run with SHMEM_PE / SHMEM_NPES
/ SHMEM_JOB_ID / SHMEM_DEVICE and SHMEM_REDUCE_LIBDIR=<repo>/osss-gasnet_amd/lib/probe.

For each size: 200 back-to-back shmem_double_sum_to_all calls (C loop), then
the last 64 calls' stamps (100 MHz real-time counter) of THIS PE's kernel,
as medians in microseconds from the first block's start: last block start,
ARRIVE wait passed, folds done, RSDONE wait passed, gathers done, AGDONE
passed; and the host's per-call time. PE 0 prints one JSON line.

usage: fused_phases.py [sizes in bytes...]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "osss-gasnet_amd")]
import shmem_reduce  # noqa: E402

NAMES = ["last_block_start", "arrive_passed", "fold_done", "rsdone_passed", "gather_done", "agdone_passed"]


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [64 << 10, 256 << 10, 1 << 20]
    shm = shmem_reduce.Shmem()
    if not hasattr(shm.lib, "mi355_fused_phases"):
        raise SystemExit("not the probe build: set SHMEM_REDUCE_LIBDIR to osss-gasnet_amd/lib/probe")
    shm.init()
    me, npes = shm.my_pe(), shm.n_pes()
    maxb = max(sizes)
    src, dst = shm.malloc_device(maxb), shm.malloc_device(maxb)
    loop = shmem_reduce.bench_loop()
    ring = (ctypes.c_ulonglong * (64 * 8))()
    out = {}
    for nb in sizes:
        n = nb // 8
        shm.put(src, np.random.default_rng(me).random(n))
        loop(dst, src, n, 0, 0, npes, None, shm._psync_ptr, 20)
        shm.sync()
        shm.lib.mi355_fused_phases_reset()
        shm.barrier_all()
        t0 = time.perf_counter()
        loop(dst, src, n, 0, 0, npes, None, shm._psync_ptr, 200)
        shm.sync()
        t = (time.perf_counter() - t0) / 200
        info = shm.last_call_info()
        shm.lib.mi355_fused_phases(ring)
        r = np.frombuffer(ring, dtype=np.uint64).reshape(64, 8).astype(np.float64)
        ok = (r[:, 0] < 2**63) & (r[:, 6] > 0)
        rel = (r[ok, 1:7] - r[ok, :1]) / 100.0   # 100 MHz ticks -> us
        rel[rel < -1e6] = np.nan                    # phases a schedule does not have
        rec = {"us_per_call": round(t * 1e6, 2), "schedule": info["schedule"], "calls_stamped": int(ok.sum())}
        for i, name in enumerate(NAMES):
            col = rel[:, i]
            col = col[np.isfinite(col) & (col >= 0)]
            rec[name] = round(float(np.median(col)), 2) if len(col) else None
        per_pe = np.array([rec[k] if rec[k] is not None else -1.0 for k in NAMES] + [rec["us_per_call"]])
        allpe = np.zeros(len(per_pe) * npes)
        mine = np.zeros(len(per_pe) * npes)
        mine[me * len(per_pe):(me + 1) * len(per_pe)] = per_pe
        shm.to_all("sum", "double", allpe.ctypes.data, mine.ctypes.data, len(allpe), 0, 0, npes)
        out[str(nb)] = {"pe0": rec, "per_pe": allpe.reshape(npes, -1).round(2).tolist()}
        shm.barrier_all()
    if me == 0:
        print(json.dumps({"npes": npes, "columns": NAMES + ["us_per_call"], "legs": out}), flush=True)
    shm.finalize()


if __name__ == "__main__":
    main()
