#!/usr/bin/env python3
"""One PE of the fused-kernel measurement: bench.py's `fused_same_gpu` leg
(NPES processes with SHMEM_DEVICE=0, every PE on this GPU; also
tools/profile_fused.sh) and its N > 1 `small_call_persistent` leg (one
process per rank, each on the rank's GPU, SHMEM_PERSISTENT=1). Run with
SHMEM_PE / SHMEM_NPES / SHMEM_JOB_ID / SHMEM_DEVICE set.

For each message size, K back-to-back shmem_double_sum_to_all calls from a C
loop (csrc/bench_loop.c): per-call time (max over PEs), then the same K calls
with the fused kernel's own HIP event stamps (its average duration), and every
PE's result checked bit-exact against the oracle's result for that PE (the
reference's own-source-first order). PE 0 prints one JSON line.

usage: fused_bench.py [calls] [sizes in bytes...] [--config1]
(--config1: also BASELINE config 1's call, config1() below)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")]
import shmem_reduce  # noqa: E402


def synth(pe, n):
    return (np.random.default_rng(1000 + pe).random(n) - 0.5) * np.exp2(np.random.default_rng(pe).integers(0, 8, n))


def config1(shm, calls, max_over_pes):
    """BASELINE config 1's call through this library: shmem_int_sum_to_all on
    4 KiB (1,024 ints) over the active set {PE 0, PE 1} (PE_start 0,
    logPE_stride 0, PE_size 2; other PEs of the job only take part in the
    allocations and barriers), on shmem_malloc's symmetric host heap -- host
    memory, as the reference's heap is (symmem.c:212-236) -- and on the
    device heap. K back-to-back calls from the C loop (csrc/bench_loop.c),
    entry-to-return per call, max over the two PEs; every element checked
    bit-exact against the oracle's result for each PE."""
    import ctypes
    import oracle
    me = shm.my_pe()
    member = me < 2
    loop = shmem_reduce.bench_loop(name="int_sum")
    n = 1024
    out = {}
    for kind in ("host_heap", "device_heap"):
        alloc = shm.malloc if kind == "host_heap" else shm.malloc_device
        src, dst = alloc(n * 4), alloc(n * 4)
        if not src or not dst:
            raise RuntimeError("allocation for the config-1 leg failed")
        xs = [np.random.default_rng(4100 + p).integers(-2**31, 2**31, n).astype(np.int32) for p in range(2)]
        if member:
            if kind == "host_heap":
                ctypes.memmove(src, xs[me].ctypes.data, n * 4)
            else:
                shm.put(src, xs[me])
            loop(dst, src, n, 0, 0, 2, None, shm._psync_ptr, 20)
        shm.barrier_all()
        t0 = time.perf_counter()
        if member:
            loop(dst, src, n, 0, 0, 2, None, shm._psync_ptr, calls)
        t = time.perf_counter() - t0
        info = shm.last_call_info() if member else None
        bad = 0
        if member:
            if kind == "host_heap":
                got = np.empty(n, dtype=np.int32)
                ctypes.memmove(got.ctypes.data, dst, n * 4)
            else:
                got = shm.get(dst, n, "int")
            bad = int((got != oracle.reduce_pe("sum", "int", xs, me)).sum())
        t = max_over_pes(t if member else 0.0) / calls
        bad = int(max_over_pes(bad))
        sched = info["schedule"] if info else None
        out[kind] = {"us_per_call": round(t * 1e6, 2), "calls": calls, "schedule": sched,
                     "check": "bit-exact vs the reference's per-PE order, every element, both PEs" if bad == 0
                     else f"MISMATCH {bad} elements"}
        shm.barrier_all()
        if kind == "host_heap":
            shm.free(dst)
            shm.free(src)
        else:
            shm.free_device(dst)
            shm.free_device(src)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    calls = int(args[0]) if args else 4096
    sizes = [int(x) for x in args[1:]] or [64 << 10, 1 << 20]
    with_config1 = "--config1" in sys.argv
    os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str(8 << 20))
    os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
    os.environ.setdefault("SHMEM_DEVICE_ORDER_SIZE", "8M")
    shm = shmem_reduce.Shmem()
    shm.init()
    me, npes = shm.my_pe(), shm.n_pes()
    maxb = max(sizes)
    src, dst = shm.malloc_device(maxb), shm.malloc_device(maxb)
    loop = shmem_reduce.bench_loop()

    def max_over_pes(x):
        a, b = np.array([x], dtype=np.float64), np.zeros(1, dtype=np.float64)
        shm.to_all("max", "double", b.ctypes.data, a.ctypes.data, 1, 0, 0, npes)
        return float(b[0])

    out = {}
    import oracle
    shared = np.array([sum(shm.lib.shmemx_pe_same_device(q) for q in range(npes) if q != me)], dtype=np.int32)
    anyshared = np.zeros(1, dtype=np.int32)
    shm.to_all("max", "int", anyshared.ctypes.data, shared.ctypes.data, 1, 0, 0, npes)
    for nb in sizes:
        n = nb // 8
        x = synth(me, n)
        shm.put(src, x)
        loop(dst, src, n, 0, 0, npes, None, shm._psync_ptr, 20)
        shm.barrier_all()
        shm.sync()
        served0, launched0 = shm.persistent_stats()
        t0 = time.perf_counter()
        loop(dst, src, n, 0, 0, npes, None, shm._psync_ptr, calls)
        info = shm.last_call_info()  # before max_over_pes (a reduction of its own)
        shm.sync()
        t = max_over_pes(time.perf_counter() - t0) / calls
        served1, launched1 = shm.persistent_stats()
        shm.barrier_all()
        shm.kernel_timing(True)
        loop(dst, src, n, 0, 0, npes, None, shm._psync_ptr, calls)
        shm.sync()
        nk, _, kavg = shm.kernel_timing_stats()
        shm.kernel_timing(False)
        got = shm.get(dst, n, "double")
        want = oracle.reduce_pe("sum", "double", [synth(p, n) for p in range(npes)], me)
        bad = int(max_over_pes(int((got.view(np.uint64) != want.view(np.uint64)).sum())))
        kmax = max_over_pes(kavg)
        out[str(nb)] = {"bytes_per_pe": nb, "calls": calls, "us_per_call": round(t * 1e6, 2),
                        "kernel_avg_us": round(kmax * 1e3, 2), "kernels_timed": nk,
                        "schedule": info["schedule"], "kernel": info["kernel"],
                        "served": served1 - served0, "servers_launched": launched1 - launched0,
                        "check": f"bit-exact vs the reference's per-PE order on every PE, {n} elements each"
                        if bad == 0 else f"MISMATCH {bad} elements (worst PE)"}
        shm.barrier_all()
    shm.free_device(dst)
    shm.free_device(src)
    c1 = config1(shm, calls, max_over_pes) if with_config1 else None
    if me == 0:
        print(json.dumps({"npes": npes, "same_gpu": bool(anyshared[0]), "legs": out, "config1": c1}), flush=True)
    shm.finalize()


if __name__ == "__main__":
    main()
