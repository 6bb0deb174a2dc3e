#!/usr/bin/env python3
"""Benchmark: GiB/s reduced by shmem_double_sum_to_all, device-resident, 256 MiB per PE.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1
it runs under torch.distributed.run, one process (= one PE = one GPU) per
rank, identity from RANK/WORLD_SIZE/LOCAL_RANK. A step is one
shmem_double_sum_to_all call over the whole active set on 256 MiB per PE,
source and target in the device symmetric heap (inputs resident in HBM when
the timed region starts). K steps are bracketed by shmem_barrier_all + a
device synchronize on both sides; the time is the max over PEs.

value = N * 256 MiB / t_step / 2^30 (whole job); per-PE S/t_step is also
printed. roofline: the dominant kernel of the schedule the library actually
ran (shmemx_last_call_info: its name as rocprofv3 prints it, its sources,
outputs and bytes), its algorithmic bytes per launch / its average duration
from HIP events recorded by the library on its own stream.
cpu_baseline: the reference algorithm restated in C (oracle/liboracle.so) as
N PE processes (the headline's shape; 1 PE on 1 core at N = 1), one pinned
host core each, on a bounded sample, run by rank 0 before any rank's PE joins
the job (the other ranks wait in the bootstrap), at every N; vs_cpu_baseline
= value / cpu_baseline.value (vs_baseline stays null: BASELINE.md holds no
published number for this metric).
"""
import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

T_START = time.perf_counter()
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "osss-gasnet_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import shmem_reduce  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
XGMI_LINK_GBS = 153.0      # per link, 7 links per GPU (AMD's per-link figure)
XGMI_LINK_DIR_GBS = 76.8   # one direction of a link, if 153.6 counts both directions (as MI300X's 128 = 2 x 64)
GIB = float(1 << 30)
# headline_rotating: disjoint source/target pairs taken in turn; 5 x 2 x 256
# MiB = 2.5 GiB of footprint, ~10x the 256 MiB Infinity Cache
ROT_PAIRS = 5


def synth(pe, idx):
    """Deterministic full-mantissa doubles: value of element idx on PE pe
    (splitmix64 of (pe, idx)); random access, so any PE can recompute any
    other PE's samples for the correctness check."""
    z = (np.uint64(pe) << np.uint64(40)) + idx.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    mant = (z >> np.uint64(11)).astype(np.float64) * 2.0**-53          # [0,1) full 53 bits
    k = (z & np.uint64(7)).astype(np.float64)
    return (mant - 0.5) * np.exp2(k)


def synth_bits(pe, idx):
    """Deterministic 64-bit words whose bits are 1 with probability 7/8 (OR
    of three splitmix64 words), so an N-way AND is not all-zero (SURVEY 8d,
    config 4's longlong and)."""
    out = np.zeros(len(idx), dtype=np.uint64)
    for r in range(3):
        z = (np.uint64(pe + 1000 * (r + 1)) << np.uint64(40)) + idx.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        out = out | (z ^ (z >> np.uint64(31)))
    return out.view(np.int64)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(S, n_gpus, budget_s):
    """The reference algorithm (reduce-op.c:226-266 restated in C,
    oracle/reduce_oracle.c: copy loop, barrier, 64-element pWrk chunks folded
    with one indirect operator call per element, barrier) on this box's host
    cores, in this run, before the GPU is touched: forked PE processes, each
    pinned to a CPU of its own (the third allowed CPU on: CPU 0 takes most
    interrupts), shared-memory transport. Bounded sample: as many calls as fit
    in about budget_s. `value` has the headline's own shape: n_gpus PEs x S
    (at N = 1 one PE on one core). Sub-records: the other PE counts of SURVEY
    8d (2 and 8 PEs; 8 = BASELINE config 3's shape), the 1-PE call at N > 1,
    BASELINE config 1 (int sum, 2 PEs, 4 KiB) and config 5's call (64 KiB
    double sum at 8 PEs)."""
    import oracle
    n = S // 8

    def timed(op, dtype, pes, nel, share):
        t1, _ = oracle.cpu_baseline(op, dtype, pes, nel, 0, 1)
        reps = int(max(3, min(100000, share / max(t1, 1e-7))))
        t, cpus = oracle.cpu_baseline(op, dtype, pes, nel, 1, reps)
        return t, reps, cpus

    runs = {}   # PE count -> (t, reps, cpus)
    runs[n_gpus] = timed("sum", "double", n_gpus, n, 0.4 * budget_s)
    for pes, share in ((1, 0.15), (2, 0.15), (8, 0.15)):
        if pes not in runs:
            runs[pes] = timed("sum", "double", pes, n, share * budget_s)
    tc, repsc, cpusc = timed("sum", "int", 2, 1024, 0.05 * budget_s)
    t5, reps5, cpus5 = timed("sum", "double", 8, 8192, 0.1 * budget_s)
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = None
    mib = S >> 20
    t, reps, cpus = runs[n_gpus]

    def sub(pes, note):
        tp, rp, cp = runs[pes]
        return {"value": round(pes * S / tp / GIB, 4), "cores": pes, "calls": rp, "ms_per_call": round(tp * 1e3, 3),
                "per_pe_gib_s": round(S / tp / GIB, 4), "cpus": cp, "note": note}
    out = {"value": round(n_gpus * S / t / GIB, 4), "unit": "GiB/s", "cores": n_gpus, "kind": "port",
           "sample": f"{reps} calls of shmem_double_sum_to_all's reference algorithm (restated in C, "
                     f"oracle/reduce_oracle.c) on {n_gpus} PE process{'es' if n_gpus > 1 else ''} x {mib} MiB, "
                     f"one pinned core each (CPUs {cpus}); median per call {t * 1e3:.1f} ms, max over PEs; "
                     f"whole-job GiB/s, the headline's shape",
           "ms_per_call": round(t * 1e3, 3), "per_pe_gib_s": round(S / t / GIB, 4)}
    for pes, key in ((1, "one_pe"), (2, "two_pe"), (8, "eight_pe")):
        if pes != n_gpus:
            out[key] = sub(pes, f"{pes} PE{'s' if pes > 1 else ''} x {mib} MiB, whole-job GiB/s"
                           + (" (BASELINE config 3's shape on host cores)" if pes == 8 else ""))
    out.update({
        "config1": {"workload": "shmem_int_sum_to_all, 2 PEs, 4 KiB (BASELINE config 1; shared-memory "
                                "transport in place of GASNet udp/mpi loopback)",
                    "us_per_call": round(tc * 1e6, 3), "per_pe_gib_s": round(4096 / tc / GIB, 4), "calls": repsc,
                    "cores": 2, "cpus": cpusc},
        "config5": {"workload": "shmem_double_sum_to_all, 8 PEs, 64 KiB per call (BASELINE config 5's call)",
                    "us_per_call": round(t5 * 1e6, 3), "calls": reps5, "cores": 8, "cpus": cpus5},
        "host": {"nproc": os.cpu_count(), "allowed_cpus": allowed, "cpu_model": cpu_model()}})
    return out


def fused_same_gpu(npes, calls, persistent=False, config1=False):
    """The fused one-launch schedule (fused.hip), which every call up to 2 MiB
    per PE takes at N > 1, measured on this box's one GPU: `npes` PE processes
    of tools/fused_bench.py sharing it (started from this process before it
    touches the GPU). Per-call time for BASELINE config 5's 64 KiB calls
    (one-shot fold) and 1 MiB (reduce-scatter + all-gather in one launch), the
    fused kernel's own duration (HIP event stamps), and a bit-exact check of
    every PE's result. Same-GPU figures: the 'remote' reads are this GPU's HBM,
    not xGMI."""
    import subprocess
    import uuid
    env = dict(os.environ, SHMEM_NPES=str(npes), SHMEM_JOB_ID="fb" + uuid.uuid4().hex[:10], SHMEM_DEVICE="0",
               SHMEM_PERSISTENT="1" if persistent else "0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    script = os.path.join(ROOT, "tools", "fused_bench.py")
    procs = [subprocess.Popen([sys.executable, script, str(calls)] + (["--config1"] if config1 else []),
                              env=dict(env, SHMEM_PE=str(pe)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for pe in range(npes)]
    outs = []
    for p in procs:
        r = wait_child(p, "fused_same_gpu")
        if r is None:
            for q in procs:
                q.kill()
                q.communicate()
            return {"error": "timed out after 150 s"}
        outs.append(r)
    if any(p.returncode != 0 for p in procs):
        return {"error": "; ".join(f"PE {i} rc {p.returncode}: {o[1][-300:]}" for i, (p, o) in enumerate(zip(procs, outs))
                                   if p.returncode != 0)}
    lines = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    if not lines:
        return {"error": "no result line from PE 0"}
    d = json.loads(lines[-1])
    d["note"] = ("fused_allreduce (one launch per call: device-side arrival/done flags) with the PEs sharing this one "
                 "GPU; us_per_call is entry-to-return, max over PEs; kernel_avg_us the fused kernel's duration")
    if persistent:
        d["note"] = ("the same calls with SHMEM_PERSISTENT=1: after the first two, each call is served by the fused "
                     "kernel left resident (mi355_fused_server, fed through a host-coherent mailbox), no launch; "
                     "kernel_avg_us covers only the launched calls")
    return d


def traffic_for(rec, key, host):
    """HBM bytes per launch from the PMC passes committed in
    profiles/pmc_traffic.json (tools/pmc_traffic.py: FETCH_SIZE x 2 +
    WRITE_SIZE, gfx950 correction), put into rec["traffic"] only when the
    entry was profiled from this library's machine code (hash of its gfx950
    code objects, shmem_reduce.kernel_code_hash); otherwise traffic stays null
    and the returned note says why."""
    if host:
        return "host-staged run: no PMC profile"
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        tr = json.load(open(path)).get(key)
    except (OSError, ValueError):
        tr = None
    if not tr:
        return f"no PMC profile for {key} in profiles/pmc_traffic.json"
    want = shmem_reduce.kernel_code_hash()
    if tr.get("kernel_code_sha") != want:
        return (f"profiles/pmc_traffic.json[{key}] was taken from kernel code {tr.get('kernel_code_sha')}, this "
                f"library's is {want}: not reported")
    rec["traffic"] = tr["hbm_bytes_per_launch"]
    rec["traffic_source"] = tr["source"]
    return f"PMC passes of this library's kernels (gfx950 code objects {want})"


def wait_child(p, name, limit=150):
    """communicate() with a child job, printing a heartbeat to stderr every
    30 s (a silent wait reads as a hang to a watchdog) and giving up after
    `limit` s. Returns (out, err) or None on the time limit (child killed)."""
    import subprocess
    t0 = time.perf_counter()
    while True:
        try:
            return p.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            waited = time.perf_counter() - t0
            if waited >= limit:
                p.kill()
                p.communicate()
                return None
            print(f"[bench rank {os.environ.get('RANK', '0')}] {name}: child job running, {waited:.0f} s",
                  file=sys.stderr, flush=True)


def persistent_child(rank, world, calls):
    """N > 1: BASELINE config 5's 64 KiB calls with the opt-in persistent
    server (SHMEM_PERSISTENT=1), run by one child PE process per rank on the
    rank's own GPU -- a job of its own (tools/fused_bench.py), started before
    this process touches the GPU -- so that the opt-in path, never run across
    GPUs before the driver's 8-GPU node, cannot take the headline line with
    it: a failure or a hang there becomes an "error" entry. Rank 0's child
    prints the record (per-call time max over PEs, bit-exact check of every
    PE's result, calls served vs servers launched)."""
    import subprocess
    job = "ps%s-%d" % (os.environ.get("MASTER_PORT", "0"), os.getppid())
    env = dict(os.environ, SHMEM_PE=str(rank), SHMEM_NPES=str(world), SHMEM_JOB_ID=job,
               SHMEM_DEVICE=os.environ.get("LOCAL_RANK", str(rank)), SHMEM_PERSISTENT="1",
               SHMEM_BARRIER_TIMEOUT="60")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    script = os.path.join(ROOT, "tools", "fused_bench.py")
    p = subprocess.Popen([sys.executable, script, str(calls), str(64 << 10)], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    r = wait_child(p, "small_call_persistent")
    if r is None:
        return {"error": "timed out after 150 s"}
    out, err = r
    if p.returncode != 0:
        return {"error": f"PE {rank} rc {p.returncode}: {err[-400:]}"}
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    if rank != 0:
        return None
    if not lines:
        return {"error": "no result line from PE 0"}
    d = json.loads(lines[-1])
    leg = d["legs"].get(str(64 << 10), {})
    leg.update({"opt_in": True, "same_gpu": d.get("same_gpu"), "npes": d.get("npes"),
                "note": "opt-in persistent server (SHMEM_PERSISTENT=1, shmemx_set_persistent): after the first two "
                        "calls a resident fused kernel takes each call from a host-coherent mailbox, no launch; "
                        "measured in a child job of one PE per GPU (tools/fused_bench.py), kernel_avg_us covers "
                        "only the launched calls"})
    return leg


def extra_legs_child(rank, world, mib, steps, algorithm, flags):
    """N > 1: external_buffers, link_probe, collectives and (round 6) the
    one-GPU-per-PE legs xgmi_ceiling and peer_fold_shapes (xgmi_legs), run by
    one child PE process per rank on the rank's own GPU (tools/extra_legs.py),
    started before this process touches the GPU, like persistent_child: none
    of them had run with one GPU per PE before the driver's 8-GPU node, and a
    fatal error in one (the library aborts the PE) or a hang would otherwise
    end this rank before the headline line is printed. Returns rank 0's
    records, or {"error": ...} under each leg's name."""
    import subprocess
    names = [k for k, f in (("external_buffers", "--no-external"), ("link_probe", "--no-link-probe"),
                            ("collectives", "--no-collectives"), ("xgmi_ceiling", "--no-xgmi-legs"),
                            ("peer_fold_shapes", "--no-xgmi-legs"), ("config1_call", "--no-config1")) if f not in flags]
    if not names:
        return {}
    job = "xl%s-%d" % (os.environ.get("MASTER_PORT", "0"), os.getppid())
    env = dict(os.environ, SHMEM_PE=str(rank), SHMEM_NPES=str(world), SHMEM_JOB_ID=job,
               SHMEM_DEVICE=os.environ.get("LOCAL_RANK", str(rank)), SHMEM_BARRIER_TIMEOUT="60")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "SHMEM_DEVICE_HEAP_SIZE", "SHMEM_DEVICE_SCRATCH_SIZE"):
        env.pop(k, None)
    script = os.path.join(ROOT, "tools", "extra_legs.py")
    p = subprocess.Popen([sys.executable, script, str(mib), str(steps), algorithm, *flags], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)

    def failed(msg):
        return {k: {"error": msg} for k in names}
    r = wait_child(p, "extra_legs_child")
    if r is None:
        return failed("child job timed out after 150 s")
    out, err = r
    if p.returncode != 0:
        return failed(f"child job: PE {rank} rc {p.returncode}: {err[-400:]}")
    if rank != 0:
        return {}
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    if not lines:
        return failed("child job: no result line from PE 0")
    return json.loads(lines[-1])


def host_staged_leg(shm, loop, S, me, npes, k, check):
    """north_star's second rate: the symmetric-heap buffers in HOST memory, as
    the reference's heap is (symmem.c:212-236, comms-inline.h:797-807):
    shmem_malloc's page-locked arrays, K blocking calls that each stage the
    source in over PCIe, reduce and stage the result out (the library's
    chunked copy-in / reduce / copy-out pipeline on two streams, or the fused
    kernel's in-kernel staging for small messages). Beside it, the same run's
    PCIe ceiling: hipMemcpyAsync of S bytes H2D alone, D2H alone, and both at
    once on two streams; a staged call moves S each way, so its ceiling is the
    two-way rate and pcie_frac = (S / t) / both_GB_s_each_direction. The result
    is checked bit-exact against the oracle on a sample."""
    import ctypes
    L, vp = shm.lib, ctypes.c_void_p
    n = S // 8
    hsrc, hdst = shm.malloc(S), shm.malloc(S)
    if not hsrc or not hdst:
        raise RuntimeError("shmem_malloc of 2 x %d bytes failed" % S)
    x = synth(me, np.arange(n, dtype=np.uint64))
    ctypes.memmove(hsrc, x.ctypes.data, S)
    del x
    loop(hdst, hsrc, n, 0, 0, npes, None, shm._psync_ptr, 2)
    shm.barrier_all()
    shm.sync()
    t0 = time.perf_counter()
    loop(hdst, hsrc, n, 0, 0, npes, None, shm._psync_ptr, k)
    shm.sync()
    t = (time.perf_counter() - t0) / k
    info = shm.last_call_info()
    ck = "skipped"
    if check:
        import oracle
        idx = np.unique(np.random.default_rng(300 + me).integers(0, n, 1 << 16)).astype(np.uint64)
        got = np.ctypeslib.as_array(ctypes.cast(hdst, ctypes.POINTER(ctypes.c_double)), shape=(n,))[idx.astype(np.int64)]
        want = oracle.reduce_pe("sum", "double", [synth(p, idx) for p in range(npes)], me)
        bad = int((got.view(np.uint64) != want.view(np.uint64)).sum())
        ck = "bit-exact vs the reference's per-PE order, %d samples" % len(idx) if bad == 0 else \
            "MISMATCH %d of %d samples" % (bad, len(idx))
    # the PCIe ceiling, same run, same page-locked arrays
    L.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    L.hipStreamSynchronize.argtypes = [vp]
    L.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
    L.hipStreamDestroy.argtypes = [vp]
    dev = [vp(), vp()]
    st = [vp(), vp()]
    for d in dev:
        if L.hipMalloc(ctypes.byref(d), ctypes.c_size_t(S)) != 0:
            raise RuntimeError("hipMalloc failed")
    for s in st:
        L.hipStreamCreate(ctypes.byref(s))
    h2d = lambda: L.hipMemcpyAsync(dev[0], vp(hsrc), S, 1, st[0])  # noqa: E731
    d2h = lambda: L.hipMemcpyAsync(vp(hdst), dev[1], S, 2, st[1])  # noqa: E731

    def rate(fns, reps=5):
        for f in fns:
            f()
        for s in st:
            L.hipStreamSynchronize(s)
        tq = time.perf_counter()
        for _ in range(reps):
            for f in fns:
                f()
        for s in st:
            L.hipStreamSynchronize(s)
        return S * reps / (time.perf_counter() - tq) / 1e9

    pcie = {"h2d_GB_s": round(rate([h2d]), 1), "d2h_GB_s": round(rate([d2h]), 1),
            "both_GB_s_each_direction": round(rate([h2d, d2h]), 1)}
    for s in st:
        L.hipStreamDestroy(s)
    for d in dev:
        L.hipFree(d)
    shm.free(hdst)
    shm.free(hsrc)
    gbs = S / t / 1e9
    # the same bytes with copy-in and copy-out one after the other: a staged
    # call at or above this did not overlap its two PCIe directions
    serial_ms = (S / (pcie["h2d_GB_s"] * 1e9) + S / (pcie["d2h_GB_s"] * 1e9)) * 1e3
    return {"bytes_per_pe": S, "calls": k, "ms_per_call": round(t * 1e3, 3), "value": round(npes * S / t / GIB, 2),
            "unit": "GiB/s", "GB_s_per_pe": round(gbs, 1), "schedule": info["schedule"], "pcie": pcie,
            "serial_copies_ms": round(serial_ms, 3), "overlap": round(serial_ms / (t * 1e3), 3),
            "pcie_frac": round(gbs / pcie["both_GB_s_each_direction"], 4), "check": ck,
            "note": "source and target in shmem_malloc's page-locked host arrays (the reference's heap is host "
                    "memory): each call stages S in over PCIe, reduces and stages S out; the headline value is "
                    "device-resident. pcie_frac = per-PE S / t against the same run's two-way hipMemcpyAsync rate"}


def rotating_leg(shm, S, me, npes, src, dst, k, check):
    """N = 1: the headline's call, shmem_double_sum_to_all on S bytes, over
    ROT_PAIRS disjoint (source, target) pairs of the device heap taken in turn
    (csrc/bench_loop.c shmemb_double_sum_rotating): between two uses of a line
    (ROT_PAIRS - 1) x 2 S of other traffic goes by, 4x the Infinity Cache, so
    every call's bytes come from HBM (MI355X_MICROARCH.md: a line stays
    resident only while the traffic between two uses of it fits in ~256 MiB).
    The headline loop re-reads ONE pair, whose 512 MiB partly stay on-die: this
    leg is its HBM-only figure. Timed like the headline (C loop, barrier +
    device synchronize on both sides), then again with HIP events on every
    dominant launch; every pair's target checked bit-exact on a sample."""
    n = S // 8
    srcs, dsts = [src], [dst]
    x = synth(me, np.arange(n, dtype=np.uint64))
    try:
        for _ in range(ROT_PAIRS - 1):
            a, b = shm.malloc_device(S), shm.malloc_device(S)
            srcs += [a] if a else []
            dsts += [b] if b else []
            if not a or not b:
                raise RuntimeError("the device heap has no room for %d more %d-byte pairs (SHMEM_DEVICE_HEAP_SIZE)"
                                   % (ROT_PAIRS - 1, S))
            shm.put(a, x)
        run = shmem_reduce.bench_rotating()
        k = max(k, 4 * ROT_PAIRS)
        run(dsts, srcs, n, 0, 0, npes, shm._psync_ptr, 2 * ROT_PAIRS)
        shm.barrier_all()
        shm.sync()
        t0 = time.perf_counter()
        run(dsts, srcs, n, 0, 0, npes, shm._psync_ptr, k)
        shm.sync()
        t = (time.perf_counter() - t0) / k
        shm.barrier_all()
        shm.kernel_timing(True)
        run(dsts, srcs, n, 0, 0, npes, shm._psync_ptr, k)
        shm.sync()
        nk, _, k_avg_ms = shm.kernel_timing_stats()
        shm.kernel_timing(False)
        info = shm.last_call_info()
        ck = "skipped"
        if check:
            import oracle
            idx = np.unique(np.random.default_rng(400 + me).integers(0, n, 1 << 14)).astype(np.uint64)
            want = oracle.reduce_pe("sum", "double", [synth(p, idx) for p in range(npes)], me)
            bad = 0
            for d in dsts:
                got = shm.get(d, n, "double")[idx.astype(np.int64)]
                bad += int((got.view(np.uint64) != want.view(np.uint64)).sum())
            ck = (f"bit-exact vs the reference, {len(idx)} samples x {len(dsts)} targets" if bad == 0
                  else f"MISMATCH in {bad} samples")
    finally:
        for d in srcs[1:] + dsts[1:]:
            shm.free_device(d)
    alg = info["alg_bytes"] // max(1, info["launches"])
    kt = k_avg_ms * 1e-3
    achieved = alg / kt / 1e9 if kt > 0 else 0.0
    return {"value": round(npes * S / t / GIB, 2), "unit": "GiB/s", "ms_per_step": round(t * 1e3, 4), "steps": k,
            "pairs": ROT_PAIRS, "footprint_MiB": ROT_PAIRS * 2 * S >> 20, "schedule": info["schedule"],
            "kernel": info["kernel"], "kernel_avg_us": round(k_avg_ms * 1e3, 2), "launches_timed": nk,
            "alg_bytes_per_launch": alg, "achieved_GB_s": round(achieved, 1),
            "frac": round(achieved / HBM_PEAK_GBS, 4), "check": ck,
            "note": "the headline call over %d disjoint 256 MiB source/target pairs taken in turn (%d MiB "
                    "footprint): every call streams from HBM; the headline re-reads one pair, part of which "
                    "the 256 MiB Infinity Cache serves" % (ROT_PAIRS, ROT_PAIRS * 2 * S >> 20)}


def offset_target_leg(shm, S, me, npes, src, k, check):
    """N = 1: the headline call with the target one element off the source's
    16-byte phase (target = &t[1], source = &s[0], nreduce - 1 elements), a
    caller's offset into an array: the target is peeled to 16 bytes and the
    source read with unaligned 16-byte loads (copy_segments_shift; before
    round 5 an 8-byte-word copy at 0.24 of peak). Timed like the headline."""
    n = S // 8 - 1
    loop = shmem_reduce.bench_loop()
    own = shm.malloc_device(S)   # its own target: the headline's stays as the headline left it
    if not own:
        raise RuntimeError("the device heap has no room for a %d-byte target" % S)
    tgt = own + 8
    try:
        loop(tgt, src, n, 0, 0, npes, None, shm._psync_ptr, 3)
        shm.barrier_all()
        shm.sync()
        t0 = time.perf_counter()
        loop(tgt, src, n, 0, 0, npes, None, shm._psync_ptr, k)
        shm.sync()
        t = (time.perf_counter() - t0) / k
        shm.kernel_timing(True)
        loop(tgt, src, n, 0, 0, npes, None, shm._psync_ptr, k)
        shm.sync()
        nk, _, k_avg_ms = shm.kernel_timing_stats()
        shm.kernel_timing(False)
        info = shm.last_call_info()
        ck = "skipped"
        if check:
            import oracle
            idx = np.unique(np.random.default_rng(600 + me).integers(0, n, 1 << 14)).astype(np.uint64)
            want = oracle.reduce_pe("sum", "double", [synth(p, idx) for p in range(npes)], me)
            got = shm.get(tgt, n, "double")[idx.astype(np.int64)]
            bad = int((got.view(np.uint64) != want.view(np.uint64)).sum())
            ck = f"bit-exact vs the reference, {len(idx)} samples" if bad == 0 else f"MISMATCH in {bad} samples"
    finally:
        shm.free_device(own)
    alg = info["alg_bytes"] // max(1, info["launches"])
    kt = k_avg_ms * 1e-3
    achieved = alg / kt / 1e9 if kt > 0 else 0.0
    rec = {"value": round(npes * n * 8 / t / GIB, 2), "unit": "GiB/s", "ms_per_step": round(t * 1e3, 4), "steps": k,
           "target_offset_bytes": 8, "schedule": info["schedule"], "kernel": info["kernel"],
           "kernel_avg_us": round(k_avg_ms * 1e3, 2), "launches_timed": nk, "alg_bytes_per_launch": alg,
           "achieved_GB_s": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
           "check": ck}
    # unaligned 16-byte loads span two lines: PMC bytes show whether the
    # line one wave shares with the next is fetched twice
    rec["traffic_note"] = traffic_for(rec, "offset_target_copy_shift", False)
    if rec.get("traffic"):
        rec["traffic_over_alg"] = round(rec["traffic"] / alg, 4)
    return rec


def full_check(shm, dst, n, op, dtype, gen, npes, me, host=False, chunk=1 << 22):
    """Every element of this PE's target against the oracle's result for this
    PE (oracle.reduce_pe(..., me): the reference's fold order for member me,
    reduce-op.c:226-264) on the sources regenerated from their generator, in
    chunks; SHA-256 of the target and of the expected array over the same
    bytes. Returns (mismatched elements, target sha256 hex, expected sha256
    hex). Run after the timed regions."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    import oracle
    es = np.dtype(shmem_reduce.NP[dtype]).itemsize
    hg, hw = hashlib.sha256(), hashlib.sha256()
    bad = 0
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))
    threads = max(1, min(8, npes, (os.cpu_count() or 8) // local))
    with ThreadPoolExecutor(threads) as ex:
        for b in range(0, n, chunk):
            m = min(chunk, n - b)
            idx = np.arange(b, b + m, dtype=np.uint64)
            srcs = list(ex.map(lambda p: gen(p, idx), range(npes)))
            want = oracle.reduce_pe(op, dtype, srcs, me)
            if host:
                import ctypes
                got = np.empty(m, dtype=want.dtype)
                ctypes.memmove(got.ctypes.data, dst + b * es, m * es)
            else:
                got = shm.get(dst + b * es, m, dtype)
            gb, wb = got.view(np.uint8), want.view(np.uint8)
            hg.update(gb)
            hw.update(wb)
            bad += int((gb != wb).reshape(m, es).any(axis=1).sum())
    return bad, hg.hexdigest(), hw.hexdigest()


def full_check_record(shm, npes, me, bad, hg, hw, max_over_pes):
    """Job-wide verdict of full_check: mismatches summed over PEs (each PE's
    own count, max-reduced so that every PE learns the worst), and whether
    every PE's target hashed to its expected array's SHA-256."""
    worst = int(max_over_pes(bad))
    hash_bad = int(max_over_pes(0 if hg == hw else 1))
    ok = worst == 0 and hash_bad == 0
    return ("bit-exact, every element, every PE (SHA-256 of each PE's target = that of the oracle's result for "
            "that PE)" if ok else "MISMATCH: %d elements on the worst PE, %s" %
            (worst, "hashes differ" if hash_bad else "hashes equal")), hg[:16]


def xgmi_ceiling_leg(shm, S, me, npes, src, buf, reps=20):
    """N > 1, one GPU per PE: what this GPU can pull from all N-1 peers at
    once -- the all-gather leg's exact pattern (reduce.c gather_segments:
    every PE copies shard q of peer q's array into its own buffer, all PEs
    together), measured two ways on the same peer mappings
    (shmemx_peer_device_ptr): the library's copy kernel (mi355_copy_segments,
    one launch of N-1 segments, HIP event pair per launch) and the copy
    engines (hipMemcpyAsync device-to-device from each peer's mapping, one
    stream per peer, wall clock). GB/s into this GPU = (N-1) shard bytes /
    time; each figure the minimum over PEs (the slowest GPU's ingress). This
    is the measured ceiling the N > 1 roofline's link constants stand beside."""
    import ctypes
    L, vp = shm.lib, ctypes.c_void_p
    shard = (S // npes) // 256 * 256
    peers = [q for q in range(npes) if q != me]
    psrc = [shm.peer_device_ptr(src, q) for q in peers]
    if any(not p for p in psrc):
        raise RuntimeError("a peer's device heap is not mapped here")
    dsts = (vp * len(peers))(*[buf + q * shard for q in peers])
    sps = (vp * len(peers))(*[p + q * shard for p, q in zip(psrc, peers)])
    nbs = (ctypes.c_size_t * len(peers))(*[shard] * len(peers))
    L.mi355_time_next_launch.argtypes = [vp, vp]
    L.mi355_time_next_launch.restype = None
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    ev = [vp() for _ in range(2 * reps)]
    for e in ev:
        L.hipEventCreate(ctypes.byref(e))
    if L.mi355_copy_segments(dsts, sps, nbs, len(peers), None) != 0:
        raise RuntimeError("mi355_copy_segments failed")
    shm.sync()
    shm.barrier_all()
    t0 = time.perf_counter()
    for r in range(reps):
        L.mi355_time_next_launch(ev[2 * r], ev[2 * r + 1])
        if L.mi355_copy_segments(dsts, sps, nbs, len(peers), None) != 0:
            raise RuntimeError("mi355_copy_segments failed")
    shm.sync()
    t_wall_k = (time.perf_counter() - t0) / reps
    ts = []
    for r in range(reps):
        ms = ctypes.c_float()
        L.hipEventElapsedTime(ctypes.byref(ms), ev[2 * r], ev[2 * r + 1])
        ts.append(ms.value * 1e-3)
    for e in ev:
        L.hipEventDestroy(e)
    t_k = float(np.mean(ts))
    # the copy engines: one stream per peer, all at once
    L.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    L.hipStreamSynchronize.argtypes = [vp]
    L.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
    L.hipStreamDestroy.argtypes = [vp]
    st = [vp() for _ in peers]
    for x in st:
        L.hipStreamCreate(ctypes.byref(x))

    def sdma_round():
        for i in range(len(peers)):
            if L.hipMemcpyAsync(vp(dsts[i]), vp(sps[i]), shard, 3, st[i]) != 0:
                raise RuntimeError("hipMemcpyAsync from a peer mapping failed")
    sdma_round()
    for x in st:
        L.hipStreamSynchronize(x)
    shm.barrier_all()
    t0 = time.perf_counter()
    for _ in range(reps):
        sdma_round()
    for x in st:
        L.hipStreamSynchronize(x)
    t_s = (time.perf_counter() - t0) / reps
    for x in st:
        L.hipStreamDestroy(x)
    # every segment landed (the last copy engine round): spot-check against the source's generator
    idx = np.arange(0, shard // 8, max(1, shard // 8 // 4096), dtype=np.uint64)
    bad = 0
    for q in peers:
        got = shm.get(buf + q * shard + 0, shard // 8, "double")[idx.astype(np.int64)]
        want = synth(q, idx + np.uint64(q * shard // 8))
        bad += int((got.view(np.uint64) != want.view(np.uint64)).sum())
    ingress = (npes - 1) * shard
    return {"bytes_into_each_pe": ingress, "shard_bytes": shard, "reps": reps,
            "kernel": "mi355_copy_segments (%d segments, one launch)" % len(peers),
            "kernel_avg_us": t_k * 1e6, "kernel_wall_us": t_wall_k * 1e6,
            "kernel_GB_s": ingress / t_k / 1e9, "sdma_us": t_s * 1e6, "sdma_GB_s": ingress / t_s / 1e9,
            "bad": bad}


def peer_fold_shapes_leg(shm, S, me, npes, src, out, reps=10):
    """N = 4 or 8, one GPU per PE: the every-member fold of config 3's shard
    (N sources of S/N bytes, N-1 of them on peers) at the library's launch
    shape (mi355_combine_orders) and at the other shapes of
    tools/libpeershapes.so (the same kernel template, other vectors per lane /
    blocks per CU), all PEs at once, HIP event pair per launch; every
    variant's N outputs compared byte for byte with the library's. The
    library's shape was tuned with every source in local HBM; this says
    whether xGMI's latency wants another one."""
    import ctypes
    import hashlib
    L, vp = shm.lib, ctypes.c_void_p
    P = ctypes.CDLL(os.path.join(ROOT, "tools", "libpeershapes.so"))
    P.peer_shapes_orders_double_sum.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                                ctypes.c_size_t, vp, vp, vp]
    L.mi355_time_next_launch.argtypes = [vp, vp]
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    lo, hi = shmem_reduce.shard_bounds(L, S // 8, 8, npes, me)
    n = (hi - lo) // 2 * 2
    shard_b = n * 8
    slot = (shard_b + 255) // 256 * 256 + 256 + 4096   # the library's version-slot spacing (reduce.c ver_slot_bytes)
    srcs = [(shm.peer_device_ptr(src, q) or 0) + lo * 8 for q in range(npes)]
    if any(s == lo * 8 for s in srcs):
        raise RuntimeError("a peer's device heap is not mapped here")
    outs = [out + q * slot for q in range(npes)]
    D = (vp * npes)(*outs)
    Sx = (vp * npes)(*srcs)
    ev = [vp() for _ in range(2 * reps)]
    for e in ev:
        L.hipEventCreate(ctypes.byref(e))

    def timed(launch):
        assert launch(None, None) == 0
        shm.sync()
        shm.barrier_all()
        for r in range(reps):
            assert launch(ev[2 * r], ev[2 * r + 1]) == 0
        shm.sync()
        ts = []
        for r in range(reps):
            ms = ctypes.c_float()
            L.hipEventElapsedTime(ctypes.byref(ms), ev[2 * r], ev[2 * r + 1])
            ts.append(ms.value * 1e-3)
        h = hashlib.sha256()
        for o in outs:
            h.update(shm.get(o, n, "double").view(np.uint8))
        return float(np.mean(ts)), h.hexdigest()

    def lib_launch(e0, e1):
        if e0 is not None:
            L.mi355_time_next_launch(e0, e1)
        return shm.combine_orders("sum", "double", outs, srcs, n)

    t_lib, h_lib = timed(lib_launch)
    alg = 2 * npes * shard_b
    remote = (npes - 1) * shard_b
    rows = [{"shape": "library (mi355_combine_orders)", "kernel_avg_us": round(t_lib * 1e6, 2),
             "remote_read_GB_s": round(remote / t_lib / 1e9, 1), "hbm_frac": round(alg / t_lib / 1e9 / HBM_PEAK_GBS, 4),
             "same_outputs": True}]
    u, b = ctypes.c_int(), ctypes.c_int()
    for v in range(P.peer_shapes_count()):
        P.peer_shapes_describe(v, ctypes.byref(u), ctypes.byref(b))
        t, h = timed(lambda e0, e1, v=v: P.peer_shapes_orders_double_sum(v, npes, D, Sx, n, e0, e1, None))
        rows.append({"shape": f"{u.value} vectors/lane, {b.value} blocks/CU", "kernel_avg_us": round(t * 1e6, 2),
                     "remote_read_GB_s": round(remote / t / 1e9, 1), "hbm_frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
                     "same_outputs": h == h_lib})
    for e in ev:
        L.hipEventDestroy(e)
    return {"kernel": "combine_orders_vec<sum,double,%d>" % npes, "sources": npes, "peer_sources": npes - 1,
            "bytes_per_source": shard_b, "reps": reps, "rows": rows}


def xgmi_legs(shm, S, me, npes, src, dst, force, max_over_pes):
    """N > 1: xgmi_ceiling_leg and (N = 4 or 8) peer_fold_shapes_leg on this
    job's buffers (src holds synth(me, ...), dst and S + N x 8 KiB more of
    device heap are free), their figures reduced over the PEs (slowest PE).
    PEs sharing a GPU: not applicable, unless `force` (a rehearsal of the code
    path, marked so, feeding no roofline). Run by tools/extra_legs.py, bench's
    child job. Returns {"xgmi_ceiling": ..., "peer_fold_shapes": ...}."""
    shared = np.array([sum(shm.lib.shmemx_pe_same_device(q) for q in range(npes) if q != me)], dtype=np.int32)
    shared_gpu = int(max_over_pes(float(shared[0]))) != 0
    na = {"not_applicable": "the PEs share a GPU: peer reads are this GPU's own HBM, no link is involved"}
    if shared_gpu and not force:
        return {"xgmi_ceiling": dict(na), "peer_fold_shapes": dict(na)}
    xc = xgmi_ceiling_leg(shm, S, me, npes, src, dst)
    xgmi_ceiling = {k: v for k, v in xc.items() if k not in ("kernel_avg_us", "kernel_GB_s", "sdma_us", "sdma_GB_s",
                                                             "bad", "kernel_wall_us")}
    slow_k = max_over_pes(xc["kernel_avg_us"])
    slow_s = max_over_pes(xc["sdma_us"])
    xgmi_ceiling.update({
        "kernel_avg_us": round(slow_k, 2), "kernel_GB_s_into_each_pe": round(xc["bytes_into_each_pe"] / slow_k / 1e3, 1),
        "sdma_us": round(slow_s, 2), "sdma_GB_s_into_each_pe": round(xc["bytes_into_each_pe"] / slow_s / 1e3, 1),
        "check": "bit-exact (sampled, every peer's segment)" if int(max_over_pes(xc["bad"])) == 0 else "MISMATCH",
        "note": "every PE pulls shard q of peer q's array from all N-1 peers at once (the all-gather's pattern) "
                "through the peer mappings: the library's copy kernel and the copy engines; GB/s into each GPU, "
                "slowest PE; measured in bench.py's child job (tools/extra_legs.py)"})
    xgmi_ceiling["peak_measured_GB_s"] = max(xgmi_ceiling["kernel_GB_s_into_each_pe"],
                                             xgmi_ceiling["sdma_GB_s_into_each_pe"])
    if shared_gpu:   # a rehearsal: local HBM copies, not a link ceiling
        xgmi_ceiling["rehearsal_same_gpu"] = xgmi_ceiling.pop("peak_measured_GB_s")
    if npes not in (4, 8):
        return {"xgmi_ceiling": xgmi_ceiling,
                "peer_fold_shapes": {"not_applicable": "the shape variants are 4- and 8-source folds (N = %d)" % npes}}
    out_buf = shm.malloc_device(S + npes * 8192)
    if not out_buf:
        raise RuntimeError("no room in the device heap for the peer fold's outputs")
    try:
        ps = peer_fold_shapes_leg(shm, S, me, npes, src, out_buf)
    finally:
        shm.free_device(out_buf)
    for r in ps["rows"]:
        r["kernel_avg_us"] = round(max_over_pes(r["kernel_avg_us"]), 2)
        r["remote_read_GB_s"] = round(ps["bytes_per_source"] * (npes - 1) / r["kernel_avg_us"] / 1e3, 1)
        r["hbm_frac"] = round(2 * npes * ps["bytes_per_source"] / r["kernel_avg_us"] / 1e3 / HBM_PEAK_GBS, 4)
        r["same_outputs"] = int(max_over_pes(0 if r["same_outputs"] else 1)) == 0
    ps["fastest"] = min(ps["rows"], key=lambda r: r["kernel_avg_us"])["shape"]
    if shared_gpu:
        ps["rehearsal_same_gpu"] = True
    ps["note"] = ("config 3's every-member fold with N-1 sources on peers, at the library's launch shape and at "
                  "tools/libpeershapes.so's (same kernel template), all PEs at once; kernel_avg_us max over PEs; "
                  "same_outputs: every output equal to the library's on every PE; measured in bench.py's child job")
    return {"xgmi_ceiling": xgmi_ceiling, "peer_fold_shapes": ps}


# ---------------------------------------------------------------------------
# kernel legs (N = 1): the fold kernels themselves, timed on one GPU
# ---------------------------------------------------------------------------
KERNEL_LEGS = [
    # name, kernel, op, dtype, sources, bytes per source, every-member orders
    ("fold_k2_double_sum", "combine_vec<sum,double,2>", "sum", "double", 2, 256 << 20, False),
    ("fold_k8_double_sum", "combine_vec<sum,double,8>", "sum", "double", 8, 256 << 20, False),
    ("rs_shard_n8_double_sum", "combine_orders_vec<sum,double,8>", "sum", "double", 8, 32 << 20, True),
    ("fold_k8_float_max", "combine_vec<max,float,8>", "max", "float", 8, 64 << 20, False),
    ("fold_k8_longlong_and", "combine_vec<and,longlong,8>", "and", "longlong", 8, 64 << 20, False),
    ("rs_shard_n8_float_max", "combine_orders_vec<max,float,8>", "max", "float", 8, 8 << 20, True),
    # long double (x87 arithmetic in software, x80.h): the sum is VALU-bound, the product HBM-bound
    ("rs_shard_n8_longdouble_sum", "combine_orders_vec<sum,x80,8>", "sum", "longdouble", 8, 32 << 20, True),
    ("rs_shard_n8_longdouble_prod", "combine_orders_vec<prod,x80,8>", "prod", "longdouble", 8, 32 << 20, True),
    # float complex product (C99 Annex G multiply; a lane whose chain met a NaN redoes it exactly)
    ("rs_shard_n8_complexf_prod", "combine_orders_vec<prod,cplxf,8>", "prod", "complexf", 8, 32 << 20, True),
    # what each GPU folds in BASELINE config 4's longlong and at N = 8: 8 shards of 8 MiB (64 MiB / 8);
    # bitwise and is order-free, so the P2P schedule runs the plain fold, one output per shard
    ("rs_shard_n8_longlong_and", "combine_vec<and,longlong,8>", "and", "longlong", 8, 8 << 20, False),
    # the same every-member folds at a quarter of their shard: with the 8 and 32 MiB legs they fit
    # t = fixed + bytes / rate per launch (FIXED_COST_FITS) -- why the small shards run below the big
    ("rs_shard_n8_float_max_2mib", "combine_orders_vec<max,float,8>", "max", "float", 8, 2 << 20, True),
    ("rs_shard_n8_double_sum_8mib", "combine_orders_vec<sum,double,8>", "sum", "double", 8, 8 << 20, True),
    # config 4's every-member float max on NaN-laden floats (the doubles' bytes read as floats: a NaN in
    # about one 16-byte vector in eight), which send min/max down their per-member chains
    ("rs_shard_n8_float_max_nan_rich", "combine_orders_vec<max,float,8>", "max", "float", 8, 8 << 20, True),
]
# float legs on the doubles' bytes read as floats; the others take the doubles' values rounded to
# float (SURVEY 8d's config-4 recipe: finite, full mantissa)
DOUBLE_BYTES_LEGS = {"rs_shard_n8_float_max_nan_rich"}
# (kernel, [legs of that kernel at two or more shard sizes]) for the fixed-cost fit
FIXED_COST_FITS = [("combine_orders_vec<max,float,8>", ["rs_shard_n8_float_max_2mib", "rs_shard_n8_float_max"]),
                   ("combine_orders_vec<sum,double,8>", ["rs_shard_n8_double_sum_8mib", "rs_shard_n8_double_sum"])]


def fixed_cost_fit(res):
    """Least-squares t = a + alg_bytes / B over the cold launches of one
    kernel at several shard sizes: a = the per-launch fixed cost (dispatch
    ramp of the grid and drain of its last wave, microseconds), B = the
    streaming rate between them; stream_frac = B / the HBM peak, what the
    kernel reaches once a launch is long enough to hide a."""
    out = {}
    for kname, legs in FIXED_COST_FITS:
        pts = [(res[g]["alg_bytes_per_launch"], res[g]["cold"]["kernel_avg_us"]) for g in legs
               if g in res and res[g].get("cold")]
        if len(pts) < 2:
            continue
        x = np.array([p[0] for p in pts], dtype=np.float64)
        y = np.array([p[1] for p in pts], dtype=np.float64)
        slope, a = np.polyfit(x, y, 1)
        if slope <= 0:
            continue
        rate = 1.0 / slope * 1e6   # bytes per second
        out[kname] = {"legs": legs, "fixed_us": round(float(a), 2), "stream_GB_s": round(rate / 1e9, 1),
                      "stream_frac": round(rate / 1e9 / HBM_PEAK_GBS, 4),
                      "fixed_share": {g: round(float(a) / res[g]["cold"]["kernel_avg_us"], 3) for g in legs}}
    out["note"] = ("cold launches of one kernel at two shard sizes fitted to t = fixed + bytes / rate: fixed = the "
                   "per-launch ramp and drain, rate = the streaming rate in between (stream_frac of the HBM peak); "
                   "fixed_share = the fixed part's share of each leg's cold time")
    return out
# each leg is timed twice: warm (the same buffers every launch, as the leg's
# own loop re-reads them) and cold (rotating disjoint buffer sets, >= 2 GiB of
# footprint, so no byte is still in the 256 MiB Infinity Cache)
COLD_FOOTPRINT = 2304 << 20
# Layout of the kernel legs' buffers: consecutive buffers LEG_STAGGER bytes
# further apart than their size. On the GPU the legs stand in for, a shard's
# sources are 8 different GPUs' arrays and its outputs this PE's target shard
# and version slots, which the library spaces by a shard + 256 + VER_STAGGER
# (4096) bytes (csrc/reduce.c ver_slot_bytes): nothing lines the streams up on
# the same HBM channels. Buffers exactly a power of two apart would
# (tools/probes/cold_probe orders_skew2); each leg also reports that layout
# ("warm_aligned", separate hipMalloc'd buffers) for comparison.
LEG_STAGGER = 4352
# the long double legs' VALU floor: their per-element instruction streams in
# this build priced at the measured issue rates -- computed by the library's
# build (csrc/Makefile, tools/valu_floor.py --bench-legs) into lib/valu_floor.json;
# a leg's bound is the larger of its VALU floor and its bytes at the HBM peak
VALU_FLOOR = os.path.join(ROOT, "osss-gasnet_amd", "lib", "valu_floor.json")


def kernel_legs(shm, reps, check):
    """The reduction's fold kernels on this GPU, called through the C ABI
    (include/mi355_reduce.h) on hipMalloc'd buffers, each launch stamped by a
    HIP event pair on its own stream (mi355_time_next_launch):
      fold_k*      mi355_combine: dst = src0 (+) ... (+) src(k-1), the
                   reduce-scatter kernel's shape with k local sources
                   (algorithmic bytes (k+1) x per-source bytes);
      rs_shard_n8  mi355_combine_orders: what each GPU runs in BASELINE
                   config 3 / 4 at N = 8 with the default result order -- 8
                   sources of one shard, 8 outputs (every member's reference
                   order), algorithmic bytes 16 x shard bytes.
    Sources: (uniform - 0.5) doubles, full mantissa (the float legs the same
    values rounded to float, except DOUBLE_BYTES_LEGS, which read the doubles'
    bytes as floats; the longlong legs read the same bytes as their type; the
    long double legs the same values widened to x87). Checked bit-exact (value bytes) against the oracle on a
    sample of every output. The long double legs also carry their VALU
    floor and the bound it implies (VALU_FLOOR)."""
    import ctypes
    import oracle
    L = shm.lib
    vp = ctypes.c_void_p
    L.mi355_time_next_launch.argtypes = [vp, vp]
    L.mi355_time_next_launch.restype = None
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    big = max(b for *_, b, _ in KERNEL_LEGS)
    nbuf = max(k for *_, k, _, _ in KERNEL_LEGS)
    srcs, hosts = [], []

    def dmalloc(nbytes):
        p = vp()
        if L.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) != 0:
            raise RuntimeError("hipMalloc failed")
        return p.value

    span = big + LEG_STAGGER
    pool0 = dmalloc(2 * nbuf * span)
    for p in range(nbuf):
        x = np.random.default_rng(77 + p).random(big // 8) - 0.5
        d = pool0 + p * span
        shm.put(d, x)
        srcs.append(d)
        hosts.append(x)
    outs = [pool0 + (nbuf + p) * span for p in range(nbuf)]
    al_srcs = [dmalloc(big) for _ in range(nbuf)]   # the power-of-two-aligned layout, for comparison
    al_outs = [dmalloc(big) for _ in range(nbuf)]
    ev = [vp() for _ in range(2 * reps)]
    for e in ev:
        L.hipEventCreate(ctypes.byref(e))
    res = {}
    rewritten = 0   # sources a float / long double / complex leg overwrote (the others read hosts' bytes)
    for name, kname, op, dtype, k, nbytes, orders in KERNEL_LEGS:
        es = np.dtype(shmem_reduce.NP[dtype]).itemsize
        n = nbytes // es
        nout = k if orders else 1
        rewrites = dtype in ("longdouble", "complexf") or (dtype == "float" and name not in DOUBLE_BYTES_LEGS)
        if not rewrites:
            for p in range(rewritten):
                shm.put(srcs[p], hosts[p])
            rewritten = 0
        else:
            rewritten = max(rewritten, k)
        if dtype == "longdouble":   # realistic x87 operands, not doubles' bytes read as x87
            lds = [hosts[p][:n].astype(np.longdouble) for p in range(k)]
            for p in range(k):
                shm.put(srcs[p], lds[p])
        if rewrites and dtype == "float":   # finite floats, full mantissa
            lds = [hosts[p][:n].astype(np.float32) for p in range(k)]
            for p in range(k):
                shm.put(srcs[p], lds[p])
        if dtype == "complexf":     # finite complex operands of magnitude ~1 (products stay finite)
            lds = [(hosts[p][:n] + 1j * hosts[p][n:2 * n]).astype(np.complex64) * np.float32(2) for p in range(k)]
            for p in range(k):
                shm.put(srcs[p], lds[p])

        def launch(so=srcs, oo=outs):
            if orders:
                return shm.combine_orders(op, dtype, oo[:k], so[:k], n)
            return shm.combine(op, dtype, oo[0], so[:k], n)

        def warm(so=srcs, oo=outs):
            for _ in range(3):
                assert launch(so, oo) == 0
            shm.sync()
            for r in range(reps):
                L.mi355_time_next_launch(ev[2 * r], ev[2 * r + 1])
                assert launch(so, oo) == 0
            shm.sync()
            ts = []
            for r in range(reps):
                ms = ctypes.c_float()
                L.hipEventElapsedTime(ctypes.byref(ms), ev[2 * r], ev[2 * r + 1])
                ts.append(ms.value * 1e-3)
            return ts

        ts = warm()
        t = float(np.mean(ts))
        alg = (k + nout) * nbytes
        gbs = alg / t / 1e9
        # the same launches on power-of-two-aligned buffers (same source bytes)
        for q in range(k):
            if L.hipMemcpy(vp(al_srcs[q]), vp(srcs[q]), ctypes.c_size_t(nbytes), 3) != 0:
                raise RuntimeError("hipMemcpy failed")
        ta = float(np.mean(warm(al_srcs, al_outs)))
        aligned = {"kernel_avg_us": round(ta * 1e6, 2), "frac": round(alg / ta / 1e9 / HBM_PEAK_GBS, 4)}
        # cold: `sets` disjoint copies of the leg's buffers taken in turn
        span_l = nbytes + LEG_STAGGER
        set_bytes = (k + nout) * span_l
        sets = max(1, -(-COLD_FOOTPRINT // set_bytes))
        cold_bufs = []
        if sets > 1:
            pool = dmalloc((sets - 1) * set_bytes)
            cold_bufs.append(pool)
            for j in range(sets - 1):
                base = pool + j * set_bytes
                for q in range(k):   # the same source bytes as set 0
                    if L.hipMemcpy(vp(base + q * span_l), vp(srcs[q]), ctypes.c_size_t(nbytes), 3) != 0:
                        raise RuntimeError("hipMemcpy failed")

        def launch_set(j):
            if j == 0:
                return launch()
            base = cold_bufs[0] + (j - 1) * set_bytes
            cs = [base + q * span_l for q in range(k)]
            co = [base + (k + q) * span_l for q in range(nout)]
            if orders:
                return shm.combine_orders(op, dtype, co, cs, n)
            return shm.combine(op, dtype, co[0], cs, n)

        creps = max(2 * sets, min(reps, 20)) if sets > 1 else min(reps, 20)
        cev = [vp() for _ in range(2 * creps)]
        for e in cev:
            L.hipEventCreate(ctypes.byref(e))
        for j in range(sets):
            assert launch_set(j) == 0
        shm.sync()
        for r in range(creps):
            L.mi355_time_next_launch(cev[2 * r], cev[2 * r + 1])
            assert launch_set(r % sets) == 0
        shm.sync()
        cts = []
        for r in range(creps):
            ms = ctypes.c_float()
            L.hipEventElapsedTime(ctypes.byref(ms), cev[2 * r], cev[2 * r + 1])
            cts.append(ms.value * 1e-3)
        for e in cev:
            L.hipEventDestroy(e)
        for b in cold_bufs:
            L.hipFree(vp(b))
        tc = float(np.mean(cts))
        cold = {"kernel_avg_us": round(tc * 1e6, 2), "achieved_GB_s": round(alg / tc / 1e9, 1),
                "frac": round(alg / tc / 1e9 / HBM_PEAK_GBS, 4), "sets": sets, "launches": creps,
                "footprint_MiB": sets * set_bytes >> 20}
        ck = "skipped"
        if check:
            idx = np.unique(np.random.default_rng(5).integers(0, n, 1 << 14))
            if rewrites:
                samp = [np.ascontiguousarray(x[idx]) for x in lds]
            else:
                samp = [np.ascontiguousarray(h.view(np.uint8)[:nbytes].view(shmem_reduce.NP[dtype])[idx])
                        for h in hosts[:k]]
            bad = 0
            for q in range(nout):
                got = shm.get(outs[q], n, dtype)[idx]
                want = oracle.reduce_pe(op, dtype, samp, q)
                bad += int((oracle.as_value_bytes(got, dtype) != oracle.as_value_bytes(want, dtype)).sum())
            ck = (f"bit-exact vs the oracle, {len(idx)} samples x {nout} output(s)" if bad == 0
                  else f"MISMATCH in {bad} bytes")
        res[name] = {"kernel": kname, "sources": k, "outputs": nout, "bytes_per_source": nbytes,
                     "alg_bytes_per_launch": alg, "kernel_avg_us": round(t * 1e6, 2),
                     "kernel_median_us": round(float(np.median(ts)) * 1e6, 2), "launches": reps,
                     "achieved_GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "check": ck,
                     "cold": cold, "warm_aligned": aligned}
        if dtype == "longdouble":
            try:
                fl = json.load(open(VALU_FLOOR))[name]
                hbm_floor_us = alg / (HBM_PEAK_GBS * 1e9) * 1e6
                res[name].update({"bound": "valu" if fl["floor_us"] > hbm_floor_us else "hbm",
                                  "valu_floor_us": fl["floor_us"], "hbm_floor_us": round(hbm_floor_us, 1),
                                  "valu_frac": round(fl["floor_us"] / (t * 1e6), 4),
                                  "valu_per_element_wave": fl["valu_per_element_wave"],
                                  "valu_note": "x87 arithmetic in integer code: valu_floor = this build's per-element "
                                               "instruction stream priced at the issue rates measured by "
                                               "tools/valu_rate.hip (profiles/r04/valu); bound = the larger of it and "
                                               "hbm_floor (alg bytes at 8 TB/s); frac above is the HBM view"})
            except (OSError, ValueError, KeyError) as e:   # the leg stands without its floor
                res[name]["valu_floor_error"] = f"{type(e).__name__}: {e}"
    for e in ev:
        L.hipEventDestroy(e)
    for d in [pool0] + al_srcs + al_outs:
        L.hipFree(vp(d))
    res["fixed_cost_fit"] = fixed_cost_fit(res)
    res["note"] = ("fold kernels timed alone (HIP event pair per launch on its stream), algorithmic bytes = "
                   "(sources + outputs) x bytes; frac against the 8 TB/s HBM peak; warm = the same buffers every "
                   "launch (a set under ~256 MiB stays in the Infinity Cache), cold = disjoint copies taken in "
                   "turn over >= 2 GiB: every byte from HBM; buffers %d bytes further apart than their size (a "
                   "shard's sources live on different GPUs, its outputs in version slots the library staggers); "
                   "warm_aligned = the same launches on separately hipMalloc'd buffers, which line the streams up "
                   "on the same HBM channels" % LEG_STAGGER)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--mib", type=int, default=256, help="MiB per PE")
    ap.add_argument("--algorithm", default=os.environ.get("SHMEM_REDUCE_ALGORITHM", "auto"))
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--no-small", action="store_true",
                    help="skip the 64 KiB small-call leg (profiling runs: keeps the dominant kernel's rocprof "
                         "average to the 256 MiB calls)")
    ap.add_argument("--no-rccl-compare", action="store_true",
                    help="N > 1: skip timing the same K calls through RCCL's ncclAllReduce (SHMEM_REDUCE_ALGORITHM"
                         "=rccl) beside the default P2P schedule")
    ap.add_argument("--force-rccl-compare", action="store_true",
                    help="attempt the RCCL comparison even when PEs share a GPU (exercises its failure path)")
    ap.add_argument("--no-ops", action="store_true",
                    help="skip the op-coverage leg (BASELINE config 4: float max + longlong and, 64 MiB per PE)")
    ap.add_argument("--no-kernels", action="store_true",
                    help="N = 1: skip the kernel legs (the fold kernels timed alone: k = 2 / 8 sources of "
                         "256 MiB, config 3 / 4's per-GPU reduce-scatter shapes)")
    ap.add_argument("--no-external", action="store_true",
                    help="N > 1: skip the leg on plain hipMalloc buffers (outside the symmetric heap)")
    ap.add_argument("--no-xgmi-legs", action="store_true",
                    help="N > 1: skip xgmi_ceiling and peer_fold_shapes (the child job's one-GPU-per-PE legs)")
    ap.add_argument("--force-xgmi-legs", action="store_true",
                    help="N > 1: run xgmi_ceiling and peer_fold_shapes even when the PEs share a GPU (a rehearsal of "
                         "their code path; the figures are local HBM rates and feed no roofline)")
    ap.add_argument("--no-link-probe", action="store_true",
                    help="N > 1: skip PE 0's one-peer-at-a-time shmem_getmem / shmem_putmem rates")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--no-rotating", action="store_true",
                    help="N = 1: skip headline_rotating (the same call over %d disjoint pairs, HBM-only)" % ROT_PAIRS)
    ap.add_argument("--no-fused", action="store_true",
                    help="N = 1: skip the fused-kernel leg (2 PE processes sharing this GPU, 64 KiB and 1 MiB calls)")
    ap.add_argument("--host", action="store_true",
                    help="source/target in host memory (shmem_malloc, page-locked): the rate includes the "
                         "H2D/D2H staging copies (DESIGN.md); not the headline metric")
    ap.add_argument("--no-collectives", action="store_true",
                    help="N > 1: skip the shmem_broadcast64 / shmem_fcollect64 leg")
    ap.add_argument("--no-threshold-sweep", action="store_true",
                    help="N > 1: skip the fused / multi-launch and one-shot / two-shot per-size comparison")
    ap.add_argument("--no-host-staged", action="store_true",
                    help="N = 1: skip the host_staged leg (the same call on page-locked host arrays, with the "
                         "same run's PCIe ceiling)")
    args = ap.parse_args()

    # wall time of every leg (legs_s in the line), and optional legs that fail
    # become an {"error": ...} entry instead of ending the headline line. A leg
    # that makes collective calls is optional only with one PE: at N > 1 a PE
    # that raised and went on would pair its next collective call with a
    # different call on its peers (a hang or a barrier-timeout abort), so
    # there it ends the run; such legs pass optional=solo.
    legs_s, leg_errors = {}, {}

    @contextlib.contextmanager
    def timed_leg(name, optional=True):
        t0 = time.perf_counter()
        # progress on stderr (the JSON line is stdout's only content): a run
        # that stops shows which leg it stopped in
        print(f"[bench rank {os.environ.get('RANK', '0')}] {name} ...", file=sys.stderr, flush=True)
        try:
            yield
        except Exception as e:  # noqa: BLE001 -- reported in the line
            if not optional:
                raise
            import traceback
            traceback.print_exc(file=sys.stderr)
            leg_errors[name] = f"{type(e).__name__}: {e}"
        finally:
            legs_s[name] = round(legs_s.get(name, 0.0) + time.perf_counter() - t0, 2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    S = args.mib << 20
    n = S // 8

    # N > 1: the opt-in persistent server's small calls, in a child job
    # (every rank at once, before any of them touches the GPU)
    small_p_child = None
    if world > 1 and not args.no_small and not args.host:
        with timed_leg("small_call_persistent"):
            small_p_child = persistent_child(rank, world, 4096)
    # N > 1: the legs never run with one GPU per PE before, in a child job too
    extra = {}
    if world > 1 and not args.host:
        with timed_leg("extra_legs_child"):
            extra = extra_legs_child(rank, world, args.mib, args.steps, args.algorithm,
                                     [f for f, on in (("--no-check", args.no_check), ("--no-external", args.no_external),
                                                      ("--no-link-probe", args.no_link_probe),
                                                      ("--no-collectives", args.no_collectives),
                                                      ("--no-xgmi-legs", args.no_xgmi_legs),
                                                      ("--no-config1", args.no_small),
                                                      ("--force-xgmi-legs", args.force_xgmi_legs)) if on])
    # CPU baseline, before this process initialises the GPU; at N > 1 the
    # other ranks wait for rank 0 in the bootstrap (SHMEM_BARRIER_TIMEOUT)
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        with timed_leg("cpu_baseline"):
            cpu = cpu_baseline(S, args.gpus, args.cpu_seconds)
    # the fused kernel on 2 PE processes sharing this GPU (children; this
    # process has not touched the GPU yet)
    fused = fused_p = None
    if world == 1 and not args.no_fused and not args.host:
        with timed_leg("fused_same_gpu"):
            fused = fused_same_gpu(2, 4096 if args.no_small is False else 512, config1=True)
        with timed_leg("fused_same_gpu_persistent"):
            fused_p = fused_same_gpu(2, 4096 if args.no_small is False else 512, persistent=True)
    t_init0 = time.perf_counter()

    # N = 1: room for headline_rotating's extra pairs too, and for the offset
    # leg's target (freed before the rotating leg allocates)
    pairs = ROT_PAIRS if world == 1 and not args.host and not args.no_rotating else 1
    heap = 2 * S * pairs
    if not args.host:
        heap = max(heap, 3 * S)   # N = 1: the offset leg's target; N > 1: peer_fold_shapes' outputs
    os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str(heap + (64 << 20)))
    os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", str(96 << 20))
    # a PE that never arrives ends the bench within two minutes with the
    # library's diagnostic (the library default, 600 s, suits long jobs)
    os.environ.setdefault("SHMEM_BARRIER_TIMEOUT", "120")
    # N > 1: ranks 1.. wait at init for rank 0, which first times the CPU
    # baseline (and, like every rank, waits for its two child jobs, at most
    # 240 s each): the bootstrap wait covers both
    os.environ.setdefault("SHMEM_BOOTSTRAP_TIMEOUT", "600")
    shm = shmem_reduce.Shmem()
    shm.init()
    legs_s["init"] = round(time.perf_counter() - t_init0, 2)
    print(f"[bench rank {rank}] headline ...", file=sys.stderr, flush=True)
    t_head0 = time.perf_counter()
    # the init self-test found peer heap reads broken: the library runs the
    # RCCL pairs through RCCL whatever is selected
    rccl_fallback = shm.n_pes() > 1 and shm.lib.shmemx_get_reduce_algorithm() == shmem_reduce.ALGORITHMS["rccl"] \
        and args.algorithm != "rccl"
    shm.set_algorithm(args.algorithm)
    me, npes = shm.my_pe(), shm.n_pes()
    solo = npes == 1
    # the init-time coherence test of peer-heap reads (runtime.c): on the
    # driver's 8-GPU node it proves or refutes the acquire protocol the P2P
    # schedules rely on
    coherence = None
    if npes > 1:
        ran, passed, stale = shm.coherence_selftest()
        sysload, no_acq = shm.coherence_sysload()
        prod_ran, prod = shm.coherence_producer()
        slow_waits, barrier_us = shm.device_wait_report()
        coherence = {"ran": ran, "passed": passed, "stale_without_acquire": stale,
                     "device_barrier_us": round(barrier_us, 1), "device_waits_timesliced": slow_waits,
                     "sysload_fresh": sysload, "fused_acquires_skipped": no_acq,
                     "producer_path": dict(prod, ran=prod_ran,
                                           note="32 words written with plain stores by a kernel on the null stream "
                                                "(a caller's producer), re-read by every peer after caching the old "
                                                "values: fused_* after the fused kernel's same-stream flag + device "
                                                "wait, host_* after the signal kernel + host wait + host barrier; "
                                                "plain loads without an acquire, 16-byte system-coherent loads, "
                                                "plain loads after a system-scope acquire"),
                     "note": "every PE read each peer's marker through its L2, the peer rewrote it (write-through), "
                             "and the re-read after mi355_acquire_system must see the new value; "
                             "stale_without_acquire: a re-read without the acquire returned the old value; "
                             "sysload_fresh: system-coherent (sc0 sc1) loads, the fused kernel's reads of the "
                             "members' buffers, saw every new value before any acquire, so the fused kernel "
                             "skips its per-block acquires (fused_acquires_skipped)"}
    if args.host:
        import ctypes
        src, dst = shm.malloc(S), shm.malloc(S)
        x = synth(me, np.arange(n, dtype=np.uint64))
        ctypes.memmove(src, x.ctypes.data, S)
        del x
    else:
        src = shm.malloc_device(S)
        dst = shm.malloc_device(S)
        shm.put(src, synth(me, np.arange(n, dtype=np.uint64)))

    # The K calls run in a C loop (osss-gasnet_amd/csrc/bench_loop.c): each is
    # shmem_double_sum_to_all called as a C program calls it, so the step time
    # is the library's entry-to-return time without ctypes marshalling.
    loop = shmem_reduce.bench_loop()

    def steps(k, nred=n):
        loop(dst, src, nred, 0, 0, npes, None, shm._psync_ptr, k)

    steps(args.warmup)
    # timed region: K steps, barrier + device synchronize on both sides
    shm.barrier_all()
    shm.sync()
    t0 = time.perf_counter()
    steps(args.steps)
    shm.sync()
    t_local = time.perf_counter() - t0
    shm.barrier_all()

    # kernel duration: the same K steps again with a HIP event pair attached to
    # each dominant kernel launch (hipExtLaunchKernel stamps on the library's
    # stream). Kept out of the region above: attaching events adds ~12 us of
    # host-side latency per call (tools/probes/overhead.py), not kernel time.
    shm.kernel_timing(True)
    t1 = time.perf_counter()
    steps(args.steps)
    shm.sync()
    t_local_ev = time.perf_counter() - t1
    shm.barrier_all()
    nk, k_total_ms, k_avg_ms = shm.kernel_timing_stats()
    nag, _, ag_avg_ms = shm.kernel_timing_phase_stats(1)   # N > 1: the all-gather copy
    shm.kernel_timing(False)
    # what the library ran for these calls: schedule, dominant kernel, bytes
    info = shm.last_call_info()
    # the per-call distribution (SURVEY 8d asks for the median over the timed
    # reps): the same K calls once more, each timed alone, outside the region
    # that yields `value`
    call_times = shmem_reduce.bench_call_times()
    shm.barrier_all()
    t_calls = call_times(dst, src, n, 0, 0, npes, shm._psync_ptr, args.steps)
    legs_s["headline"] = round(time.perf_counter() - t_head0, 2)

    # the call's fixed cost: the same entry point on 2 elements (one launch of
    # the same copy kernel, its completion flag, the return) -- what a
    # blocking call pays beside its kernel's duration
    t_tiny = None
    if npes == 1 and not args.host and not args.no_small:   # (profiling runs: the copy's rocprof average stays the headline's)
        steps(50, 2)
        ttq = time.perf_counter()
        steps(2000, 2)
        shm.sync()
        t_tiny = (time.perf_counter() - ttq) / 2000
        steps(1)   # the headline target again for the checks below

    # N = 1: the same call into a target one element off (offset_target_leg);
    # before the rotating leg, whose launches rocprof's split counts last
    offset_target = None
    if npes == 1 and not args.host:
        with timed_leg("headline_offset_target"):
            offset_target = offset_target_leg(shm, S, me, npes, src, args.steps, not args.no_check)

    # N = 1: the same call with every byte from HBM (rotating_leg)
    rotating = None
    if npes == 1 and not args.host and not args.no_rotating:
        with timed_leg("headline_rotating"):
            rotating = rotating_leg(shm, S, me, npes, src, dst, args.steps, not args.no_check)

    # the many-small-bucket regime (BASELINE config 5 shape: 64 KiB per call)
    small_n, small_calls = 8192, 0 if args.no_small else 4096   # BASELINE config 5: 4096 x 64 KiB
    t_small = None
    with timed_leg("small_call", optional=solo):
        if small_calls:
            steps(20, small_n)
            shm.barrier_all()
            shm.sync()
            ts0 = time.perf_counter()
            steps(small_calls, small_n)
            shm.sync()
            t_small = (time.perf_counter() - ts0) / small_calls
            small_info = shm.last_call_info()
            shm.barrier_all()
            t_small_calls = call_times(dst, src, small_n, 0, 0, npes, shm._psync_ptr, small_calls)
            # the last small call's result on every element: at N > 1 these calls run the fused
            # kernel, with its per-block acquires skipped when the init test allowed it
            # (coherence_selftest.fused_acquires_skipped), so the driver's multi-GPU line pins
            # that decision's correctness across GPUs
            small_bad = 0
            if not args.no_check:
                import oracle
                sidx = np.arange(small_n, dtype=np.uint64)
                got_s = shm.get(dst, small_n, "double")
                want_s = oracle.reduce_pe("sum", "double", [synth(p, sidx) for p in range(npes)], me)
                small_bad = int((got_s.view(np.uint64) != want_s.view(np.uint64)).sum())

    # N = 1: the same calls with the opt-in persistent server (shmemx.h
    # shmemx_set_persistent): the identity copy served by a resident one-member
    # fused kernel, no launch per call. Not at N > 1 (kept out of the driver's
    # multi-GPU line; the same-GPU multi-PE figures are in fused_same_gpu_persistent).
    with timed_leg("small_call_persistent"):
        t_small_p = None
        if small_calls and npes == 1 and not args.host:
            shm.set_persistent(True)
            served0, launched0 = shm.persistent_stats()
            steps(20, small_n)
            shm.barrier_all()
            ts0 = time.perf_counter()
            steps(small_calls, small_n)
            t_small_p = (time.perf_counter() - ts0) / small_calls
            served1, launched1 = shm.persistent_stats()
            shm.set_persistent(False)  # stops the server
            shm.sync()
            shm.barrier_all()

    # The same 64 KiB calls through the stream-ordered API (shmemx.h), 64 of
    # them captured once into a HIP graph and the graph replayed: how a caller
    # that batches small buckets into a graph (e.g. torch.cuda.graph) sees
    # them; the graph launch and its wait amortised over its 64 calls.
    with timed_leg("small_call_graph", optional=solo):
        small_graph = None
        if small_calls and not args.host and not rccl_fallback:
            per_graph, replays = 64, max(1, small_calls // 64)
            st = shm.stream_create()
            gsrc, gdst = shm.malloc_device(small_n * 8), shm.malloc_device(small_n * 8)
            shm.put(gsrc, synth(me, np.arange(small_n, dtype=np.uint64)))
            shm.to_all_on_stream("sum", "double", gdst, gsrc, small_n, 0, 0, npes, st)
            shm.stream_sync(st)
            shm.capture_begin(st)
            for _ in range(per_graph):
                shm.to_all_on_stream("sum", "double", gdst, gsrc, small_n, 0, 0, npes, st)
            graph, exe = shm.capture_end(st)
            shm.graph_launch(exe, st)
            shm.stream_sync(st)
            shm.barrier_all()
            tg0 = time.perf_counter()
            for _ in range(replays):
                shm.graph_launch(exe, st)
                shm.stream_sync(st)
            t_graph_local = (time.perf_counter() - tg0) / (replays * per_graph)
            gsched = shm.last_call_info()["schedule"]
            ck = "skipped"
            if not args.no_check:
                import oracle
                idx = np.arange(small_n, dtype=np.uint64)
                got = shm.get(gdst, small_n, "double")
                want = oracle.reduce_pe("sum", "double", [synth(p, idx) for p in range(npes)], me)
                ck = (got.view(np.uint64) != want.view(np.uint64)).sum()
            shm.graph_destroy(graph, exe)
            shm.stream_destroy(st)
            shm.barrier_all()
            shm.free_device(gdst)
            shm.free_device(gsrc)
            small_graph = {"bytes_per_pe": small_n * 8, "calls": replays * per_graph, "calls_per_graph": per_graph,
                           "t_local": t_graph_local, "schedule": gsched, "bad": ck,
                           "note": "the 64 KiB calls as shmemx_double_sum_to_all_on_stream, 64 per HIP graph, the graph "
                                   "replayed and waited for: per-call time including the graph launch and wait"}

    # N > 1: the same K calls through RCCL (ncclAllReduce on the whole job,
    # SHMEM_REDUCE_ALGORITHM=rccl) for comparison with the P2P schedule; the
    # headline value stays the default schedule's
    t_rccl0 = time.perf_counter()
    t_rccl_local = None
    distinct_gpus = shared_gpu = False
    pes_on_gpu = 1   # PEs on this PE's GPU, itself included (test layouts share one)
    if npes > 1:
        # RCCL refuses two ranks on one device: compare only with one GPU per
        # PE. Same GPU = same PCI bus id (not the HIP ordinal, which is 0 on
        # every rank under a launcher that shows each rank one GPU).
        shared = np.array([sum(shm.lib.shmemx_pe_same_device(q) for q in range(npes) if q != me)],
                          dtype=np.int32)
        anyshared = np.zeros(1, dtype=np.int32)
        shm.to_all("max", "int", anyshared.ctypes.data, shared.ctypes.data, 1, 0, 0, npes)
        shared_gpu = int(anyshared[0]) != 0
        pes_on_gpu = 1 + int(shared[0])
        distinct_gpus = not shared_gpu or args.force_rccl_compare
    rccl_ok = False
    # RCCL prints a version banner on stdout at communicator creation; keep
    # stdout to the one JSON line by pointing fd 1 at stderr meanwhile
    sys.stdout.flush()
    saved_stdout = os.dup(1)
    os.dup2(2, 1)
    if npes > 1 and distinct_gpus and not args.no_rccl_compare and not args.host and not rccl_fallback:
        # non-blocking RCCL bring-up with a deadline; every PE must have it
        mine = np.array([1 if shm.lib.shmemx_rccl_init(60.0) == 0 else 0], dtype=np.int32)
        allok = np.zeros(1, dtype=np.int32)
        shm.to_all("min", "int", allok.ctypes.data, mine.ctypes.data, 1, 0, 0, npes)
        rccl_ok = bool(allok[0])
        if rccl_ok:
            # one probe allreduce through the glue, which reports a failure
            # instead of aborting the job (the timed loop below goes through
            # the public entry point, where a failure is fatal)
            import ctypes
            f = shm.lib.shmemi_rccl_allreduce
            f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
            f.restype = ctypes.c_int
            mine[0] = 1 if f(shmem_reduce.OPS.index("sum"), shmem_reduce.DTYPES.index("double"), src, dst,
                             1024) == 0 else 0
            shm.to_all("min", "int", allok.ctypes.data, mine.ctypes.data, 1, 0, 0, npes)
            rccl_ok = bool(allok[0])
    if rccl_ok:
        shm.set_algorithm("rccl")
        steps(3)
        shm.barrier_all()
        shm.sync()
        tr0 = time.perf_counter()
        steps(args.steps)
        shm.sync()
        t_rccl_local = time.perf_counter() - tr0
        shm.barrier_all()
        shm.set_algorithm(args.algorithm)
    if npes > 1 and distinct_gpus and not args.no_rccl_compare and not args.host and not rccl_fallback:
        steps(1)  # the target again from the default schedule (RCCL wrote it), for the check below
    sys.stdout.flush()
    os.dup2(saved_stdout, 1)
    os.close(saved_stdout)
    legs_s["rccl_compare"] = round(time.perf_counter() - t_rccl0, 2)
    # an optional leg that failed reports {"error": ...} (below), not a partial record
    if "small_call" in leg_errors:
        t_small = None
    if "small_call_persistent" in leg_errors:
        t_small_p = None
    if "small_call_graph" in leg_errors:
        small_graph = None

    # max over PEs, through the library's own host-staged double max reduction
    def max_over_pes(x):
        tbuf = np.array([x], dtype=np.float64)
        tout = np.zeros(1, dtype=np.float64)
        shm.to_all("max", "double", tout.ctypes.data, tbuf.ctypes.data, 1, 0, 0, npes)
        return float(tout[0])

    t_check0 = time.perf_counter()
    t_step = max_over_pes(t_local) / args.steps
    call_dist = {"median_us": round(max_over_pes(float(np.median(t_calls))), 2),
                "p10_us": round(max_over_pes(float(np.percentile(t_calls, 10))), 2),
                "p90_us": round(max_over_pes(float(np.percentile(t_calls, 90))), 2),
                "max_us": round(max_over_pes(float(t_calls.max())), 2), "calls": int(len(t_calls)),
                "note": "the headline call timed one by one (CLOCK_MONOTONIC around each blocking call, a separate "
                        "run of K calls); each statistic is the max over PEs of that PE's statistic"}
    if small_graph is not None:
        t_sg = max_over_pes(small_graph.pop("t_local"))
        bad = small_graph.pop("bad")
        small_graph["us_per_call"] = round(t_sg * 1e6, 2)
        small_graph["check"] = "skipped" if isinstance(bad, str) else \
            "bit-exact, every element" if int(max_over_pes(int(bad))) == 0 else "MISMATCH"

    if t_small is not None:
        t_small = max_over_pes(t_small)
        small_dist = {"median_us": round(max_over_pes(float(np.median(t_small_calls))), 2),
                      "p99_us": round(max_over_pes(float(np.percentile(t_small_calls, 99))), 2)}
        small_check = "skipped" if args.no_check else \
            "bit-exact vs the reference's per-PE order, every element, every PE" \
            if int(max_over_pes(small_bad)) == 0 else "MISMATCH"
    rccl = None
    if npes > 1 and distinct_gpus and not args.no_rccl_compare and not args.host and not rccl_ok and not rccl_fallback:
        rccl = {"error": "RCCL did not come up (communicator within 60 s, or a probe allreduce) on every PE; "
                         "comparison skipped"}
    if t_rccl_local is not None:
        tr_step = max_over_pes(t_rccl_local) / args.steps
        rccl = {"ms_per_step": round(tr_step * 1e3, 4), "value": round(npes * S / tr_step / GIB, 2),
                "busbw_GB_s_per_pe": round(2.0 * (npes - 1) / npes * S / tr_step / 1e9, 1),
                "p2p_speedup": round(tr_step / t_step, 3),
                "note": "same K calls with SHMEM_REDUCE_ALGORITHM=rccl (ncclAllReduce, RCCL's order: "
                        "FP results within tolerance, not bit-exact); comparison only, not the headline"}

    # correctness of the last result on a sample: every PE holds the
    # reference's result for itself (own source first, then ascending)
    check, check_sha = "skipped", None
    if not args.no_check and not rccl_fallback:
        # every element of every PE's target against the oracle's result for
        # that PE (a stale line from a peer would not hide in a sample)
        bad, hg, hw = full_check(shm, dst, n, "sum", "double", synth, npes, me, host=args.host)
        check, check_sha = full_check_record(shm, npes, me, bad, hg, hw, max_over_pes)
    elif not args.no_check:
        idx = np.unique(np.random.default_rng(me).integers(0, n, 1 << 16).astype(np.uint64))
        got_full = shm.get(dst, n, "double")
        got = got_full[idx.astype(np.int64)]
        import oracle
        srcs = [synth(p, idx) for p in range(npes)]
        want = oracle.reduce_pe("sum", "double", srcs, me)
        if rccl_fallback:
            # RCCL's order: within 2 (N-1) u sum|x_i| of the reference's result
            bound = 2 * (npes - 1) * 2.0 ** -53 * np.abs(np.stack(srcs)).sum(axis=0)
            bad = int(max_over_pes(int((np.abs(got - want) > bound).sum())))
            check = ("RCCL fallback (peer heap reads failed the init self-test): within 2(N-1)u sum|x| of the "
                     "reference's per-PE result on every PE, %d samples each" % len(idx) if bad == 0
                     else "MISMATCH %d of %d samples beyond the FP bound (worst PE)" % (bad, len(idx)))
        del got_full
    legs_s["check"] = round(time.perf_counter() - t_check0, 2)

    # N > 1, one GPU per PE: the measured xGMI ceiling and the peer-fold
    # shapes, measured in the child job (extra_legs_child, before this rank
    # touched the GPU: a failure there cannot take the headline with it)
    xgmi_ceiling = peer_shapes = None
    if npes > 1 and not args.host:
        xgmi_ceiling = extra.get("xgmi_ceiling")
        peer_shapes = extra.get("peer_fold_shapes")

    # N = 1: north_star's host-memory rate -- the same call on shmem_malloc's
    # page-locked host arrays, staged over PCIe inside each call, with the
    # same run's PCIe ceiling (host_staged_leg)
    host_staged = None
    if npes == 1 and not args.host and not args.no_host_staged:
        with timed_leg("host_staged"):
            host_staged = host_staged_leg(shm, loop, S, me, npes, max(10, args.steps), not args.no_check)

    with timed_leg("kernels"):
        kernels = None
        if npes == 1 and not args.no_kernels and not args.host:
            kernels = kernel_legs(shm, args.kernel_reps, not args.no_check)
            for name, leg in kernels.items():
                if isinstance(leg, dict) and "alg_bytes_per_launch" in leg:
                    leg["traffic_note"] = traffic_for(leg, f"kernel_{name}", False)
                    if leg.get("traffic"):
                        leg["traffic_over_alg"] = round(leg["traffic"] / leg["alg_bytes_per_launch"], 4)

    # BASELINE config 4 (op coverage): shmem_float_max_to_all and
    # shmem_longlong_and_to_all on 64 MiB per PE, timed like the headline
    # (C loop, max over PEs) and checked bit-exact on a sample
    with timed_leg("op_coverage", optional=solo):
        ops = None
        if not args.no_ops and not args.host:
            import oracle
            ops = {}
            ob = min(64 << 20, S)
            for name, op, dtype, es, gen in (
                    ("float_max", "max", "float", 4, lambda pe, i: synth(pe, i).astype(np.float32)),
                    ("longlong_and", "and", "longlong", 8, synth_bits)):
                if rccl_fallback and op == "and":
                    ops[name] = {"skipped": "RCCL fallback (peer heap reads failed the init self-test): no bitwise and"}
                    continue
                no = ob // es
                shm.put(src, gen(me, np.arange(no, dtype=np.uint64)))
                oloop = shmem_reduce.bench_loop(name=name)
                k = max(10, args.steps // 4)
                oloop(dst, src, no, 0, 0, npes, None, shm._psync_ptr, 3)
                shm.barrier_all()
                shm.sync()
                to0 = time.perf_counter()
                oloop(dst, src, no, 0, 0, npes, None, shm._psync_ptr, k)
                shm.sync()
                t_op = max_over_pes(time.perf_counter() - to0) / k
                shm.barrier_all()
                ck, sha = "skipped", None
                if not args.no_check:
                    bad, hg, hw = full_check(shm, dst, no, op, dtype, gen, npes, me)
                    ck, sha = full_check_record(shm, npes, me, bad, hg, hw, max_over_pes)
                ops[name] = {"bytes_per_pe": ob, "steps": k, "us_per_call": round(t_op * 1e6, 2),
                             "value": round(npes * ob / t_op / GIB, 2), "per_pe_gib_s": round(ob / t_op / GIB, 2),
                             "check": ck, "target_sha256_pe0": sha}
            ops["note"] = ("BASELINE config 4 (op coverage): shmem_float_max_to_all and shmem_longlong_and_to_all, "
                           "64 MiB per PE, GiB/s reduced whole job; longlong words with bits 1 at p = 7/8")

    # BASELINE config 1's call through the library (2 PEs, 4 KiB int sum, host
    # and device heap): at N = 1 from fused_same_gpu's two PE processes, at
    # N > 1 on PEs 0 and 1 of the child job, beside the CPU's figure for the same call
    config1_call = None
    if not args.host:
        with timed_leg("config1_call", optional=solo):
            if npes > 1:   # measured in the child job (extra_legs_child)
                config1_call = extra.get("config1_call")
                if config1_call is not None and "error" not in config1_call:
                    config1_call["layout"] = ("PEs 0 and 1 of this job" +
                                              (" (sharing one GPU)" if shared_gpu else ", one GPU each"))
            elif fused and fused.get("config1"):
                config1_call = dict(fused["config1"], layout="2 PE processes sharing this GPU (fused_same_gpu)")
            if config1_call is not None and "error" not in config1_call:
                cpu_c1 = (cpu or {}).get("config1", {}).get("us_per_call")
                config1_call["cpu_us_per_call"] = cpu_c1
                config1_call["note"] = ("BASELINE config 1's call: shmem_int_sum_to_all, 4 KiB, active set of 2 PEs; "
                                        "host_heap = shmem_malloc's arrays (host memory, as the reference's heap), "
                                        "device_heap = shmemx_malloc_device's; us per call entry-to-return, max over "
                                        "the 2 PEs; cpu_us_per_call = cpu_baseline.config1 (the reference algorithm "
                                        "on 2 host cores)")

    # N > 1: the same call on plain hipMalloc buffers (a framework's tensors,
    # outside the symmetric heap: the members map each other's allocations for
    # the call, csrc/extmap.c), PE 0's one-peer-at-a-time link rates and the
    # broadcast / fcollect collectives -- measured in the child job before
    # this process touched the GPU (extra_legs_child); their records here
    external = extra.get("external_buffers")
    if external and "us_per_call" in external:
        external["over_heap_buffers"] = round(external["us_per_call"] * 1e-6 / t_step, 3)
    link_probe = extra.get("link_probe")
    if link_probe and shared_gpu and "note" in link_probe:
        link_probe["note"] += "; the PEs share ONE GPU here: local HBM copies, not link rates"
    collectives = extra.get("collectives")

    # N > 1: where the fused one-launch kernel stops paying, on this layout --
    # the same calls per message size with the fused path forced on (fused_max
    # 1 GiB) and off (0, the multi-launch schedule), and one-shot vs two-shot
    # inside the fused kernel: the data to set SHMEM_FUSED_MAX_BYTES /
    # SHMEM_ONESHOT_MAX_BYTES from one GPU per PE (defaults 2 MiB / 64 KiB were
    # set with the PEs sharing one GPU)
    threshold_sweep = None
    if npes > 1 and not args.host and not args.no_threshold_sweep and not rccl_fallback:
        with timed_leg("threshold_sweep", optional=solo):
            import oracle
            f0, o0 = shm.thresholds()

            def per_call(nel, fused_max, oneshot_max, calls=200):
                shm.set_fused_max(fused_max)
                shm.set_oneshot_max(oneshot_max)
                loop(dst, src, nel, 0, 0, npes, None, shm._psync_ptr, 10)
                shm.barrier_all()
                tq = time.perf_counter()
                loop(dst, src, nel, 0, 0, npes, None, shm._psync_ptr, calls)
                shm.sync()
                t_loc = (time.perf_counter() - tq) / calls
                sched = shm.last_call_info()["schedule"]   # before max_over_pes: its own call replaces it
                t = max_over_pes(t_loc)
                m = min(nel, 4096)
                sidx = np.arange(m, dtype=np.uint64)
                got = shm.get(dst, m, "double")
                want = oracle.reduce_pe("sum", "double", [synth(p, sidx) for p in range(npes)], me)
                bad = int(max_over_pes(int((got.view(np.uint64) != want.view(np.uint64)).sum())))
                return round(t * 1e6, 2), sched, bad

            shm.put(src, synth(me, np.arange(n, dtype=np.uint64)))  # the op-coverage leg rewrote src
            rows, bad_total, oneshot = [], 0, []
            try:
                for nb in (64 << 10, 256 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20):
                    fu, fs, b1 = per_call(nb // 8, 1 << 30, o0)
                    mu, ms, b2 = per_call(nb // 8, 0, o0)
                    bad_total += b1 + b2
                    rows.append({"bytes": nb, "fused_us": fu, "fused_schedule": fs, "multi_launch_us": mu,
                                 "multi_launch_schedule": ms})
                for nb in (16 << 10, 64 << 10, 256 << 10):
                    ou, osch, b1 = per_call(nb // 8, 1 << 30, 1 << 30)
                    tu, tsch, b2 = per_call(nb // 8, 1 << 30, 0)
                    bad_total += b1 + b2
                    oneshot.append({"bytes": nb, "oneshot_us": ou, "oneshot_schedule": osch, "twoshot_us": tu,
                                    "twoshot_schedule": tsch})
            finally:   # the thresholds in force for any later call, whatever happened
                shm.set_fused_max(f0)
                shm.set_oneshot_max(o0)
            wins = [r["bytes"] for r in rows if r["fused_us"] < r["multi_launch_us"]]
            cal = shm.threshold_calibration()
            threshold_sweep = {
                "fused_vs_multi_launch": rows, "oneshot_vs_twoshot": oneshot,
                "largest_size_fused_wins": max(wins) if wins else 0,
                "defaults": {"fused_max": f0, "oneshot_max": o0},
                "calibrated_at_init": None if cal is None else {
                    "fused_max": f0, "oneshot_max": o0,
                    "fused_vs_multi_launch_us": [[b, round(a, 2), round(m, 2)] for b, a, m in cal["fused"]],
                    "oneshot_vs_twoshot_us": [[b, round(a, 2), round(m, 2)] for b, a, m in cal["oneshot"]],
                    "note": "set by shmem_init on this layout (shmemx_threshold_calibration): each threshold is the "
                            "largest size of the prefix where the fused (one-shot) call's median, max over PEs, was "
                            "no slower"},
                "fused_no_slower_up_to_fused_max": all(r["fused_us"] <= r["multi_launch_us"] for r in rows
                                                       if r["bytes"] <= f0),
                "check": "bit-exact (first 4096 elements, every PE, every size and mode)" if bad_total == 0
                else "MISMATCH in %d elements" % bad_total,
                "note": "us per shmem_double_sum_to_all call (200 calls, max over PEs) with the fused path forced "
                        "on (shmemx_set_fused_max_bytes(1 GiB)) and off (0: multi-launch), and inside the fused "
                        "kernel one-shot vs two-shot (shmemx_set_oneshot_max_bytes)"}

    # dominant kernel and its algorithmic bytes per launch, from the schedule
    # the library reports for the timed calls (shmemx_last_call_info)
    launches = max(1, info["launches"])
    alg_bytes = info["alg_bytes"]
    kname = info["kernel"] or "ncclAllReduce (RCCL's kernels)"
    kt_s = k_avg_ms * 1e-3 * launches   # the dominant kernel's time per call
    sched = {"schedule": info["schedule"], "ordered": bool(info["ordered"]), "sources": info["sources"],
             "outputs": info["outputs"], "peer_sources": info["peer_sources"], "launches_per_call": launches,
             "bytes_per_buffer": info["bytes_per_buffer"]}
    if npes == 1:
        achieved = alg_bytes / kt_s / 1e9 if k_avg_ms > 0 else 0.0
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                    "kernel": kname, "alg_bytes_per_launch": alg_bytes // launches,
                    "kernel_avg_us": round(k_avg_ms * 1e3, 2),
                    "launches_timed": nk, "ms_per_step_with_events": round(t_local_ev / args.steps * 1e3, 4),
                    "call": sched}
        if rotating and "frac" in rotating:
            # which figure is HBM: the timed region re-reads one pair, the
            # rotating leg streams every byte from HBM. Scalar keys: the
            # driver's record of the line keeps no nested objects.
            roofline.update({"hbm_only_frac": rotating["frac"], "hbm_only_kernel_avg_us": rotating["kernel_avg_us"],
                             "hbm_only_achieved": rotating["achieved_GB_s"],
                             "hbm_only_footprint_MiB": rotating["footprint_MiB"],
                             "hbm_only_launches_timed": rotating["launches_timed"]})
            roofline["attribution"] = (
                "frac is the timed region's: the same 256 MiB source/target pair every call (512 MiB per call), "
                "part of which the 256 MiB Infinity Cache serves, so it is a device-memory rate, not HBM alone; "
                "hbm_only_* is the same kernel over %d disjoint pairs taken in turn (headline_rotating, %d MiB "
                "footprint): every byte from HBM" % (ROT_PAIRS, rotating["footprint_MiB"]))
        roofline.update({"call_schedule": sched["schedule"], "call_launches": sched["launches_per_call"]})
    else:
        # N > 1: the reduce-scatter fold reads N-1 of its N shard sources from
        # peers over xGMI, so its bound is the links into this GPU: achieved =
        # those peer bytes / the fold's duration against (N-1) x 153 GB/s. Its
        # local-HBM view (every source and output byte) is kept in `hbm`.
        remote = info["peer_bytes"]
        achieved = remote / kt_s / 1e9 if k_avg_ms > 0 else 0.0
        peak = (npes - 1) * XGMI_LINK_GBS
        hbm_gbs = alg_bytes / kt_s / 1e9 if k_avg_ms > 0 else 0.0
        if rccl_fallback:
            kname = "ncclAllReduce (RCCL fallback: P2P self-test failed; the whole exchange, not one leg)"
        measured = (xgmi_ceiling or {}).get("peak_measured_GB_s")
        # a bound that this run's own pull exceeds is no bound: take the measured ceiling
        peak_source = "(N-1) x 153 GB/s"
        if measured and measured > peak:
            peak, peak_source = measured, "measured (xgmi_ceiling): above (N-1) x 153 GB/s"
        roofline = {"bound": "xgmi", "achieved": round(achieved, 1), "peak": peak, "unit": "GB/s",
                    "frac": round(achieved / peak, 4), "traffic": None, "kernel": kname,
                    "alg_bytes_per_launch": remote // launches, "kernel_avg_us": round(k_avg_ms * 1e3, 2),
                    "launches_timed": nk, "ms_per_step_with_events": round(t_local_ev / args.steps * 1e3, 4),
                    "call": sched,
                    "peak_note": "(N-1) links x 153 GB/s into this GPU (SURVEY 8d); if 153.6 GB/s counts both "
                                 "directions the one-way bound is half: see xgmi.frac_one_direction; "
                                 "peak_measured_GB_s = this run's all-peers pull ceiling (xgmi_ceiling)",
                    "peak_measured_GB_s": measured, "peak_source": peak_source,
                    "frac_of_measured": round(achieved / measured, 4) if measured and achieved <= measured else None,
                    "call_schedule": sched["schedule"], "call_launches": sched["launches_per_call"],
                    "hbm_frac": round(hbm_gbs / HBM_PEAK_GBS, 4),
                    "hbm": {"bytes_per_launch": alg_bytes // launches, "achieved": round(hbm_gbs, 1),
                            "peak": HBM_PEAK_GBS, "frac": round(hbm_gbs / HBM_PEAK_GBS, 4),
                            "note": "the same fold counted as local HBM traffic: its %d shard sources read + %d "
                                    "output(s) written (%s)" % (info["sources"], info["outputs"],
                                                                 "this PE's target shard and the other members' "
                                                                 "versions" if info["ordered"] else
                                                                 "this PE's target shard")}}
        if shared_gpu:
            # PEs sharing ONE GPU (test layout): the 'remote' reads are this
            # GPU's own HBM, so the bound is HBM; the link view is kept aside.
            # The device rate counts every PE's fold bytes on this GPU over a
            # window that holds all of their launches: each call's wall time
            # (t_step, max over PEs) -- every PE's folds ran between the
            # call's first entry and its last return, so this is a lower
            # bound on the rate the folds achieved together (<= 1 of HBM by
            # construction). One launch's own rate is kept as per_launch_*.
            for k in ("bound", "achieved", "peak", "frac", "alg_bytes_per_launch", "peak_note", "peak_measured_GB_s",
                      "frac_of_measured", "peak_source"):
                roofline.pop(k)
            h = roofline.pop("hbm")
            dev = pes_on_gpu * alg_bytes / t_step / 1e9
            roofline = {"bound": "hbm", "achieved": round(dev, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(dev / HBM_PEAK_GBS, 4), "traffic": None,
                        "alg_bytes_per_launch": h["bytes_per_launch"], "pes_on_gpu": pes_on_gpu,
                        "per_launch_achieved": h["achieved"], "per_launch_frac": h["frac"],
                        **roofline, "hbm_note": h["note"], "xgmi_view": None,
                        "xgmi_view_note": "not applicable: the PEs share a GPU, no link carries the peer reads",
                        "note": "the PEs share ONE GPU (test layout): every 'remote' read is this GPU's own HBM, "
                                "so the fold is HBM-bound here; achieved = %d PEs x one call's fold bytes / the "
                                "call's wall time (max over PEs), a window holding every PE's launches: a lower "
                                "bound on their combined rate; per_launch_* = one launch's bytes over its own "
                                "duration; with one GPU per PE the line reports the link view instead" % pes_on_gpu}
    roofline["traffic_note"] = traffic_for(roofline, f"n{npes}_{args.mib}mib", args.host)

    # N > 1: bus bandwidth of the reduce-scatter + all-gather exchange against
    # the full-mesh xGMI bound: each PE moves 2(N-1)/N * S
    # over its N-1 links, t >= 2 S / (N * 153 GB/s)
    xgmi = None
    if npes > 1:
        busbw = 2.0 * (npes - 1) / npes * S / t_step / 1e9
        bound = (npes - 1) * XGMI_LINK_GBS
        rs_remote = info["peer_bytes"] / (k_avg_ms * 1e-3 * launches) / 1e9 if k_avg_ms > 0 else None
        bound_dir = (npes - 1) * XGMI_LINK_DIR_GBS
        xgmi = {"busbw_GB_s_per_pe": round(busbw, 1), "mesh_bound_GB_s_per_pe": bound,
                "frac": round(busbw / bound, 4),
                "mesh_bound_one_direction_GB_s_per_pe": round(bound_dir, 1),
                "frac_one_direction": round(busbw / bound_dir, 4),
                "rs_kernel_remote_read_GB_s": None if rs_remote is None else round(rs_remote, 1),
                "ag_kernel_avg_us": round(ag_avg_ms * 1e3, 2) if nag else None,
                "ag_kernel_remote_read_GB_s": round((npes - 1) / npes * S / (ag_avg_ms * 1e-3) / 1e9, 1)
                if nag and ag_avg_ms > 0 else None,
                "note": "busbw = 2(N-1)/N * S / t_step = bytes each PE receives over xGMI per second; "
                        "bound = (N-1) links x 153 GB/s (SURVEY 8d), or x 76.8 GB/s if 153.6 is both directions; "
                        "peak_measured = this run's all-peers pull ceiling (xgmi_ceiling)"}
        pm = (xgmi_ceiling or {}).get("peak_measured_GB_s")
        xgmi["peak_measured_GB_s"] = pm
        xgmi["frac_of_measured"] = round(busbw / pm, 4) if pm and busbw <= pm else None
        # a constant bound below what this run moved is refuted, not exceeded
        for k, b in (("frac", bound), ("frac_one_direction", bound_dir)):
            if not shared_gpu and xgmi[k] is not None and xgmi[k] > 1:
                xgmi[k] = None
                xgmi["refuted_" + k] = "busbw %.1f GB/s exceeds this bound (%.1f GB/s)" % (busbw, b)
        import ctypes
        lt, hp = ctypes.c_int(), ctypes.c_int()
        links = {}
        for q in range(1, npes):
            if shm.lib.shmemx_peer_link(q, ctypes.byref(lt), ctypes.byref(hp)) == 0:
                links[str(q)] = {"type": {4: "xgmi", 2: "pcie"}.get(lt.value, str(lt.value)), "hops": hp.value}
        xgmi["links_from_pe0"] = links or None
        if shared_gpu:
            # no link: a fraction of a link bound would be meaningless (> 1)
            for k in ("frac", "frac_one_direction", "frac_of_measured"):
                xgmi[k] = None
            xgmi["note"] = ("the PEs share ONE GPU (test layout): peer 'xGMI' reads are local HBM reads, so "
                            "these figures are not xGMI rates and no link fraction is given")

    if me == 0:
        out = {
            "metric": ("GiB/s reduced (host-staged incl. H2D/D2H), shmem_double_sum_to_all @256MiB" if args.host else
                       "GiB/s reduced (device-resident), shmem_double_sum_to_all @256MiB, 1/2/4/8 GPU"),
            "value": round(npes * S / t_step / GIB, 2),
            "unit": "GiB/s",
            "n_gpus": npes,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 full-mantissa doubles, device-resident symmetric heap)",
            "config": {"workload": f"shmem_double_sum_to_all, {npes} PE = {npes} GPU"
                                   f"{f' (test layout: {pes_on_gpu} PEs share each GPU)' if shared_gpu else ''}, {args.mib} MiB "
                                   f"{'host-memory (staged)' if args.host else 'device-resident'} array per PE", "nreduce": n, "bytes_per_pe": S,
                       "algorithm": "rccl (fallback: P2P self-test failed)" if rccl_fallback else args.algorithm,
                       "parallelism": f"pe{npes}"},
            "per_pe_gib_s": round(S / t_step / GIB, 2),
            "per_call": call_dist,
            "fixed_cost": None if t_tiny is None else {
                "tiny_call_us": round(t_tiny * 1e6, 2),
                "step_minus_kernel_us": round(t_step * 1e6 - k_avg_ms * 1e3, 2),
                "note": "tiny_call_us: the same call on 2 elements (one launch of the same copy kernel, its completion "
                        "flag, the return), 2000 back to back; step_minus_kernel_us: ms_per_step minus the dominant "
                        "kernel's event-timed duration -- the blocking call's launch and completion round trip"},
            "roofline": roofline,
            "xgmi": xgmi,
            "rccl_compare": rccl,
            "cpu_baseline": cpu,
            "vs_cpu_baseline": round(npes * S / t_step / GIB / cpu["value"], 1) if cpu and cpu.get("value") else None,
            "vs_cpu_baseline_note": ("N = 1: both sides run the reference algorithm's 1-PE identity copy "
                                     "(reduce-op.c:226-229) -- one host core's memcpy against the GPU's HBM copy, "
                                     "so the ratio is a bandwidth ratio, not a reduction's; the combining "
                                     "comparison is cpu_baseline.eight_pe (config 3's shape on 8 host cores) beside "
                                     "an 8-GPU line" if npes == 1 else
                                     "the reference algorithm on %d host cores (one PE each) against %d GPUs"
                                     % (npes, npes)),
            "headline_rotating": rotating,
            "headline_offset_target": offset_target,
            "small_call": None if t_small is None else
            {"bytes_per_pe": small_n * 8, "us_per_call": round(t_small * 1e6, 2), "calls": small_calls,
             "schedule": small_info["schedule"], "kernel": small_info["kernel"], "check": small_check,
             "per_call": small_dist,
             "note": "BASELINE config 5 shape: 4096 back-to-back 64 KiB shmem_double_sum_to_all calls, max over PEs"},
            "small_call_persistent": small_p_child if world > 1 else None if t_small_p is None else
            {"bytes_per_pe": small_n * 8, "us_per_call": round(t_small_p * 1e6, 2), "calls": small_calls,
             "served": served1 - served0, "servers_launched": launched1 - launched0, "opt_in": True,
             "note": "the same calls with the opt-in persistent server (SHMEM_PERSISTENT): a resident kernel takes each "
                     "call from a host-coherent mailbox instead of a launch; the call ends when the host sees its "
                     "completion flag, as launched ones do (the timed region ends at the last call's return)"},
            "small_call_graph": small_graph,
            "coherence_selftest": coherence,
            "check": check,
            "target_sha256_pe0": check_sha,
            "xgmi_ceiling": xgmi_ceiling,
            "peer_fold_shapes": peer_shapes,
            "op_coverage": ops,
            "config1_call": config1_call,
            "external_buffers": external,
            "link_probe": link_probe,
            "kernels": kernels,
            "fused_same_gpu": fused,
            "fused_same_gpu_persistent": fused_p,
            "host_staged": host_staged,
            "threshold_sweep": threshold_sweep,
            "collectives": collectives,
        }
        for name, err in leg_errors.items():   # optional legs that raised
            out[name] = {"error": err}
        legs_s["total_before_print"] = round(time.perf_counter() - T_START, 2)
        out["legs_s"] = legs_s
        print(json.dumps(out), flush=True)
    if args.host:
        shm.free(dst)
        shm.free(src)
    else:
        shm.free_device(dst)
        shm.free_device(src)
    shm.finalize()


if __name__ == "__main__":
    main()
