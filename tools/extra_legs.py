#!/usr/bin/env python3
"""One PE of bench.py's child job for the N > 1 legs that have never run with
one GPU per PE (round 4): the headline call on plain hipMalloc buffers
(external_buffers: the peers map each other's allocations, csrc/extmap.c),
PE 0's one-peer-at-a-time shmem_getmem / shmem_putmem rates (link_probe;
putmem to another GPU is the HIP runtime's peer copy), and shmem_broadcast64 /
shmem_fcollect64 (collectives). They run here, in a job of their own (one
process per rank on the rank's GPU, started before the bench rank touches the
GPU), so that a failure in one of them -- a fatal error aborts a PE -- becomes
an "error" entry of the driver's line instead of taking the headline with it.

Round 6 adds the legs that only mean something with one GPU per PE, for the
same reason: the measured all-peers xGMI pull ceiling and the every-member
fold's launch shapes with N-1 remote sources (bench.py xgmi_legs; not
applicable when the PEs share a GPU, unless --force-xgmi-legs).

Run with SHMEM_PE / SHMEM_NPES / SHMEM_JOB_ID / SHMEM_DEVICE set; PE 0 prints
one JSON line {"external_buffers": ..., "link_probe": ..., "collectives": ...,
"xgmi_ceiling": ..., "peer_fold_shapes": ..., "config1_call": ...} (config 1's
2-PE 4 KiB int sum, tools/fused_bench.py config1, also new across GPUs).
usage: extra_legs.py MiB_per_PE steps algorithm [--no-check] [--no-external] [--no-link-probe] [--no-collectives]
       [--no-xgmi-legs] [--force-xgmi-legs] [--no-config1]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")]
import shmem_reduce  # noqa: E402
from bench import GIB, synth, xgmi_legs  # noqa: E402  (the same synthetic values as the bench rank's)


def main():
    S = int(sys.argv[1]) << 20
    steps = int(sys.argv[2])
    algorithm = sys.argv[3]
    flags = set(sys.argv[4:])
    check = "--no-check" not in flags
    n = S // 8
    # link_probe: 2 x 16 MiB, collectives: at most (1 + N) x 4 MiB; the xGMI
    # legs: source, target and the peer fold's staggered outputs (3 x S + a bit)
    xgmi = "--no-xgmi-legs" not in flags
    os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str((3 * S if xgmi else 0) + (128 << 20)))
    os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", str(96 << 20))
    shm = shmem_reduce.Shmem()
    shm.init()
    # the init self-test found peer heap reads broken: every call goes
    # through RCCL, so the external-buffer mapping is not what runs
    rccl_fallback = shm.n_pes() > 1 and shm.lib.shmemx_get_reduce_algorithm() == shmem_reduce.ALGORITHMS["rccl"] \
        and algorithm != "rccl"
    shm.set_algorithm(algorithm)
    me, npes = shm.my_pe(), shm.n_pes()
    # test hook (tests/test_gpu_bench.py): the PE dies as a fatal library
    # error would end it, after init -- bench.py must still print its line
    if os.environ.get("SHMEM_TEST_EXTRA_LEGS_ABORT") == "1":
        os.abort()
    loop = shmem_reduce.bench_loop()
    out = {}

    def max_over_pes(x):
        tbuf = np.array([x], dtype=np.float64)
        tout = np.zeros(1, dtype=np.float64)
        shm.to_all("max", "double", tout.ctypes.data, tbuf.ctypes.data, 1, 0, 0, npes)
        return float(tout[0])

    def guarded(name, fn):
        try:
            out[name] = fn()
        except Exception as e:  # noqa: BLE001 -- reported in the line
            out[name] = {"error": f"{type(e).__name__}: {e}"}

    def external():
        """the headline call on plain hipMalloc buffers outside the heap"""
        hip = ctypes.CDLL("libamdhip64.so")
        bufs = [ctypes.c_void_p(), ctypes.c_void_p()]
        if not all(hip.hipMalloc(ctypes.byref(b), ctypes.c_size_t(S)) == 0 for b in bufs):
            for b in bufs:
                if b.value:
                    hip.hipFree(b)
            return {"error": "hipMalloc of the two buffers failed"}
        esrc, edst = bufs[0].value, bufs[1].value
        shm.put(esrc, synth(me, np.arange(n, dtype=np.uint64)))
        k = max(5, steps // 4)
        loop(edst, esrc, n, 0, 0, npes, None, shm._psync_ptr, 3)
        shm.barrier_all()
        shm.sync()
        te0 = time.perf_counter()
        loop(edst, esrc, n, 0, 0, npes, None, shm._psync_ptr, k)
        shm.sync()
        t_loc = time.perf_counter() - te0
        info = shm.last_call_info()   # before max_over_pes: its own call replaces it
        t = max_over_pes(t_loc) / k
        ck = "skipped"
        if check:
            import oracle
            idx = np.unique(np.random.default_rng(50 + me).integers(0, n, 1 << 14)).astype(np.uint64)
            got = shm.get(edst, n, "double")[idx.astype(np.int64)]
            want = oracle.reduce_pe("sum", "double", [synth(p, idx) for p in range(npes)], me)
            bad = int(max_over_pes(int((got.view(np.uint64) != want.view(np.uint64)).sum())))
            ck = "bit-exact, %d samples" % len(idx) if bad == 0 else "MISMATCH %d samples" % bad
        shm.barrier_all()
        _, opened, _ = shm.external_map_stats()
        for b in bufs:
            hip.hipFree(b)
        return {"bytes_per_pe": S, "steps": k, "us_per_call": round(t * 1e6, 2),
                "value": round(npes * S / t / GIB, 2), "schedule": info["schedule"], "mappings_opened": opened,
                "fallbacks": shm.external_map_fallbacks(), "check": ck,
                "note": "the headline call on plain hipMalloc buffers (outside the symmetric heap): the members "
                        "map each other's allocations for the call (IPC, cached) instead of staging them through "
                        "scratch (SHMEM_EXTERNAL_MAP); measured in bench.py's child job (tools/extra_legs.py)"}

    def link_probe():
        """PE 0 alone, one peer at a time: getmem (copy kernel over the peer
        mapping) and putmem (HIP peer copy) of 16 MiB"""
        nbp, reps = min(S, 16 << 20), 10
        psym, ploc = shm.malloc_device(nbp), shm.malloc_device(nbp)
        if not psym or not ploc:
            raise RuntimeError("shmemx_malloc_device of 2 x %d bytes failed" % nbp)
        shm.put(psym, synth(me, np.arange(nbp // 8, dtype=np.uint64)))
        shm.barrier_all()
        get, put = shm.lib.shmem_getmem, shm.lib.shmem_putmem
        for f in (get, put):
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            f.restype = None
        peers, ok = {}, True
        if me == 0:
            for q in range(1, npes):
                rec = {}
                for name, f, a, b in (("get_GB_s", get, ploc, psym), ("put_GB_s", put, psym, ploc)):
                    f(a, b, nbp, q)
                    tq0 = time.perf_counter()
                    for _ in range(reps):
                        f(a, b, nbp, q)
                    shm.sync()
                    rec[name] = round(nbp * reps / (time.perf_counter() - tq0) / 1e9, 1)
                peers[str(q)] = rec
            if check:   # the last get brought PE npes-1's bytes
                got = shm.get(ploc, 1 << 16, "double").view(np.uint64)
                ok = bool((got == synth(npes - 1, np.arange(1 << 16, dtype=np.uint64)).view(np.uint64)).all())
        shm.barrier_all()
        shm.free_device(ploc)
        shm.free_device(psym)
        return {"bytes": nbp, "reps": reps, "from_pe0": peers,
                "check": "skipped" if not check else "bit-exact" if ok else "MISMATCH",
                "note": "PE 0 alone, one peer at a time: shmem_getmem (copy kernel pulling over the peer mapping) "
                        "and shmem_putmem (HIP peer copy) of 16 MiB, blocking calls"}

    def collectives():
        """shmem_broadcast64 (root PE 0) and shmem_fcollect64, 64 KiB and 4 MiB per PE"""
        vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        bc, fc = shm.lib.shmem_broadcast64, shm.lib.shmem_fcollect64
        bc.argtypes, bc.restype = [vp, vp, sz, ci, ci, ci, ci, vp], None
        fc.argtypes, fc.restype = [vp, vp, sz, ci, ci, ci, vp], None
        res, bad_total = {}, 0
        for nb in (64 << 10, 4 << 20):
            nw = nb // 8
            csrc, cdst = shm.malloc_device(nb), shm.malloc_device(npes * nb)
            if not csrc or not cdst:
                raise RuntimeError("shmemx_malloc_device for the collectives leg failed")
            shm.put(csrc, synth(me, np.arange(nw, dtype=np.uint64)).view(np.int64))
            rec = {}
            for name, call, moved in (
                    ("broadcast64", lambda: bc(cdst, csrc, nw, 0, 0, 0, npes, shm._psync_ptr), nb),
                    ("fcollect64", lambda: fc(cdst, csrc, nw, 0, 0, npes, shm._psync_ptr), npes * nb)):
                reps = 20
                call()
                shm.barrier_all()
                tq = time.perf_counter()
                for _ in range(reps):
                    call()
                shm.sync()
                t_loc = (time.perf_counter() - tq) / reps
                if name == "broadcast64":   # PE 0's target is not written (OpenSHMEM broadcast)
                    want = synth(0, np.arange(nw, dtype=np.uint64)).view(np.int64) if me != 0 else None
                    got = shm.get(cdst, nw, "longlong") if me != 0 else None
                else:
                    want = np.concatenate([synth(p, np.arange(nw, dtype=np.uint64)).view(np.int64)
                                           for p in range(npes)])
                    got = shm.get(cdst, npes * nw, "longlong")
                bad = 0 if (want is None or not check) else int((got != want).sum())
                bad_total += int(max_over_pes(bad))
                t = max_over_pes(t_loc)
                rec[name] = {"us_per_call": round(t * 1e6, 2), "GB_s_into_each_pe": round(moved / t / 1e9, 1)}
            res[str(nb)] = rec
            shm.barrier_all()
            shm.free_device(cdst)
            shm.free_device(csrc)
        res["check"] = "skipped" if not check else \
            "bit-exact on every PE" if bad_total == 0 else "MISMATCH in %d words" % bad_total
        res["note"] = ("shmem_broadcast64 (root PE 0) and shmem_fcollect64 over the whole job, 20 blocking calls "
                       "per size, max over PEs; GB/s = bytes landing in each PE's target / time")
        return res

    if "--no-external" not in flags and not rccl_fallback:
        guarded("external_buffers", external)
    if "--no-link-probe" not in flags:
        guarded("link_probe", link_probe)
    if "--no-collectives" not in flags:
        guarded("collectives", collectives)
    if xgmi and not rccl_fallback:
        src, dst = shm.malloc_device(S), shm.malloc_device(S)
        if not src or not dst:
            out["xgmi_ceiling"] = out["peer_fold_shapes"] = {"error": "shmemx_malloc_device of 2 x S failed"}
        else:
            shm.put(src, synth(me, np.arange(n, dtype=np.uint64)))
            shm.barrier_all()
            try:
                out.update(xgmi_legs(shm, S, me, npes, src, dst, "--force-xgmi-legs" in flags, max_over_pes))
            except Exception as e:  # noqa: BLE001 -- reported in the line
                out["xgmi_ceiling"] = out["peer_fold_shapes"] = {"error": f"{type(e).__name__}: {e}"}
            shm.free_device(dst)
            shm.free_device(src)
    elif xgmi:
        out["xgmi_ceiling"] = out["peer_fold_shapes"] = {
            "not_applicable": "peer heap reads failed the init self-test (RCCL fallback)"}
    if "--no-config1" not in flags:   # BASELINE config 1's call on PEs 0 and 1 (tools/fused_bench.py)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import fused_bench
        guarded("config1_call", lambda: fused_bench.config1(shm, 4096, max_over_pes))
    shm.barrier_all()
    if me == 0:
        print(json.dumps(out), flush=True)
    shm.finalize()


if __name__ == "__main__":
    main()
