#!/usr/bin/env python3
"""One PE of a multi-PE GPU test: runs every case of a spec through the public
shmem_<T>_<op>_to_all entry points and saves what its target holds afterwards.

usage: pe_worker.py SPEC.json OUTDIR   (identity from SHMEM_PE / SHMEM_NPES)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import shmem_reduce  # noqa: E402
from _inputs import source  # noqa: E402


def members(start, logstride, size):
    return [start + i * (1 << logstride) for i in range(size)]


def dm_source(c, pe):
    """Source block of PE pe for a data-movement case (collect: length varies by PE)."""
    import _inputs
    bits = c["bits"]
    n = c["n"] if c["kind"] != "collect" else ((c["n"] + pe) % 4) * 37
    rng = np.random.default_rng(c["seed"] * 1009 + pe)
    return rng.integers(-2**(bits - 1), 2**(bits - 1), n, dtype=np.int32 if bits == 32 else np.int64)


def run_datamove(shm, c, me, da, db, ha, hb, results):
    import ctypes
    kind, bits = c["kind"], c["bits"]
    dt = np.int32 if bits == 32 else np.int64
    es = bits // 8
    s = None
    for cand in c["sets"]:
        if me in members(*cand):
            s = cand
    if s is None:
        return
    start, logstride, size = s
    mem = members(*s)
    x = dm_source(c, me)
    kind_t = c.get("target", "device")
    if kind_t == "mixed":  # pageable host target on odd PEs, device on even ones
        kind_t = "pageable" if me % 2 else "device"
    tgt_host = kind_t in ("host", "pageable")
    cap = c["cap"]
    pageable = np.empty(cap * 8 + 64, dtype=np.uint8)  # plain malloc'd numpy memory
    tgt = hb if kind_t == "host" else pageable.ctypes.data + 8 if kind_t == "pageable" else db
    sentinel = np.full(cap, -7, dtype=dt)
    if tgt_host:
        ctypes.memmove(tgt, sentinel.ctypes.data, sentinel.nbytes)
    else:
        shm.put(tgt, sentinel)
    # "source": "host" -- the symmetric objects in shmem_malloc's host heap
    # (every PE's segment mapped by every PE, csrc/hostheap.c) instead of the
    # device heap: the collectives' sources, put targets and get sources
    sym_host = c.get("source") == "host"
    sa = ha if sym_host else da
    if len(x):
        if sym_host:
            ctypes.memmove(ha, x.ctypes.data, x.nbytes)
        else:
            shm.put(da, x)
    psync = shm._psync_ptr
    L = shm.lib
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    if kind == "broadcast":
        f = getattr(L, f"shmem_broadcast{bits}")
        f.argtypes = [vp, vp, sz, i, i, i, i, vp]
        f(tgt, sa, c["n"], c["root"], start, logstride, size, psync)
    elif kind in ("fcollect", "collect"):
        f = getattr(L, f"shmem_{kind}{bits}")
        f.argtypes = [vp, vp, sz, i, i, i, vp]
        f(tgt, sa, len(x), start, logstride, size, psync)
    elif kind == "putget":
        # put my block into the next member's target at my slot, barrier, then
        # get the previous member's block from its source
        nxt, prv = mem[(mem.index(me) + 1) % size], mem[(mem.index(me) - 1) % size]
        if sym_host:
            ctypes.memmove(hb, sentinel.ctypes.data, sentinel.nbytes)
        L.shmem_barrier(start, logstride, size, psync)  # every target holds its sentinel
        f = getattr(L, f"shmem_put{bits}")
        f.argtypes = [vp, vp, sz, i]
        g = getattr(L, f"shmem_get{bits}")
        g.argtypes = [vp, vp, sz, i]
        src = ha if sym_host else da     # the local side holding x by default
        if c.get("put_from") == "host":  # page-locked shmem_malloc source
            ctypes.memmove(ha, x.ctypes.data, x.nbytes)
            src = ha
        elif c.get("put_from") == "pageable":
            keep = np.ascontiguousarray(x)
            src = keep.ctypes.data
        elif c.get("put_from") == "device":
            src = da
        # symmetric target of the put: the device heap's db, or (host heap) the
        # slot array hb; the get's symmetric source is sa, its local target
        # the other array
        symt = hb if sym_host else db
        if sym_host and c.get("put_from") == "device":
            shm.put(da, x)
        f(symt + mem.index(me) * c["n"] * es, src, c["n"], nxt)
        L.shmem_barrier(start, logstride, size, psync)
        if sym_host:   # local side of the get: device memory unless target=host (then plain numpy)
            keep_get = np.zeros(c["n"], dtype=dt)
            gdst = keep_get.ctypes.data if c.get("target") == "host" else db
        else:
            gdst = hb if tgt_host else db + size * c["n"] * es
        g(gdst, sa, c["n"], prv)
        L.shmem_barrier(start, logstride, size, psync)
        if sym_host and c.get("target") == "host":
            got2 = keep_get.copy()
        elif sym_host or not tgt_host:
            got2 = shm.get(gdst, c["n"], dt)
        else:
            got2 = np.empty(c["n"], dtype=dt)
            ctypes.memmove(got2.ctypes.data, hb, got2.nbytes)
        results[str(c["id"]) + "_get"] = got2
        if sym_host:   # the put slots, read locally from this PE's host heap
            got = np.empty(cap, dtype=dt)
            ctypes.memmove(got.ctypes.data, hb, got.nbytes)
            results[str(c["id"])] = got
            return
        tgt_host = False
        tgt = db
    if tgt_host:
        got = np.empty(cap, dtype=dt)
        ctypes.memmove(got.ctypes.data, tgt, got.nbytes)
    else:
        got = shm.get(tgt, cap, dt)
    results[str(c["id"])] = got


def run_stream(shm, c, me, da, db, results):
    """kind "stream": a chain of `chain` stream-ordered reductions on one HIP
    stream, buf[i+1] <- reduce(buf[i]), enqueued back to back with no host
    wait; or (graph > 0) the same chain captured once into a HIP graph and
    replayed `graph` times with a fresh input each time."""
    op, dtype, n, k = c["op"], c["dtype"], c["n"], c["chain"]
    es = np.dtype(shmem_reduce.NP[dtype]).itemsize
    off = c.get("offset", 0)                      # elements off 16-byte alignment
    stride = ((n + off) * es + 255) // 256 * 256 + 256
    base = shm.malloc_device(stride * (k + 1))    # collective: every PE allocates
    mine = None
    for s in c["sets"]:
        if me in members(*s):
            mine = s
    if mine is not None:
        shm.set_order(c.get("order", "reference"))
        bufs = [base + i * stride + off * es for i in range(k + 1)]
        st = shm.stream_create()

        def enqueue():
            for i in range(k):
                shm.to_all_on_stream(op, dtype, bufs[i + 1], bufs[i], n, *mine, st)
                if c.get("barriers"):
                    shm.barrier_on_stream(*mine, st)

        replays = c.get("graph", 0)
        if replays:
            shm.capture_begin(st)
            enqueue()
            graph, exe = shm.capture_end(st)
            for r in range(replays):
                if n:
                    shm.put(bufs[0], source(op, dtype, n, c["seed"] + r, me))
                shm.graph_launch(exe, st)
                shm.stream_sync(st)
                results[f"{c['id']}_r{r}"] = shm.get(bufs[k], n, dtype)
            shm.graph_destroy(graph, exe)
        else:
            if n:
                shm.put(bufs[0], source(op, dtype, n, c["seed"], me))
                if c.get("mixed"):
                    shm.put(da, source(op, dtype, n, c["seed"] + 1, me))
            enqueue()
            if c.get("mixed"):
                # a host-side call while the stream chain is in flight
                shm.to_all(op, dtype, db, da, n, *mine)
                results[f"{c['id']}_host"] = shm.get(db, n, dtype)
            shm.stream_sync(st)
            for i in range(1, k + 1):
                results[f"{c['id']}_{i}"] = shm.get(bufs[i], n, dtype)
        shm.stream_destroy(st)
    shm.free_device(base)


def run_config(shm, c, me, results):
    """kind "config": a BASELINE.json config at its full size with SURVEY
    §8(d)'s inputs (tests/_configs.py); saves digests, not whole arrays.
    c5: `calls` back-to-back calls cycling over `slots` source/target pairs."""
    import _configs
    op, dtype = _configs.CONFIGS[c["config"]]
    n, slots, calls = c["n"], c.get("slots", 1), c.get("calls", 1)
    es = np.dtype(shmem_reduce.NP[dtype]).itemsize
    stride = (n * es + 255) // 256 * 256
    src, dst = shm.malloc_device(stride * slots), shm.malloc_device(stride * slots)
    for k in range(slots):
        shm.put(src + k * stride, _configs.source(c["config"], n, me, k))
    shm.barrier_all()
    for j in range(calls):
        k = j % slots
        shm.to_all(op, dtype, dst + k * stride, src + k * stride, n, 0, 0, shm.n_pes())
    for k in range(slots):
        h, sample = _configs.digest(shm.get(dst + k * stride, n, dtype))
        results[f"{c['id']}_{k}_sha"] = np.frombuffer(bytes.fromhex(h), dtype=np.uint8)
        results[f"{c['id']}_{k}_sample"] = sample
    shm.free_device(dst)
    shm.free_device(src)


def big_source(c, pe):
    """Inputs of a "big" case, cheap to generate at GiB sizes: config 1's
    int pattern for integers; for floats random values with NaN / +0 / -0
    planted on some PEs (the selects of min/max then depend on the order)."""
    n, dtype = c["n"], c["dtype"]
    if dtype in ("short", "int", "long", "longlong"):
        i = np.arange(n, dtype=np.int64)
        return (i * 7 + pe * 1000003).astype(shmem_reduce.NP[dtype])
    x = np.random.default_rng(c["seed"] + pe).random(n, dtype=np.float32).astype(shmem_reduce.NP[dtype]) - 0.5
    x[pe::97 + pe] = np.nan if pe % 2 == 0 else 0.0
    x[3::89] = -0.0 if pe % 2 else 0.0
    return x


def run_big(shm, c, me, results):
    """kind "big": one reduction of c["n"] elements (GiB-scale, up to nreduce =
    INT_MAX) on device-heap buffers allocated for it; checked here, on every
    PE: the whole target at one PE (the identity), else a million sampled
    elements against the oracle's result for this PE."""
    import oracle
    op, dtype, n = c["op"], c["dtype"], c["n"]
    es = np.dtype(shmem_reduce.NP[dtype]).itemsize
    start, logstride, size = c["sets"][0]
    src, dst = shm.malloc_device(n * es), shm.malloc_device(n * es)
    x = big_source(c, me)
    shm.put(src, x)
    shm.to_all(op, dtype, dst, src, n, start, logstride, size)
    got = shm.get(dst, n, dtype)
    if size == 1:
        bad = int((got.view(np.uint8) != x.view(np.uint8)).sum())
    else:
        idx = np.unique(np.random.default_rng(7).integers(0, n, 1 << 20))
        idx = np.concatenate([idx, [0, n - 1]])
        srcs = [big_source(c, p)[idx] for p in range(size)]
        want = oracle.reduce_pe(op, dtype, srcs, me)
        bad = int((got[idx].view(np.uint8) != want.view(np.uint8)).sum())
    results[str(c["id"]) + "_bad"] = np.array([bad])
    shm.free_device(dst)
    shm.free_device(src)


FORTRAN_KIND = {"short": "int2", "int": "int4", "long": "int8", "float": "real4", "double": "real8",
                "longdouble": "real16", "complexf": "comp4", "complexd": "comp8"}


def fortran_to_all(shm, op, dtype, dst, src, n, start, logstride, size):
    """The Fortran binding (csrc/fortran.c): every argument by reference and an
    INTEGER (4-byte) pSync, as a Fortran program passes them."""
    import ctypes
    f = getattr(shm.lib, f"shmem_{FORTRAN_KIND[dtype]}_{op}_to_all_")
    f.restype = None
    psync = np.full(shmem_reduce.SHMEM_REDUCE_SYNC_SIZE, -1, dtype=np.int32)
    ints = [ctypes.c_int(v) for v in (n, start, logstride, size)]
    f(ctypes.c_void_p(dst), ctypes.c_void_p(src), *[ctypes.byref(v) for v in ints], None,
      ctypes.c_void_p(psync.ctypes.data))
    assert (psync == -1).all(), "pSync modified"


def main():
    import ctypes
    spec = json.load(open(sys.argv[1]))
    outdir = sys.argv[2]
    shm = shmem_reduce.Shmem()
    shm.init()
    me = shm.my_pe()
    maxb = max(max(c["n"] + 16, c.get("cap", 0)) * 16 if c.get("kind") not in ("config", "big") else 4096
               for c in spec["cases"])
    da, db = shm.malloc_device(maxb), shm.malloc_device(maxb)
    ha, hb = shm.malloc(maxb), shm.malloc(maxb)
    hip = ctypes.CDLL("libamdhip64.so")
    pa, pb = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(pa), ctypes.c_size_t(maxb + 4096)) == 0
    assert hip.hipMalloc(ctypes.byref(pb), ctypes.c_size_t(maxb + 4096)) == 0
    priv_a, priv_b = pa.value, pb.value
    results = {}
    fds_start = len(os.listdir("/proc/self/fd"))
    for c in spec["cases"]:
        if c.get("kind") == "config":
            run_config(shm, c, me, results)
            continue
        if c.get("kind") == "big":
            run_big(shm, c, me, results)
            continue
        if c.get("kind") == "stream":
            run_stream(shm, c, me, da, db, results)
            continue
        if c.get("kind", "reduce") != "reduce":
            run_datamove(shm, c, me, da, db, ha, hb, results)
            continue
        mine = None
        for s in c["sets"]:
            if me in members(*s):
                mine = s
        if mine is None:
            continue
        op, dtype, n = c["op"], c["dtype"], c["n"]
        es = np.dtype(shmem_reduce.NP[dtype]).itemsize
        if "golden" in c:  # the committed fixture's inputs (tests/golden/), member i's row
            fam = c.get("family", "")   # "nan_": the NaN-payload families
            g = np.load(os.path.join(HERE, "golden", f"golden_{fam}{op}_{dtype}.npz"))
            x = np.ascontiguousarray(g[f"in_{c['golden']}"][members(*mine).index(me)])
        else:
            x = source(op, dtype, n, c["seed"], me)
        mode = c["mode"]
        if mode == "dev":
            src, dst = da, db
        elif mode == "inplace":
            src = dst = da
        elif mode == "overlap_up":       # target 5 elements above source
            src, dst = da, da + 5 * es
        elif mode == "overlap_down":     # target 5 elements below source
            src, dst = da + 5 * es, da
        elif mode == "host":
            src, dst = ha, hb
        elif mode in ("devother", "devother_mixed"):
            # plain hipMalloc buffers (outside the symmetric heap, like a
            # framework's tensors); _mixed: odd PEs pass page-locked host
            # arrays instead (both kinds are staged through the scratch)
            if mode == "devother" or me % 2 == 0:
                src, dst = priv_a, priv_b
            else:
                src, dst = ha, hb
        elif mode == "host_overlap_up":      # page-locked host arrays, target 5 elements above source
            src, dst = ha, ha + 5 * es
        elif mode == "host_overlap_down":    # target 5 elements below source
            src, dst = ha + 5 * es, ha
        elif mode == "devother_overlap_up":  # hipMalloc buffer, target 5 elements above source
            src, dst = priv_a, priv_a + 5 * es
        elif mode == "devother_overlap_down":
            src, dst = priv_a + 5 * es, priv_a
        elif mode == "mixed_heapdst_hostsrc":   # target in the device heap, source a host array
            src, dst = ha, db
        elif mode == "mixed_hostdst_heapsrc":   # target a host array, source in the device heap
            src, dst = da, hb
        elif mode == "mixed_hostdst_devsrc":    # target a host array, source a hipMalloc buffer
            src, dst = priv_a, hb
        elif mode == "devmap_inplace":   # one hipMalloc buffer, target == source
            src = dst = priv_a
        elif mode == "devmap_offset":    # each PE's buffers at other offsets into its allocations
            src, dst = priv_a + 64 * (me + 1), priv_b + 32 * me
        elif mode == "devmap_symtarget":  # target in the symmetric heap, source a hipMalloc buffer
            src, dst = priv_a, db
        elif mode == "devmap_unaligned_pe1":  # PE 1's pair 8 bytes off 16-byte alignment: every PE stages
            src, dst = (priv_a + 8, priv_b + 8) if me == 1 else (priv_a, priv_b)
        elif mode == "devmap_realloc":   # fresh allocations before the call (the peers' cached mappings go stale)
            hip.hipFree(pa)
            hip.hipFree(pb)
            keep = ctypes.c_void_p()   # so the new ones need not land on the old addresses
            assert hip.hipMalloc(ctypes.byref(keep), ctypes.c_size_t(4096 * (1 + c["id"] % 3))) == 0
            assert hip.hipMalloc(ctypes.byref(pa), ctypes.c_size_t(maxb + 4096)) == 0
            assert hip.hipMalloc(ctypes.byref(pb), ctypes.c_size_t(maxb + 4096)) == 0
            hip.hipFree(keep)
            priv_a, priv_b = pa.value, pb.value
            src, dst = priv_a, priv_b
        elif mode == "host_mixed":
            # even PEs: page-locked shmem_malloc arrays (one-launch in-kernel
            # staging for small n); odd PEs: plain numpy arrays (staged copies)
            if me % 2 == 0:
                src, dst = ha, hb
            else:
                np_src = np.zeros(max(n, 1), dtype=shmem_reduce.NP[dtype])
                np_dst = np.zeros(max(n, 1), dtype=shmem_reduce.NP[dtype])
                src, dst = np_src.ctypes.data, np_dst.ctypes.data
        elif mode == "unaligned":        # device, both one element off 16-byte alignment
            src, dst = da + es, db + es
        else:
            raise ValueError(mode)
        host_src = mode.startswith("host") or mode == "mixed_heapdst_hostsrc"
        host_dst = mode.startswith("host") or mode in ("mixed_hostdst_heapsrc", "mixed_hostdst_devsrc")
        if n:
            if host_src:
                ctypes.memmove(src, x.ctypes.data, x.nbytes)
            else:
                shm.put(src, x)
        shm.set_algorithm(c.get("algorithm", "auto"))
        shm.set_order(c.get("order", "reference"))
        busy_t0 = None
        if c.get("busy_ms") and me == 0:
            # another kernel holds every CU of the GPU while this PE enters the
            # collective (tests/native/busy_kernel.hip, its own non-blocking stream)
            import time
            busy = ctypes.CDLL(os.path.join(ROOT, "osss-gasnet_amd", "lib", "libtestbusy.so"))
            busy.test_busy_launch.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
            st = ctypes.c_void_p()
            assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
            shm.barrier_all()
            assert busy.test_busy_launch(float(c["busy_ms"]), 8, st) == 0
            busy_t0 = time.perf_counter()
        elif c.get("busy_ms"):
            shm.barrier_all()
        if c.get("api") == "fortran":
            fortran_to_all(shm, op, dtype, dst, src, n, *mine)
        else:
            shm.to_all(op, dtype, dst, src, n, *mine)
        if busy_t0 is not None:
            import time
            results[str(c["id"]) + "_seconds"] = np.array([time.perf_counter() - busy_t0])
            assert hip.hipStreamSynchronize(st) == 0
            hip.hipStreamDestroy(st)
        if host_dst:
            out = np.empty(n, dtype=shmem_reduce.NP[dtype])
            if n:
                ctypes.memmove(out.ctypes.data, dst, out.nbytes)
            results[str(c["id"])] = out
        else:
            results[str(c["id"])] = shm.get(dst, n, dtype) if n else np.zeros(0, dtype=shmem_reduce.NP[dtype])
        if n and c.get("api") != "fortran":
            results[str(c["id"]) + "_schedule"] = np.array([shm.last_call_info()["schedule"]])
    results["external_map_stats"] = np.array(shm.external_map_stats())
    results["external_map_fallbacks"] = np.array([shm.external_map_fallbacks()])
    results["fd_count"] = np.array([fds_start, len(os.listdir("/proc/self/fd"))])
    hip.hipFree(pa)
    hip.hipFree(pb)
    shm.free(hb)
    shm.free(ha)
    shm.free_device(db)
    shm.free_device(da)
    shm.finalize()
    np.savez(os.path.join(outdir, f"pe{me}.npz"), **results)


if __name__ == "__main__":
    main()
