#!/usr/bin/env python3
"""One PE of the persistent-server tests (tests/test_gpu_persistent.py): runs a
scripted sequence of blocking reductions with SHMEM_PERSISTENT=1 and checks
every result against the oracle's result for this PE (the reference's order:
own source first, reduce-op.c:226-264). Every PE runs the same script (the
parameters come from a seed shared by all PEs, the data from seed + PE).

usage: persistent_worker.py SCRIPT SEED   (identity from SHMEM_PE / SHMEM_NPES)
  SCRIPT: burst | mixed | idle | race | orderflip | ordered
Prints one JSON line (calls checked, calls served by a resident server,
servers launched); exits 1 on the first mismatch.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import oracle  # noqa: E402
import shmem_reduce  # noqa: E402
from _compare import assert_match  # noqa: E402
from _inputs import source  # noqa: E402

script, seed = sys.argv[1], int(sys.argv[2])
shm = shmem_reduce.Shmem()
shm.init()
me, npes = shm.my_pe(), shm.n_pes()
assert shm.set_persistent(True) is True, "SHMEM_PERSISTENT=1 should have enabled it at init"
CAP = 8 << 20  # bytes per buffer
src_buf, dst_buf = shm.malloc_device(CAP), shm.malloc_device(CAP)
prng = np.random.default_rng(seed)  # the same on every PE
checked = 0
ncall = 0


def batch(op, dtype, calls, nmax, inplace_every=4, gap=None):
    """`calls` reductions run back to back (the server's use: no other HIP
    work between them; a hipMemcpy from pageable memory waits for a resident
    server to leave), each in a region of its own, the sources written
    before and the targets checked after. gap(): seconds to spin between two
    calls, or None."""
    global checked, ncall
    es = np.dtype(oracle.NP[dtype]).itemsize
    region = (nmax * es + 1024 + 4095) // 4096 * 4096
    assert calls * region <= CAP
    plan = []
    for k in range(calls):
        n = int(prng.integers(1, nmax + 1))
        soff = k * region + 16 * int(prng.integers(0, 64))
        inplace = inplace_every and k % inplace_every == inplace_every - 1
        doff = soff if inplace else k * region + 16 * int(prng.integers(0, 64))
        xs = [source(op, dtype, n, seed * 7919 + ncall + k, p) for p in range(npes)]
        shm.put(src_buf + soff, xs[me])
        plan.append((n, soff, doff, inplace, xs))
    ncall += calls
    shm.barrier_all()
    for n, soff, doff, inplace, xs in plan:
        s = src_buf + soff
        shm.to_all(op, dtype, s if inplace else dst_buf + doff, s, n, 0, 0, npes)
        if gap is not None:
            t_end = time.perf_counter() + gap()
            while time.perf_counter() < t_end:
                pass
    for k, (n, soff, doff, inplace, xs) in enumerate(plan):
        got = shm.get((src_buf + soff) if inplace else dst_buf + doff, n, dtype)
        assert_match(got, oracle.reduce_pe(op, dtype, xs, me), op, dtype,
                     f"PE {me} call {k} of a batch (n {n}, in place {bool(inplace)})")
        checked += 1


if script == "burst":
    # one (op, type) at a time: one-shot and two-shot sizes, in place or not,
    # varying offsets; ordered pairs (double sum from 3 PEs, float max) among them
    batch("sum", "double", 60, 8192)
    batch("max", "float", 40, 4096)
    batch("sum", "int", 40, 16384)
    batch("prod", "complexd", 20, 2048)
    batch("min", "longdouble", 12, 1024)
    batch("xor", "short", 20, 30000)
elif script == "mixed":
    # batches interrupted by operations that must stop the server: a larger
    # call (multi-launch schedule with device barriers), a different
    # (op, type), a broadcast, then a barrier and shmemx_device_synchronize
    L = shm.lib
    L.shmem_broadcast64.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_int] * 4 + [
        ctypes.c_void_p]
    for rnd in range(3):
        batch("sum", "double", 12, 4096)
        xs = [source("sum", "double", 131072, seed + rnd, p) for p in range(npes)]
        shm.put(src_buf + (CAP >> 1), xs[me])  # beyond the batches' regions
        shm.barrier_all()
        batch("sum", "double", 6, 4096)
        shm.to_all("sum", "double", dst_buf + (CAP >> 1), src_buf + (CAP >> 1), 131072, 0, 0, npes)  # 1 MiB
        assert_match(shm.get(dst_buf + (CAP >> 1), 131072, "double"), oracle.reduce_pe("sum", "double", xs, me),
                     "sum", "double", f"PE {me} large call")
        checked += 1
        batch("sum", "double", 6, 4096)
        batch("and", "long", 6, 4096)
        bsrc = np.arange(64, dtype=np.int64) * (me + 1)
        shm.put(src_buf + (CAP >> 1), bsrc)
        shm.barrier_all()
        L.shmem_broadcast64(dst_buf + (CAP >> 1), src_buf + (CAP >> 1), 64, 0, 0, 0, npes, shm._psync_ptr)
        if me != 0:
            b = shm.get(dst_buf + (CAP >> 1), 64, "long")
            assert (b == np.arange(64, dtype=np.int64)).all(), f"broadcast mismatch on PE {me}"
        batch("sum", "double", 6, 4096)
        # a stream-ordered reduction (its own spin-waiting kernel) while a server is resident
        xs = [source("max", "float", 3000, seed + 10 + rnd, p) for p in range(npes)]
        shm.put(src_buf + (CAP >> 1), xs[me])
        batch("sum", "double", 4, 4096)
        st = shm.stream_create()
        shm.to_all_on_stream("max", "float", dst_buf + (CAP >> 1), src_buf + (CAP >> 1), 3000, 0, 0, npes, st)
        shm.stream_sync(st)
        shm.stream_destroy(st)
        assert_match(shm.get(dst_buf + (CAP >> 1), 3000, "float"), oracle.reduce_pe("max", "float", xs, me), "max",
                     "float", f"PE {me} stream-ordered call")
        checked += 1
        batch("sum", "double", 4, 4096)
        shm.sync()
elif script == "idle":
    # gaps longer than the server's idle time: it leaves between calls, and
    # a call rung at that moment falls back to a launch
    idle = float(os.environ.get("SHMEM_PERSISTENT_IDLE_US", "1000")) * 1e-6
    for k in range(6):
        batch("sum", "double", 15, 4096, gap=lambda: idle * (0.5 + 2.0 * prng.random()))
elif script == "race":
    # gaps spread around the idle time: the server leaves just before or
    # after a call is rung
    idle = float(os.environ.get("SHMEM_PERSISTENT_IDLE_US", "1000")) * 1e-6
    for k in range(10):
        batch("sum", "double", 40, 2048, gap=lambda: idle * 2.0 * prng.random())
elif script == "orderflip":
    # the result order switched INSIDE a burst, with no other GPU work between
    # the calls (a resident server keeps the order it was started with: every
    # member of a float max must switch together, and shmemx_set_reduce_order
    # stops the server so the next call starts one with the new order)
    op, dtype, n = "max", "float", 3000
    for rnd in range(4):
        k = 8
        xs = [[source(op, dtype, n, seed * 31 + rnd * 97 + c, p) for p in range(npes)] for c in range(2 * k)]
        for c in range(2 * k):
            shm.put(src_buf + c * 16384, xs[c][me])
        shm.barrier_all()
        first = "reference" if rnd % 2 == 0 else "pe_start"
        second = "pe_start" if first == "reference" else "reference"
        shm.set_order(first)
        for c in range(k):
            shm.to_all(op, dtype, dst_buf + c * 16384, src_buf + c * 16384, n, 0, 0, npes)
        shm.set_order(second)
        for c in range(k, 2 * k):
            shm.to_all(op, dtype, dst_buf + c * 16384, src_buf + c * 16384, n, 0, 0, npes)
        shm.set_order("reference")
        for c in range(2 * k):
            who = me if (first if c < k else second) == "reference" else 0
            assert_match(shm.get(dst_buf + c * 16384, n, dtype), oracle.reduce_pe(op, dtype, xs[c], who), op, dtype,
                         f"PE {me} round {rnd} call {c} ({first} then {second})")
            checked += 1
elif script == "ordered":
    # the documented contract: GPU work the caller queued on the null stream
    # (a 30 ms kernel, then a device-to-device copy of new data into the
    # source) is completed by the caller before the call; that wait returns
    # once a resident server idles out, and the call sees the new data
    L = shm.lib
    busy = ctypes.CDLL(os.path.join(ROOT, "osss-gasnet_amd", "lib", "libtestbusy.so"))
    busy.test_busy_launch.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
    L.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    n = 4096
    for rnd in range(4):
        xa = [source("sum", "double", n, seed + 2 * rnd, p) for p in range(npes)]
        xb = [source("sum", "double", n, seed + 2 * rnd + 1, p) for p in range(npes)]
        shm.put(src_buf, xa[me])
        shm.put(src_buf + (CAP >> 1), xb[me])  # the new data, elsewhere in the heap
        shm.barrier_all()
        for k in range(6):  # a burst: the server is resident after the second call
            shm.to_all("sum", "double", dst_buf, src_buf, n, 0, 0, npes)
        assert busy.test_busy_launch(30.0, 1, None) == 0
        assert L.hipMemcpyAsync(src_buf, src_buf + (CAP >> 1), n * 8, 3, None) == 0  # hipMemcpyDeviceToDevice
        assert L.hipStreamSynchronize(None) == 0
        shm.to_all("sum", "double", dst_buf, src_buf, n, 0, 0, npes)
        assert_match(shm.get(dst_buf, n, "double"), oracle.reduce_pe("sum", "double", xb, me), "sum", "double",
                     f"PE {me} round {rnd}: the call after queued null-stream work")
        checked += 1
else:
    raise SystemExit(f"unknown script {script}")

served, launched = shm.persistent_stats()
shm.barrier_all()
print(json.dumps({"pe": me, "checked": checked, "served": served, "launched": launched}), flush=True)
shm.free_device(dst_buf)
shm.free_device(src_buf)
shm.finalize()
