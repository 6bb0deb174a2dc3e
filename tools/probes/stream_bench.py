#!/usr/bin/env python3
"""Per-call time of shmem_double_sum_to_all through its three front ends, on
N PE processes sharing this box's GPU (measurement tool):

  host    shmem_double_sum_to_all: the host waits for every call
  stream  shmemx_double_sum_to_all_on_stream: CALLS calls enqueued back to
          back, one stream synchronize at the end
  graph   the same CALLS calls captured once into a HIP graph, replayed REPS
          times

usage: stream_bench.py [NPES ...]   (prints one JSON line per (npes, bytes))
"""
import json
import os
import subprocess
import sys
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import json, os, sys, time
sys.path.insert(0, os.path.join(%r, "osss-gasnet_amd"))
import numpy as np
import shmem_reduce
shm = shmem_reduce.Shmem(); shm.init()
me, np_ = shm.my_pe(), shm.n_pes()
CALLS, REPS = 200, 5
for nbytes in (64 << 10, 1 << 20, 16 << 20, 256 << 20):
    n = nbytes // 8
    a, b = shm.malloc_device(nbytes), shm.malloc_device(nbytes)
    shm.put(a, np.random.default_rng(me).standard_normal(n)); shm.put(b, np.zeros(n))
    calls = CALLS if nbytes <= (1 << 20) else 20
    res = {"npes": np_, "bytes": nbytes, "calls": calls}
    # host API
    for _ in range(5):
        shm.to_all("sum", "double", b, a, n, 0, 0, np_)
    shm.barrier_all()
    t0 = time.perf_counter()
    for _ in range(calls):
        shm.to_all("sum", "double", b, a, n, 0, 0, np_)
    res["host_us"] = (time.perf_counter() - t0) / calls * 1e6
    # stream API
    st = shm.stream_create()
    for _ in range(5):
        shm.to_all_on_stream("sum", "double", b, a, n, 0, 0, np_, st)
    shm.stream_sync(st); shm.barrier_all()
    t0 = time.perf_counter()
    for _ in range(calls):
        shm.to_all_on_stream("sum", "double", b, a, n, 0, 0, np_, st)
    t1 = time.perf_counter()
    shm.stream_sync(st)
    t2 = time.perf_counter()
    res["stream_us"] = (t2 - t0) / calls * 1e6
    res["stream_enqueue_us"] = (t1 - t0) / calls * 1e6
    # graph
    shm.barrier_all()
    shm.capture_begin(st)
    for _ in range(calls):
        shm.to_all_on_stream("sum", "double", b, a, n, 0, 0, np_, st)
    g, e = shm.capture_end(st)
    shm.graph_launch(e, st); shm.stream_sync(st); shm.barrier_all()
    t0 = time.perf_counter()
    for _ in range(REPS):
        shm.graph_launch(e, st)
    shm.stream_sync(st)
    res["graph_us"] = (time.perf_counter() - t0) / (REPS * calls) * 1e6
    shm.graph_destroy(g, e)
    shm.stream_destroy(st)
    # every PE holds the same bits
    got = shm.get(b, min(n, 4096), np.float64)
    res["check_sum"] = float(np.sum(got))
    if me == 0:
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
    shm.free_device(b); shm.free_device(a)
shm.finalize()
''' % ROOT


def run(npes):
    env = dict(os.environ, SHMEM_NPES=str(npes), SHMEM_JOB_ID=uuid.uuid4().hex[:12], SHMEM_DEVICE="0",
               SHMEM_DEVICE_HEAP_SIZE="1200M", SHMEM_DEVICE_SCRATCH_SIZE="3M")
    procs = [subprocess.Popen([sys.executable, "-c", CHILD], env=dict(env, SHMEM_PE=str(pe)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for pe in range(npes)]
    outs = [p.communicate(timeout=600)[0] for p in procs]
    for pe, (p, o) in enumerate(zip(procs, outs)):
        if p.returncode != 0:
            print(f"PE {pe} exited {p.returncode}:\n{o[-2000:]}", flush=True)
            sys.exit(1)
    print(outs[0].strip(), flush=True)


if __name__ == "__main__":
    for npes in [int(x) for x in sys.argv[1:]] or [1, 2, 4]:
        run(npes)
