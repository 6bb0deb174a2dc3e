#!/usr/bin/env python3
"""Per-call overhead of a 1-PE device-resident shmem_double_sum_to_all under
runtime knobs (tuning tool). Each variant runs in its own child process."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import os, sys, time
sys.path.insert(0, os.path.join(%r, "osss-gasnet_amd"))
import shmem_reduce
shm = shmem_reduce.Shmem(); shm.init()
res = []
for n in (1, 8192, 1 << 25):
    a, b = shm.malloc_device(8 * n), shm.malloc_device(8 * n)
    import numpy as np
    shm.put(a, np.random.default_rng(0).standard_normal(n)); shm.put(b, np.zeros(n))
    reps = 2000 if n < 100000 else 50
    for _ in range(50 if n < 100000 else 5):
        shm.to_all("sum", "double", b, a, n, 0, 0, 1)
    t0 = time.perf_counter()
    for _ in range(reps):
        shm.to_all("sum", "double", b, a, n, 0, 0, 1)
    res.append((time.perf_counter() - t0) / reps * 1e6)
    shm.free_device(b); shm.free_device(a)
print("n=1 %%.2f us | 64KiB %%.2f us | 256MiB %%.2f us" %% tuple(res))
shm.finalize()
''' % ROOT

for timing in ("0", "1"):
    env = dict(os.environ, SHMEM_DEVICE_HEAP_SIZE="600M", SHMEM_DEVICE_SCRATCH_SIZE="3M")
    child = CHILD.replace("shm.init()", "shm.init(); shm.kernel_timing(%s)" % timing)
    out = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=120)
    print(f"kernel_timing={timing}: {out.stdout.strip()} {out.stderr.strip()[-300:]}", flush=True)
