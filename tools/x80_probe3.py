#!/usr/bin/env python3
"""Debug tool for x80.h: test_longdouble_random_encodings' exact steps
(hipMalloc'd buffers through the test's allocator, ops sum, prod, min, max),
repeated, printing every mismatch's bits."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
import shmem_reduce  # noqa: E402

os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", "1600M")
os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
shm = shmem_reduce.Shmem()
shm.init()
from test_gpu_combine import Dev, gpu_fold  # noqa: E402
dev = Dev(shm)

rng = np.random.default_rng(99)
n = 200000
raw = np.zeros((3, n, 16), dtype=np.uint8)
for k in range(3):
    m = rng.integers(0, 2**64, n, dtype=np.uint64, endpoint=False)
    se = rng.integers(0, 2**16, n, dtype=np.uint16)
    near = rng.random(n) < 0.5
    se[near] = (se[near] & 0x8000) | (16383 + rng.integers(-70, 70, int(near.sum()))).astype(np.uint16)
    m[near] |= np.uint64(1 << 63)
    raw[k, :, 0:8] = m.view(np.uint8).reshape(n, 8)
    raw[k, :, 8:10] = se.view(np.uint8).reshape(n, 2)
srcs = [raw[k].view(np.longdouble).reshape(n) for k in range(3)]


def vb(a):
    return np.ascontiguousarray(a).view(np.uint8).reshape(len(a), 16)[:, :10]


for rep in range(20):
    for op in ("sum", "prod", "min", "max"):
        got = gpu_fold(shm, dev, op, "longdouble", srcs)
        want = oracle.reduce_pe(op, "longdouble", srcs, 0)
        bad = np.nonzero((vb(got) != vb(want)).any(axis=1))[0]
        if len(bad):
            print("rep", rep, op, len(bad), "mismatches")
            for i in bad[:4]:
                print("  i", i, "ops", [vb(s[i:i + 1])[0][::-1].tobytes().hex() for s in srcs],
                      "gpu", vb(got[i:i + 1])[0][::-1].tobytes().hex(), "host", vb(want[i:i + 1])[0][::-1].tobytes().hex())
        dev.free()
print("done")
shm.finalize()
