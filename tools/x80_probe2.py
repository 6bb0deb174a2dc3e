#!/usr/bin/env python3
"""Debug tool for x80.h: test_longdouble_random_encodings' data folded on the
GPU (prod of 3 sources), mismatches against the host x87, then the wave
(64 elements) around the first mismatch alone, and that element alone."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
import shmem_reduce  # noqa: E402

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
os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", "64M")
shm = shmem_reduce.Shmem()
shm.init()
bufs = [shm.malloc_device(n * 16 + 4096) for _ in range(4)]


def vb(a):
    return np.ascontiguousarray(a).view(np.uint8).reshape(len(a), 16)[:, :10]


def fold(op, ss):
    for b, s in zip(bufs, ss):
        shm.put(b, s)
    assert shm.combine(op, "longdouble", bufs[3], bufs[:len(ss)], len(ss[0])) == 0
    shm.sync()
    got = shm.get(bufs[3], len(ss[0]), "longdouble")
    want = oracle.reduce_pe(op, "longdouble", ss, 0)
    return np.nonzero((vb(got) != vb(want)).any(axis=1))[0], got, want


for op in ("prod", "sum"):
    bad, got, want = fold(op, srcs)
    print(op, "full:", len(bad), "mismatches", bad[:10].tolist())
    for i in bad[:3]:
        print("  i", i, "ops", [vb(s[i:i + 1])[0][::-1].tobytes().hex() for s in srcs],
              "gpu", vb(got[i:i + 1])[0][::-1].tobytes().hex(), "host", vb(want[i:i + 1])[0][::-1].tobytes().hex())
        w0 = i // 64 * 64
        wbad, _, _ = fold(op, [s[w0:w0 + 64].copy() for s in srcs])
        print("  its wave alone:", len(wbad), "mismatches", (wbad + w0).tolist())
        sbad, _, _ = fold(op, [s[i:i + 1].copy() for s in srcs])
        print("  the element alone:", len(sbad), "mismatches")
shm.finalize()
