#!/usr/bin/env python3
"""Bits of a few long double products/sums folded on the GPU (mi355_combine)
next to the host x87's (debug tool for x80.h)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
import shmem_reduce  # noqa: E402

hexes = sys.argv[1:] or ["2013585ddb45df8c37f3", "fd9c59a13fbf229cc44c", "7b7440ad4bd902fedb3f"]
vals = []
for h in hexes:
    b = bytes.fromhex(h) + bytes(6)
    vals.append(np.frombuffer(b, dtype=np.longdouble)[0])
os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", "16M")
shm = shmem_reduce.Shmem()
shm.init()
bufs = [shm.malloc_device(4096) for _ in range(len(vals) + 1)]
for b, v in zip(bufs, vals):
    shm.put(b, np.array([v] * 4, dtype=np.longdouble))


def bits(x):
    return np.array([x], dtype=np.longdouble).view(np.uint8)[:10][::-1].tobytes().hex()


for op in ("prod", "sum"):
    for k in range(2, len(vals) + 1):
        assert shm.combine(op, "longdouble", bufs[-1], bufs[:k], 4) == 0
        shm.sync()
        got = shm.get(bufs[-1], 4, "longdouble")[0]
        want = oracle.reduce_pe(op, "longdouble", [np.array([v]) for v in vals[:k]], 0)[0]
        print(op, k, "gpu", bits(got), "host", bits(want), "OK" if bits(got) == bits(want) else "DIFF")
shm.finalize()
