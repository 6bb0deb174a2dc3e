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


def main():
    spec = json.load(open(sys.argv[1]))
    outdir = sys.argv[2]
    shm = shmem_reduce.Shmem()
    shm.init()
    me = shm.my_pe()
    maxb = max((c["n"] + 16) * 16 for c in spec["cases"])
    da, db = shm.malloc_device(maxb), shm.malloc_device(maxb)
    ha, hb = shm.malloc(maxb), shm.malloc(maxb)
    results = {}
    for c in spec["cases"]:
        mine = None
        for s in c["sets"]:
            if me in members(*s):
                mine = s
        if mine is None:
            continue
        op, dtype, n = c["op"], c["dtype"], c["n"]
        es = np.dtype(shmem_reduce.NP[dtype]).itemsize
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
        elif mode == "unaligned":        # device, both one element off 16-byte alignment
            src, dst = da + es, db + es
        else:
            raise ValueError(mode)
        if n:
            shm.put(src, x)
        shm.set_algorithm(c.get("algorithm", "auto"))
        shm.to_all(op, dtype, dst, src, n, *mine)
        results[str(c["id"])] = shm.get(dst, n, dtype) if n else np.zeros(0, dtype=shmem_reduce.NP[dtype])
    shm.free(hb)
    shm.free(ha)
    shm.free_device(db)
    shm.free_device(da)
    shm.finalize()
    np.savez(os.path.join(outdir, f"pe{me}.npz"), **results)


if __name__ == "__main__":
    main()
