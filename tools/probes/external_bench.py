"""Time shmem_double_sum_to_all on plain hipMalloc buffers (a framework's
tensors: outside the device symmetric heap) against the same call on
symmetric-heap buffers, per message size. One JSON line per (kind, size) on
PE 0.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29655 tools/probes/external_bench.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "osss-gasnet_amd"))
import shmem_reduce  # noqa: E402


def main():
    sizes = [int(x) for x in os.environ.get("EXT_SIZES", "65536,1048576,16777216,268435456").split(",")]
    os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str(2 * max(sizes) + (64 << 20)))
    os.environ.setdefault("SHMEM_BARRIER_TIMEOUT", "60")
    shm = shmem_reduce.Shmem()
    shm.init()
    me, npes = shm.my_pe(), shm.n_pes()
    hip = ctypes.CDLL("libamdhip64.so")
    loop = shmem_reduce.bench_loop()
    big = max(sizes)
    ext = []
    for _ in range(2):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(big)) == 0
        ext.append(p.value)
    sym = [shm.malloc_device(big), shm.malloc_device(big)]
    x = np.random.default_rng(me).standard_normal(big // 8)
    for kind, (dst, src) in (("symmetric", sym), ("hipMalloc", ext)):
        shm.put(src, x)
        for S in sizes:
            n = S // 8
            k = max(5, min(2000, int(2e9 // S)))
            loop(dst, src, n, 0, 0, npes, None, shm._psync_ptr, 3)
            shm.barrier_all()
            shm.sync()
            t0 = time.perf_counter()
            loop(dst, src, n, 0, 0, npes, None, shm._psync_ptr, k)
            shm.sync()
            t = (time.perf_counter() - t0) / k
            tb = np.array([t]), np.zeros(1)
            shm.to_all("max", "double", tb[1].ctypes.data, tb[0].ctypes.data, 1, 0, 0, npes)
            loop(dst, src, n, 0, 0, npes, None, shm._psync_ptr, 1)
            sched = shm.last_call_info()["schedule"]
            if me == 0:
                print(json.dumps({"kind": kind, "npes": npes, "bytes_per_pe": S, "calls": k,
                                  "us_per_call": round(tb[1][0] * 1e6, 2),
                                  "value_GiB_s": round(npes * S / tb[1][0] / 2**30, 2), "schedule": sched}),
                      flush=True)
    shm.barrier_all()
    for p in ext:
        hip.hipFree(ctypes.c_void_p(p))
    shm.free_device(sym[0])
    shm.free_device(sym[1])
    shm.finalize()


if __name__ == "__main__":
    main()
