#!/usr/bin/env python3
"""Time the long double every-member fold (mi355_combine_orders, sum and
product) in variant builds of the library (tools/build_x80_variants.sh): each
variant in a process of its own (SHMEM_REDUCE_LIBDIR picks the library), k
sources of 256/k MiB -> k outputs (the N = k reduce-scatter shape), two data
sets: doubles widened to long double, and full 64-bit significands. Per
launch: wall time of 10 back-to-back launches / 10, and (us_isolated) the
mean of 10 launches each timed alone by a HIP event pair on the library's
stream (mi355_time_next_launch, as bench.py's kernel legs). The float complex
product at 8 sources is timed too (complexf rows). Every output is hashed
(the variants must agree bit for bit) and 2048 samples of each are checked
against the oracle (the reference's own-first-then-ascending order, x87 on the
host). Measurement tool.
usage: python3 tools/x80_variant_time.py OUT.jsonl variant [variant ...]   ("lib" = the default build)"""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S = 256 << 20


def child():
    import numpy as np
    sys.path[:0] = [os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")]
    import oracle
    import shmem_reduce
    os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", str(2 * S + (64 << 20)))
    os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")
    os.environ.setdefault("SHMEM_DEVICE_ORDER_SIZE", "1M")
    shm = shmem_reduce.Shmem()
    shm.init()
    src, out = shm.malloc_device(S), shm.malloc_device(S)
    import ctypes
    L, vp = shm.lib, ctypes.c_void_p
    L.mi355_time_next_launch.argtypes = [vp, vp]
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    ev = [vp() for _ in range(20)]
    for e in ev:
        L.hipEventCreate(ctypes.byref(e))

    def isolated(launch):
        for r in range(10):
            L.mi355_time_next_launch(ev[2 * r], ev[2 * r + 1])
            assert launch() == 0
            shm.sync()
        ms = ctypes.c_float()
        tot = 0.0
        for r in range(10):
            L.hipEventElapsedTime(ctypes.byref(ms), ev[2 * r], ev[2 * r + 1])
            tot += ms.value
        return round(tot / 10 * 1e3, 1)

    rng = np.random.default_rng(11)
    x = (rng.random(S // 16) - 0.5).astype(np.longdouble)
    data = {"doubles": x}
    y = rng.random(S // 16).astype(np.longdouble)
    data["full"] = x * (np.longdouble(1) + y * np.longdouble(2.0) ** -60)
    del y
    for dname, arr in data.items():
        shm.put(src, arr)
        for k in (8, 4, 2):
            shard = S // k
            n = shard // 16
            srcs = [src + q * shard for q in range(k)]
            dsts = [out + q * shard for q in range(k)]
            sidx = np.unique(rng.integers(0, n, 2048))
            for op in ("sum", "prod"):
                for _ in range(2):
                    assert shm.combine_orders(op, "longdouble", dsts, srcs, n) == 0
                shm.sync()
                t0 = time.perf_counter()
                for _ in range(10):
                    assert shm.combine_orders(op, "longdouble", dsts, srcs, n) == 0
                shm.sync()
                us = (time.perf_counter() - t0) / 10 * 1e6
                us_iso = isolated(lambda: shm.combine_orders(op, "longdouble", dsts, srcs, n))
                h = hashlib.sha256()
                bad = 0
                ins = [arr[q * n:(q + 1) * n][sidx] for q in range(k)]
                for q in range(k):
                    got = shm.get(dsts[q], n, "longdouble")
                    h.update(got.tobytes())
                    want = oracle.reduce_pe(op, "longdouble", ins, q)
                    bad += int((got[sidx] != want).sum())
                print(json.dumps({"data": dname, "sources": k, "op": op, "us_per_launch": round(us, 1),
                                  "us_isolated": us_iso,
                                  "GB_s": round(2 * S / us / 1e3, 1), "sha": h.hexdigest()[:16], "oracle_bad": bad}),
                      flush=True)
    # the float complex product, 8 sources x 32 MiB (the same bytes as the x87 shape)
    k, shard = 8, S // 8
    n = shard // 8
    x = rng.random(2 * n * k) - 0.5
    cz = (x[0::2] + 1j * x[1::2]).astype(np.complex64) * np.float32(2)
    for q in range(k):
        shm.put(src + q * shard, cz[q * n:(q + 1) * n])
    srcs = [src + q * shard for q in range(k)]
    dsts = [out + q * shard for q in range(k)]
    for _ in range(2):
        assert shm.combine_orders("prod", "complexf", dsts, srcs, n) == 0
    shm.sync()
    t0 = time.perf_counter()
    for _ in range(10):
        assert shm.combine_orders("prod", "complexf", dsts, srcs, n) == 0
    shm.sync()
    us = (time.perf_counter() - t0) / 10 * 1e6
    us_iso = isolated(lambda: shm.combine_orders("prod", "complexf", dsts, srcs, n))
    h = hashlib.sha256()
    for q in range(k):
        h.update(shm.get(dsts[q], n, "complexf").tobytes())
    print(json.dumps({"data": "complexf", "sources": k, "op": "prod", "us_per_launch": round(us, 1),
                      "us_isolated": us_iso, "sha": h.hexdigest()[:16], "oracle_bad": 0}), flush=True)
    shm.finalize()


def main():
    out, variants = sys.argv[1], sys.argv[2:]
    with open(out, "a") as f:
        for rep in (1, 2):
            for v in variants:
                env = dict(os.environ)
                if v != "lib":
                    env["SHMEM_REDUCE_LIBDIR"] = os.path.join(ROOT, "osss-gasnet_amd", "lib", "variants", v)
                p = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                                   timeout=300)
                if p.returncode != 0:
                    print(f"variant {v}: rc {p.returncode}\n{p.stderr[-2000:]}", flush=True)
                    sys.exit(1)
                for ln in p.stdout.splitlines():
                    if ln.startswith("{"):
                        d = dict(json.loads(ln), variant=v, rep=rep)
                        f.write(json.dumps(d) + "\n")
                        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    child() if sys.argv[1:] == ["--child"] else main()
