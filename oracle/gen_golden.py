#!/usr/bin/env python3
"""Generate tests/golden/: input/output vectors for all 44 reductions.

Expected outputs come from the REFERENCE's own compiled operator functions
(oracle/_ref/libref_ops.so, built from /root/reference/src/reduce/reduce-op.c
by `make -C oracle ref`), applied in the fold order of reduce-op.c:226-264:
member `me` starts from its own source and folds in every other member in
ascending active-set order, the accumulator on the left.

Each file golden_<op>_<dtype>.npz holds, per case k:
    in_k   [npes, n]  sources in active-set order
    out_k  [npes, n]  the reference's result on each member
and manifest.json lists the cases. Inputs include the edge values the path
must survive: integer overflow, NaN / +-0 / +-Inf / denormals, complex
Inf/NaN products, x87 denormal / unnormal / NaN encodings.

NaN-payload families golden_nan_<op>_<dtype>.npz (sum/prod of float, double,
float complex, double complex; manifest "nan_cases"): operands rich in NaNs of
every sign, payload and quiet/signalling kind, infinities, zeros and values
whose sums overflow, so that which NaN comes out -- the SSE rule: the first
NaN operand, quieted, or the negative "indefinite" NaN of an invalid
operation -- and libgcc's complex-multiply operand order are pinned by the
reference's compiled code.

Usage: python3 oracle/gen_golden.py [outdir]   (needs oracle/_ref built)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import oracle  # noqa: E402

# (npes, n) cases per pair; n covers 0, 1, chunk edges 63/64/65, 127/128, a
# few hundred, and npes covers 1,2,3,4,5,8
CASES = [(1, 65), (2, 300), (3, 127), (4, 64), (8, 130), (2, 0), (5, 1), (8, 63), (3, 128)]
# the NaN-payload families: npes up to 9 (a fold beyond one launch's 8 sources)
NAN_CASES = [(2, 515), (3, 257), (5, 130), (8, 300), (9, 67)]
NAN_PAIRS = [(op, t) for op in ("sum", "prod") for t in ("float", "double", "complexf", "complexd")]


def fp_values(rng, n, np_t):
    """Full-mantissa values (x in (-1,1) * (1 + u*2^-40) * 2^k) with specials."""
    k = rng.integers(0, 8, n)
    x = rng.uniform(-1, 1, n) * (1 + rng.uniform(0, 1, n) * 2.0**-40) * np.exp2(k)
    x = x.astype(np_t)
    fi = np.finfo(np_t)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, fi.tiny / 4, -fi.tiny / 3,
                         fi.max, -fi.max, fi.max / 2, 1.0, -1.0], dtype=np_t)
    m = rng.random(n) < 0.08
    x[m] = rng.choice(specials, int(m.sum()))
    return x


def nan_rich(rng, n, np_t):
    """Bit patterns of np_t (float32/float64): 35 % NaNs (random sign and
    payload, quiet or signalling), 10 % +-inf, 10 % +-0, 15 % huge values
    (their sums overflow: inf - inf later), the rest ordinary numbers."""
    u_t = np.uint32 if np_t == np.float32 else np.uint64
    bits = 32 if np_t == np.float32 else 64
    mbits = 23 if np_t == np.float32 else 52
    exp_all = u_t(((1 << (bits - 1 - mbits)) - 1) << mbits)
    quiet = u_t(1 << (mbits - 1))
    sign = u_t(1 << (bits - 1))
    x = (rng.uniform(-4, 4, n)).astype(np_t).view(u_t).copy()
    r = rng.random(n)
    payload = rng.integers(1, 1 << (mbits - 1), n, dtype=np.uint64).astype(u_t)
    sgn = np.where(rng.random(n) < 0.5, sign, u_t(0)).astype(u_t)
    qnan = exp_all | quiet | payload | sgn
    snan = exp_all | payload | sgn                       # quiet bit clear, payload != 0
    fi = np.finfo(np_t)
    huge = (np.where(rng.random(n) < 0.5, fi.max, -fi.max) * rng.uniform(0.5, 1, n)).astype(np_t).view(u_t)
    x = np.where(r < 0.25, qnan, x)
    x = np.where((r >= 0.25) & (r < 0.35), snan, x)
    x = np.where((r >= 0.35) & (r < 0.45), exp_all | sgn, x)    # +-inf
    x = np.where((r >= 0.45) & (r < 0.55), sgn, x)              # +-0
    x = np.where((r >= 0.55) & (r < 0.70), huge, x)
    return x.astype(u_t).view(np_t)


def nan_values(rng, dtype, n):
    if dtype in ("float", "double"):
        return nan_rich(rng, n, oracle.NP[dtype])
    base = np.float32 if dtype == "complexf" else np.float64
    out = np.empty(n, dtype=oracle.NP[dtype])
    out.real, out.imag = nan_rich(rng, n, base), nan_rich(rng, n, base)
    return out


def int_values(rng, n, np_t, op):
    info = np.iinfo(np_t)
    bits = np.dtype(np_t).itemsize * 8
    if op == "and":  # bits set with p = 0.9 so an 8-way AND is not all zero
        u = np.zeros(n, dtype=np.uint64)
        for b in range(bits):
            u |= ((rng.random(n) < 0.9).astype(np.uint64) << np.uint64(b))
        x = u.astype(np.dtype(f"u{bits // 8}")).view(np_t)
    else:
        x = rng.integers(info.min, info.max, n, dtype=np_t, endpoint=True)
    specials = np.array([0, -1, 1, info.min, info.max], dtype=np_t)
    m = rng.random(n) < 0.08
    x[m] = rng.choice(specials, int(m.sum()))
    return x


def ld_values(rng, n):
    """x87 extended values as raw 16-byte slots, including odd encodings."""
    raw = np.zeros((n, 16), dtype=np.uint8)
    mant = rng.integers(0, 2**63, n, dtype=np.uint64) | np.uint64(1 << 63)
    exp = (16383 + rng.integers(-8, 8, n)).astype(np.uint16)
    sign = (rng.random(n) < 0.5).astype(np.uint16) << np.uint16(15)
    kind = rng.random(n)
    for i in range(n):
        m, e, s = int(mant[i]), int(exp[i]), int(sign[i])
        r = kind[i]
        if r < 0.02:
            m, e = 0, 0                              # +-0
        elif r < 0.04:
            m, e = int(mant[i]) >> 5, 0              # denormal
        elif r < 0.05:
            m, e = int(mant[i]) | (1 << 63), 0       # pseudo-denormal
        elif r < 0.06:
            m, e = 1 << 63, 0x7FFF                   # +-inf
        elif r < 0.07:
            m, e = (3 << 62) | 12345, 0x7FFF         # quiet NaN
        elif r < 0.075:
            m, e = (1 << 63) | 777, 0x7FFF           # signalling NaN
        elif r < 0.08:
            m, e = int(mant[i]) & ((1 << 63) - 1), 100  # unnormal (invalid operand)
        elif r < 0.09:
            e = 32767 - 2                            # near overflow
        elif r < 0.10:
            e = 3                                    # near underflow
        raw[i, 0:8] = np.frombuffer(np.uint64(m).tobytes(), dtype=np.uint8)
        raw[i, 8:10] = np.frombuffer(np.uint16(s | e).tobytes(), dtype=np.uint8)
    return raw.view(np.longdouble).reshape(n)


def values(rng, op, dtype, n):
    t = oracle.NP[dtype]
    if dtype in ("short", "int", "long", "longlong"):
        return int_values(rng, n, t, op)
    if dtype in ("float", "double"):
        return fp_values(rng, n, t)
    if dtype == "longdouble":
        return ld_values(rng, n)
    base = np.float32 if dtype == "complexf" else np.float64
    re, im = fp_values(rng, n, base), fp_values(rng, n, base)
    if op == "prod":  # keep products finite mostly: magnitudes near 1
        re = np.where(np.isfinite(re), re / 4, re).astype(base)
        im = np.where(np.isfinite(im), im / 4, im).astype(base)
    out = np.empty(n, dtype=t)
    out.real, out.imag = re, im
    return out


def main():
    outdir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "..", "tests", "golden")
    if not oracle.ref_available():
        sys.exit("oracle/_ref/libref_ops.so missing: run `make -C oracle ref` (needs /root/reference)")
    os.makedirs(outdir, exist_ok=True)
    manifest = {"generator": "oracle/gen_golden.py",
                "expected_from": "reference src/reduce/reduce-op.c operator functions "
                                 "(oracle/_ref/libref_ops.so), fold order of reduce-op.c:226-264",
                "cases": {}}
    seed = 20261015
    for op, dtype in oracle.PAIRS:
        rng = np.random.default_rng(seed)
        seed += 1
        arrays = {}
        cases = []
        for k, (npes, n) in enumerate(CASES):
            srcs = [values(rng, op, dtype, n) for _ in range(npes)]
            outs = [oracle.ref_reduce_pe(op, dtype, srcs, me) for me in range(npes)]
            arrays[f"in_{k}"] = np.stack(srcs) if n else np.zeros((npes, 0), dtype=oracle.NP[dtype])
            arrays[f"out_{k}"] = np.stack(outs) if n else np.zeros((npes, 0), dtype=oracle.NP[dtype])
            cases.append({"npes": npes, "n": n})
        np.savez_compressed(os.path.join(outdir, f"golden_{op}_{dtype}.npz"), **arrays)
        manifest["cases"][f"{op}_{dtype}"] = cases
    manifest["nan_cases"] = {}
    seed = 20261018
    for op, dtype in NAN_PAIRS:
        rng = np.random.default_rng(seed)
        seed += 1
        arrays = {}
        cases = []
        for k, (npes, n) in enumerate(NAN_CASES):
            srcs = [nan_values(rng, dtype, n) for _ in range(npes)]
            outs = [oracle.ref_reduce_pe(op, dtype, srcs, me) for me in range(npes)]
            arrays[f"in_{k}"] = np.stack(srcs)
            arrays[f"out_{k}"] = np.stack(outs)
            cases.append({"npes": npes, "n": n})
        np.savez_compressed(os.path.join(outdir, f"golden_nan_{op}_{dtype}.npz"), **arrays)
        manifest["nan_cases"][f"{op}_{dtype}"] = cases
    with open(os.path.join(outdir, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"wrote {len(oracle.PAIRS)} fixture files to {outdir}")


if __name__ == "__main__":
    main()
