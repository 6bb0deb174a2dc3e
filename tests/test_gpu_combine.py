"""GPU: the combine layer (include/mi355_reduce.h) against the golden vectors
and the oracle, called through the C ABI on device buffers.

A fold of the sources in order [me, every other member ascending] is exactly
what the reference computes on member `me` (reduce-op.c:226-264), so one GPU
reproduces every PE's reference result of a golden case.
"""
import numpy as np
import pytest

import oracle
from _compare import assert_match
from test_oracle_golden import load_cases

pytestmark = pytest.mark.gpu


class Dev:
    """Device buffers from the symmetric heap, freed at the end of a test."""

    def __init__(self, shm):
        self.shm, self.ptrs = shm, []

    def upload(self, arr):
        p = self.shm.malloc_device(max(arr.nbytes, 16))
        if arr.nbytes:
            self.shm.put(p, arr)
        self.ptrs.append(p)
        return p

    def empty(self, nbytes):
        p = self.shm.malloc_device(max(nbytes, 16))
        self.ptrs.append(p)
        return p

    def free(self):
        for p in reversed(self.ptrs):
            self.shm.free_device(p)
        self.ptrs = []


@pytest.fixture
def dev(shm):
    d = Dev(shm)
    yield d
    d.free()


def gpu_fold(shm, dev, op, dtype, srcs, offset_elems=0):
    n = len(srcs[0])
    es = np.dtype(oracle.NP[dtype]).itemsize
    ptrs = []
    for s in srcs:
        pad = np.zeros(offset_elems, dtype=oracle.NP[dtype])
        ptrs.append(dev.upload(np.concatenate([pad, s])) + offset_elems * es)
    out = dev.empty((n + offset_elems) * es) + offset_elems * es
    rc = shm.combine(op, dtype, out, ptrs, n)
    assert rc == 0, rc
    shm.sync()
    return shm.get(out, n, dtype)


@pytest.mark.parametrize("op,dtype", oracle.PAIRS)
def test_combine_reproduces_every_pe_of_golden(shm, dev, op, dtype):
    for npes, ins, outs in load_cases(op, dtype):
        if ins.shape[1] == 0:
            continue
        for me in range(npes):
            order = [me] + [i for i in range(npes) if i != me]
            got = gpu_fold(shm, dev, op, dtype, [ins[i] for i in order])
            assert_match(got, outs[me], op, dtype, ctx=f"golden npes={npes} me={me}")
        dev.free()


def gpu_orders(shm, dev, op, dtype, srcs, offset_elems=0, skip=(), inplace=None):
    """mi355_combine_orders: member q's reference order into dst q (None for q in skip);
    inplace = q: dst q is src q itself. Returns {q: result}."""
    n = len(srcs[0])
    es = np.dtype(oracle.NP[dtype]).itemsize
    pad = np.zeros(offset_elems, dtype=oracle.NP[dtype])
    sp = [dev.upload(np.concatenate([pad, s])) + offset_elems * es for s in srcs]
    dp = []
    for q in range(len(srcs)):
        if q in skip:
            dp.append(None)
        elif q == inplace:
            dp.append(sp[q])
        else:
            dp.append(dev.empty((n + offset_elems) * es) + offset_elems * es)
    rc = shm.combine_orders(op, dtype, dp, sp, n)
    assert rc == 0, rc
    shm.sync()
    return {q: shm.get(d, n, dtype) for q, d in enumerate(dp) if d is not None}


@pytest.mark.parametrize("op,dtype", oracle.PAIRS)
def test_combine_orders_reproduces_every_pe_of_golden(shm, dev, op, dtype):
    """One launch over the golden sources yields every member's reference
    result (the owner-computes-every-order fold of the P2P schedule)."""
    for npes, ins, outs in load_cases(op, dtype):
        if ins.shape[1] == 0 or npes < 2:
            continue
        got = gpu_orders(shm, dev, op, dtype, [ins[i] for i in range(npes)])
        for me in range(npes):
            assert_match(got[me], outs[me], op, dtype, ctx=f"golden npes={npes} me={me}")
        dev.free()


@pytest.mark.parametrize("op,dtype", [("sum", "double"), ("max", "float"), ("min", "double"), ("prod", "complexd"),
                                      ("sum", "longdouble"), ("xor", "short")])
@pytest.mark.parametrize("nsrc", [2, 3, 8, 9, 13, 32])
def test_combine_orders_any_number_of_sources(shm, dev, op, dtype, nsrc):
    """Up to 8 sources in one launch, beyond that one left fold per member;
    one member in place, one skipped, element tails, user offsets."""
    import gen_golden
    rng = np.random.default_rng(100 + nsrc)
    n = 2051
    srcs = [gen_golden.values(rng, op, dtype, n) for _ in range(nsrc)]
    want = oracle.reduce_all(op, dtype, srcs)
    for off, skip, inplace in ((0, (), None), (1, (nsrc - 1,), 0), (3, (0,), nsrc - 1)):
        got = gpu_orders(shm, dev, op, dtype, srcs, offset_elems=off, skip=skip, inplace=inplace)
        assert sorted(got) == [q for q in range(nsrc) if q not in skip]
        for q, g in got.items():
            assert_match(g, want[q], op, dtype, ctx=f"nsrc={nsrc} off={off} member {q}")
        dev.free()


@pytest.mark.parametrize("op,dtype", [("min", "double"), ("max", "double"), ("min", "float"), ("max", "float")])
@pytest.mark.parametrize("nsrc", [2, 3, 5, 8])
def test_combine_orders_minmax_sparse_specials(shm, dev, op, dtype, nsrc):
    """The every-member min/max folds one value for every member on vectors
    whose operands hold no NaN and no zero, and runs the per-member chains
    only where they do: 200 000 full-mantissa elements per source with a few
    NaNs, +-0 and equal-value ties planted, so that one launch mixes both
    paths; every member's output against the reference's own order."""
    rng = np.random.default_rng(7 * nsrc + len(op))
    n = 200000
    t = oracle.NP[dtype]
    srcs = []
    for k in range(nsrc):
        x = ((rng.uniform(-1, 1, n) + 2.0 ** -30) * np.exp2(rng.integers(-4, 4, n))).astype(t)
        x[x == 0] = t(1.5)
        pos = rng.integers(0, n, 24)
        x[pos[:8]] = t(np.nan)
        x[pos[8:16]] = t(0.0)
        x[pos[16:20]] = t(-0.0)
        x[pos[20:]] = t(0.25)  # ties with the other sources' planted 0.25
        srcs.append(x)
    common = rng.integers(0, n, 16)  # the same positions in every source: +0/-0 and NaN across members
    for k, x in enumerate(srcs):
        x[common[:8]] = t(0.0) if k % 2 else t(-0.0)
        x[common[8:12]] = t(np.nan) if k == nsrc - 1 else t(0.5)
        x[common[12:]] = t(0.25)
    want = oracle.reduce_all(op, dtype, srcs)
    got = gpu_orders(shm, dev, op, dtype, srcs)
    for q, g in got.items():
        assert_match(g, want[q], op, dtype, ctx=f"nsrc={nsrc} member {q}")
    dev.free()


def x87(sign, efield, mant):
    """One long double from its fields (x86 80-bit format in 16 bytes)."""
    b = np.zeros(16, dtype=np.uint8)
    b[:8] = np.frombuffer(np.uint64(mant).tobytes(), dtype=np.uint8)
    b[8:10] = np.frombuffer(np.uint16((sign << 15) | efield).tobytes(), dtype=np.uint8)
    return b.view(np.longdouble)[0]


@pytest.mark.parametrize("op", ["min", "max"])
@pytest.mark.parametrize("nsrc", [2, 5, 8])
def test_combine_orders_x87_minmax_sparse_specials(shm, dev, op, nsrc):
    """Long double min/max: one fold serves every member only where every
    operand is a normal number; sparse NaNs, +-0, denormals and -- the x87's
    own case -- a pseudo-denormal beside the normal of the same value (equal
    numbers, different encodings: the select keeps the first) must take the
    per-member chains."""
    rng = np.random.default_rng(11 * nsrc + len(op))
    n = 100000
    t = np.longdouble
    tie_normal, tie_pseudo = x87(0, 1, 0x8000000000000123), x87(0, 0, 0x8000000000000123)
    assert tie_normal == tie_pseudo
    srcs = []
    for k in range(nsrc):
        x = ((rng.uniform(-1, 1, n) + 2.0 ** -30) * np.exp2(rng.integers(-4, 4, n))).astype(t)
        pos = rng.integers(0, n, 16)
        x[pos[:4]] = t(np.nan)
        x[pos[4:8]] = t(0.0)
        x[pos[8:12]] = np.finfo(t).tiny / 8
        x[pos[12:]] = tie_pseudo
        srcs.append(x)
    common = rng.integers(0, n, 12)
    for k, x in enumerate(srcs):
        x[common[:6]] = tie_pseudo if k % 2 else tie_normal  # equal values, two encodings, across members
        x[common[6:]] = t(-0.0) if k % 2 else t(0.0)
    want = oracle.reduce_all(op, "longdouble", srcs)
    got = gpu_orders(shm, dev, op, "longdouble", srcs)
    for q, g in got.items():
        assert_match(g, want[q], op, "longdouble", ctx=f"nsrc={nsrc} member {q}")
    dev.free()


@pytest.mark.parametrize("case", ["near", "bounds", "sparse"])
@pytest.mark.parametrize("op", ["sum", "prod"])
@pytest.mark.parametrize("nsrc", [2, 3, 5, 8])
def test_combine_orders_x87_chains(shm, dev, op, nsrc, case):
    """The every-member x87 sum/product (combine_kernels.h x80_orders_vector):
    every member's chain in the fast form, one wave vote, the general chains
    for the whole wave otherwise; every member against the host x87 in the
    reference's order (reduce-op.c:99 element function, one rounding per
    operation).
      near    exponent fields 16383 +- 70: the fast chains throughout
      bounds  the fast form's edges: fields at and around x80.h kChainLo and
              kFastMax - steps (sums), +-L around the bias (products),
              exponent differences 58-70 (exact alignment up to 62, general
              63-65, a dropped operand from 66), all-ones significands (round
              ups that wrap), operands that cancel to their last bits
      sparse  near, with a few zeros, denormals, infinities and NaNs planted:
              both kinds of waves in one launch"""
    rng = np.random.default_rng(1000 * nsrc + 10 * len(op) + len(case))
    n = 120000
    steps = nsrc - 1
    srcs = []
    for k in range(nsrc):
        e = 16383 + rng.integers(-70, 71, n)
        m = rng.integers(0, 2**64, n, dtype=np.uint64, endpoint=False) | np.uint64(1 << 63)
        if case == "bounds":
            pick = rng.integers(0, 6, n)
            lim = (0x7FFF - 3 - 16383 - steps) // (steps + 1)
            e = np.where(pick == 0, 62 + rng.integers(0, 6, n), e)
            e = np.where(pick == 1, 0x7FFC - steps + rng.integers(-3, 3, n), e)
            e = np.where(pick == 2, 16383 + np.where(rng.random(n) < 0.5, -lim, lim) + rng.integers(-2, 3, n), e)
            e = np.where(pick == 3, 16383 - (k % 2) * rng.integers(58, 71, n), e)
            m = np.where(pick == 4, m | (~np.uint64(0) << rng.integers(0, 12, n).astype(np.uint64)), m)
            e = np.clip(e, 1, 0x7FFE)
        x = _x80(rng, n, e, m=m)
        if case == "bounds" and k == 1:  # member 1 nearly cancels member 0 on a sixth of the elements
            c = rng.random(n) < 1 / 6
            raw0, raw1 = srcs[0].view(np.uint8).reshape(n, 16), x.view(np.uint8).reshape(n, 16)
            m0 = raw0[:, 0:8].copy().view(np.uint64).reshape(n) ^ rng.integers(0, 1 << 10, n, dtype=np.uint64)
            se0 = raw0[:, 8:10].copy().view(np.uint16).reshape(n) ^ np.uint16(0x8000)
            raw1[c, 0:8] = (m0 | np.uint64(1 << 63))[c].view(np.uint8).reshape(-1, 8)
            raw1[c, 8:10] = se0[c].view(np.uint8).reshape(-1, 2)
        if case == "sparse":
            pos = rng.integers(0, n, 12)
            x[pos[:3]] = np.longdouble(0.0)
            x[pos[3:6]] = np.finfo(np.longdouble).tiny / 16
            x[pos[6:9]] = np.longdouble(np.inf) if k % 2 else -np.longdouble(np.inf)
            x[pos[9:]] = np.longdouble(np.nan)
        srcs.append(x)
    want = oracle.reduce_all(op, "longdouble", srcs)
    got = gpu_orders(shm, dev, op, "longdouble", srcs)
    for q, g in got.items():
        assert_match(g, want[q], op, "longdouble", ctx=f"{case} nsrc={nsrc} member {q}")
    dev.free()
    if case == "sparse":
        # each member's output is stored as its chain ends, before the wave
        # vote; a wave that fails it rewrites them from the general path: with
        # an output skipped (member 1, whose value the first chain also gives)
        # and one in place (the early store lands on its own source)
        got = gpu_orders(shm, dev, op, "longdouble", srcs, skip=(1,), inplace=0 if nsrc == 2 else nsrc - 1)
        assert sorted(got) == [q for q in range(nsrc) if q != 1]
        for q, g in got.items():
            assert_match(g, want[q], op, "longdouble", ctx=f"{case} nsrc={nsrc} member {q} skip/in place")
        dev.free()


@pytest.mark.parametrize("op,dtype", [("sum", "double"), ("xor", "int"), ("max", "float"), ("prod", "complexf"),
                                      ("min", "longdouble"), ("sum", "short")])
@pytest.mark.parametrize("nsrc", [1, 2, 5, 8, 9, 12, 17])
def test_combine_any_number_of_sources(shm, dev, op, dtype, nsrc):
    import gen_golden
    rng = np.random.default_rng(nsrc)
    srcs = [gen_golden.values(rng, op, dtype, 3001) for _ in range(nsrc)]
    got = gpu_fold(shm, dev, op, dtype, srcs)
    assert_match(got, oracle.reduce_pe(op, dtype, srcs, 0), op, dtype, ctx=f"nsrc={nsrc}")


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 255, 256, 257, 4095, 100003])
@pytest.mark.parametrize("dtype", ["short", "float", "double", "complexd"])
def test_combine_sizes_and_tails(shm, dev, n, dtype):
    import gen_golden
    rng = np.random.default_rng(n)
    srcs = [gen_golden.values(rng, "sum", dtype, n) for _ in range(3)]
    got = gpu_fold(shm, dev, "sum", dtype, srcs)
    assert_match(got, oracle.reduce_pe("sum", dtype, srcs, 0), "sum", dtype)


@pytest.mark.parametrize("off", [1, 3, 5])
@pytest.mark.parametrize("op,dtype", [("sum", "double"), ("and", "short"), ("min", "float"), ("prod", "int"),
                                      ("xor", "longlong"), ("sum", "complexf")])
def test_combine_unaligned_pointers(shm, dev, op, dtype, off):
    import gen_golden
    rng = np.random.default_rng(off)
    srcs = [gen_golden.values(rng, op, dtype, 1000) for _ in range(4)]
    got = gpu_fold(shm, dev, op, dtype, srcs, offset_elems=off)
    assert_match(got, oracle.reduce_pe(op, dtype, srcs, 0), op, dtype, ctx=f"offset {off}")


def test_longdouble_random_encodings(shm, dev):
    """Every 16-bit sign/exponent with random significands, all four ops, against
    the host x87 (the oracle is gcc-compiled long double arithmetic)."""
    rng = np.random.default_rng(99)
    n = 200000
    raw = np.zeros((3, n, 16), dtype=np.uint8)
    for k in range(3):
        m = rng.integers(0, 2**64, n, dtype=np.uint64, endpoint=False)
        se = rng.integers(0, 2**16, n, dtype=np.uint16)
        # bias half the exponents towards the normal range around 1.0 so sums interact
        near = rng.random(n) < 0.5
        se[near] = (se[near] & 0x8000) | (16383 + rng.integers(-70, 70, int(near.sum()))).astype(np.uint16)
        m[near] |= np.uint64(1 << 63)
        raw[k, :, 0:8] = m.view(np.uint8).reshape(n, 8)
        raw[k, :, 8:10] = se.view(np.uint8).reshape(n, 2)
    srcs = [raw[k].view(np.longdouble).reshape(n) for k in range(3)]
    for op in ("sum", "prod", "min", "max"):
        got = gpu_fold(shm, dev, op, "longdouble", srcs)
        assert_match(got, oracle.reduce_pe(op, "longdouble", srcs, 0), op, "longdouble")
        dev.free()


def _x80(rng, n, e, m=None, s=None):
    """long doubles from sign, biased exponent field and significand arrays"""
    raw = np.zeros((n, 16), dtype=np.uint8)
    if m is None:
        m = rng.integers(0, 2**64, n, dtype=np.uint64, endpoint=False) | np.uint64(1 << 63)
    if s is None:
        s = rng.integers(0, 2, n).astype(np.uint16)
    se = (s.astype(np.uint16) << np.uint16(15)) | np.asarray(e, dtype=np.uint16)
    raw[:, 0:8] = m.view(np.uint8).reshape(n, 8)
    raw[:, 8:10] = se.view(np.uint8).reshape(n, 2)
    return raw.view(np.longdouble).reshape(n)


@pytest.mark.parametrize("case", ["near", "spread", "cancel", "edges", "mixed"])
def test_longdouble_add_mul_paths(shm, dev, case):
    """x80.h's fast add/mul (normal operands, exponent fields up to 0x7FFC,
    alignment within 64 bits, normal results) and its general path meet at
    their boundaries: sums and products of two sources, 2^20 pairs per case,
    bit-exact against the host x87 (gcc long double, the oracle).
      near    exponent differences 0-3, random signs: carries, cancellations
      spread  differences 0-70: the 64-bit alignment limit and beyond
      cancel  b = -a with its last significand bits perturbed: deep cancellation
      edges   exponent fields near 1 and near 0x7FFC-0x7FFE: denormal and
              overflowing results, and operands just outside the fast path
      mixed   the above with zeros, denormals, infinities and NaNs sprinkled in"""
    rng = np.random.default_rng({"near": 1, "spread": 2, "cancel": 3, "edges": 4, "mixed": 5}[case])
    n = 1 << 20
    e0 = rng.integers(1, 0x7FFF, n)
    if case == "near":
        ea, eb = e0 % 0x7F00 + 100, None
        eb = ea + rng.integers(-3, 4, n)
    elif case == "spread":
        ea = rng.integers(16000, 16800, n)
        eb = ea - rng.integers(0, 71, n)
    elif case == "cancel":
        a = _x80(rng, n, rng.integers(100, 32000, n))
        m = a.view(np.uint8).reshape(n, 16)[:, 0:8].copy().view(np.uint64).reshape(n)
        m2 = m ^ rng.integers(0, 1 << 12, n, dtype=np.uint64)
        se = a.view(np.uint8).reshape(n, 16)[:, 8:10].copy().view(np.uint16).reshape(n)
        b = _x80(rng, n, se & np.uint16(0x7FFF), m=m2 | np.uint64(1 << 63), s=((se >> np.uint16(15)) ^ np.uint16(1)))
        srcs = [a, b]
    elif case in ("edges", "mixed"):
        pick = rng.integers(0, 3, n)
        ea = np.where(pick == 0, rng.integers(1, 80, n), np.where(pick == 1, rng.integers(0x7FF8, 0x7FFF, n),
                                                                   rng.integers(16000, 16800, n)))
        eb = np.where(pick == 0, rng.integers(1, 80, n), np.where(pick == 1, rng.integers(0x3F80, 0x4080, n),
                                                                   ea - rng.integers(-2, 3, n)))
        eb = np.clip(eb, 1, 0x7FFE)
    if case != "cancel":
        srcs = [_x80(rng, n, ea), _x80(rng, n, eb)]
    if case == "mixed":
        specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-4940], dtype=np.longdouble)
        for k in range(2):
            where = rng.random(n) < 0.05
            srcs[k][where] = specials[rng.integers(0, len(specials), int(where.sum()))]
    for op in ("sum", "prod"):
        got = gpu_fold(shm, dev, op, "longdouble", srcs)
        assert_match(got, oracle.reduce_pe(op, "longdouble", srcs, 0), op, "longdouble", ctx=case)
        dev.free()


def test_complex_prod_annex_g_cases(shm, dev):
    inf, nan = np.inf, np.nan
    vals = [complex(inf, nan), complex(nan, inf), complex(inf, inf), complex(nan, nan), complex(0, 0),
            complex(1, 2), complex(-0.0, inf), complex(1e308, 1e308), complex(nan, 0), complex(0, -inf)]
    a = np.array([x for x in vals for _ in vals], dtype=np.complex128)
    b = np.array([y for _ in vals for y in vals], dtype=np.complex128)
    for dtype in ("complexd", "complexf"):
        srcs = [a.astype(oracle.NP[dtype]), b.astype(oracle.NP[dtype])]
        got = gpu_fold(shm, dev, "prod", dtype, srcs)
        assert_match(got, oracle.reduce_pe("prod", dtype, srcs, 0), "prod", dtype)
        dev.free()


@pytest.mark.parametrize("nsrc", [3, 8])
@pytest.mark.parametrize("dtype", ["complexf", "complexd"])
def test_complex_prod_annex_g_every_member(shm, dev, dtype, nsrc):
    """The every-member complex product (combine_kernels.h: float complex
    chains with plain products and one wave vote on Annex G's recovery case,
    double complex with the recovery after each product): the Annex G operands
    planted sparsely among finite values, so one launch has waves that pass
    the vote and waves that redo their chains; every member against the
    reference's order, with one output skipped and one in place."""
    inf, nan = np.inf, np.nan
    specials = [complex(inf, nan), complex(nan, inf), complex(inf, inf), complex(nan, nan), complex(0, 0),
                complex(-0.0, inf), complex(1e30, 1e30), complex(nan, 0), complex(0, -inf)]
    rng = np.random.default_rng(31 * nsrc + len(dtype))
    n = 30000
    srcs = []
    for k in range(nsrc):
        x = (rng.uniform(-1.5, 1.5, n) + 1j * rng.uniform(-1.5, 1.5, n)).astype(np.complex128)
        pos = rng.integers(0, n, 40)
        x[pos] = [specials[(k + j) % len(specials)] for j in range(len(pos))]
        srcs.append(x.astype(oracle.NP[dtype]))
    want = oracle.reduce_all("prod", dtype, srcs)
    for skip, inplace in (((), None), ((1,), nsrc - 1)):
        got = gpu_orders(shm, dev, "prod", dtype, srcs, skip=skip, inplace=inplace)
        assert sorted(got) == [q for q in range(nsrc) if q not in skip]
        for q, g in got.items():
            assert_match(g, want[q], "prod", dtype, ctx=f"nsrc={nsrc} member {q} skip={skip}")
        dev.free()


def test_full_size_256mib_properties(shm, dev):
    """At the benchmark size (2^25 doubles = 256 MiB per source):
    - 2-source double sum equals numpy's IEEE a + b bit for bit,
    - xor is an involution (a ^ b ^ b == a), and
    - a one-source fold (copy) is the identity."""
    n = 1 << 25
    rng = np.random.default_rng(5)
    a = rng.standard_normal(n) * np.exp2(rng.integers(-20, 20, n))
    b = rng.standard_normal(n)
    pa, pb = dev.upload(a), dev.upload(b)
    out = dev.empty(8 * n)
    assert shm.combine("sum", "double", out, [pa, pb], n) == 0
    shm.sync()
    got = shm.get(out, n, "double")
    assert (got.view(np.uint64) == (a + b).view(np.uint64)).all()
    ai, bi = a.view(np.int64), b.view(np.int64)
    assert shm.combine("xor", "longlong", out, [pa, pb, pb], n) == 0
    shm.sync()
    assert (shm.get(out, n, "longlong") == ai).all()
    assert shm.combine("sum", "double", out, [pb], n) == 0
    shm.sync()
    assert (shm.get(out, n, "double").view(np.uint64) == b.view(np.uint64)).all()


def test_copy_segments_sizes_offsets_and_many_segments(shm, dev):
    """mi355_copy_segments (the 1-PE identity and the all-gather leg): every
    byte lands for sizes around the vector/pass boundaries, 16-byte aligned and
    not, one segment and 7 / 64 segments per launch (the launch shape divides
    the grid between segments). Regression for a store-data hazard: an
    inline-asm store whose data VGPRs the next VALU overwrote corrupted the
    upper lanes of small copies (fixed by the wait states in st16)."""
    import ctypes
    rng = np.random.default_rng(17)
    sizes = [1, 15, 16, 17, 255, 4096, 8000, 16383, 16384, 16400, 65536 + 48, 1 << 20, (1 << 22) + 16]
    for nb in sizes:
        # (target offset, source offset): aligned, equally misaligned (head
        # peeled, then vectors), differently misaligned (shifted loads:
        # funnel16, every source phase 1-15 against an aligned target)
        for doff, soff in ((0, 0), (16, 16), (3, 3), (8, 8), (3, 5), (0, 8), (8, 0), (0, 4), (4, 12), (0, 1),
                           (1, 0), (15, 2), (7, 0), (0, 15), (5, 30)):
            x = rng.integers(0, 256, nb + soff, dtype=np.uint8)
            s = dev.upload(x)
            d = dev.empty(nb + doff)
            dsts = (ctypes.c_void_p * 1)(d + doff)
            srcs = (ctypes.c_void_p * 1)(s + soff)
            nbs = (ctypes.c_size_t * 1)(nb)
            assert shm.lib.mi355_copy_segments(dsts, srcs, nbs, 1, None) == 0
            shm.sync()
            got = shm.get(d + doff, nb, np.uint8)
            assert (got == x[soff:]).all(), (nb, doff, soff, int(np.argmax(got != x[soff:])))
    for k, seg in ((7, 33333), (64, 4112)):
        # segments at mixed phases: aligned, shifted by 8, by 3
        xs = [rng.integers(0, 256, seg, dtype=np.uint8) for _ in range(k)]
        sp = [_upload_at(dev, x, (0, 8, 3)[i % 3]) for i, x in enumerate(xs)]
        dp = [dev.empty(seg) for _ in range(k)]
        dsts = (ctypes.c_void_p * k)(*dp)
        srcs = (ctypes.c_void_p * k)(*sp)
        nbs = (ctypes.c_size_t * k)(*([seg] * k))
        assert shm.lib.mi355_copy_segments(dsts, srcs, nbs, k, None) == 0
        shm.sync()
        for i in range(k):
            assert (shm.get(dp[i], seg, np.uint8) == xs[i]).all(), (k, i)


def _upload_at(dev, arr, off):
    """arr on the device at byte offset `off` from a fresh (256-byte aligned) buffer."""
    return dev.upload(np.concatenate([np.zeros(off, np.uint8), np.ascontiguousarray(arr).view(np.uint8)])) + off


def test_combine_target_and_sources_misaligned_differently(shm, dev):
    """Target one element off, sources three off: the sources share a phase
    the target lacks, so the fold runs as vectors with unaligned source
    loads; sources at different phases from each other too (shift_head).
    Results as the oracle's."""
    import gen_golden
    n, es = 3001, 8
    rng = np.random.default_rng(77)
    srcs = [gen_golden.values(rng, "sum", "double", n) for _ in range(3)]
    for soffs in ((3 * es,) * 3, (3 * es, 0, 3 * es)):
        ptrs = [_upload_at(dev, s, o) for s, o in zip(srcs, soffs)]
        out = dev.empty((n + 1) * es) + es
        assert shm.combine("sum", "double", out, ptrs, n) == 0
        shm.sync()
        assert_match(shm.get(out, n, "double"), oracle.reduce_pe("sum", "double", srcs, 0), "sum", "double",
                     ctx=str(soffs))


# (target byte offset, source byte offset) pairs whose 16-byte phases differ:
# the shifted-load vector kernels (combine_kernels.h shift_head / funnel16)
SHIFT_PAIRS = {2: [(0, 2), (2, 0), (0, 6), (6, 14), (10, 4)], 4: [(0, 4), (4, 0), (0, 8), (12, 4), (8, 12)],
               8: [(0, 8), (8, 0), (24, 16)], 16: [(0, 8)]}
SHIFT_TYPES = [("sum", "short"), ("xor", "int"), ("prod", "int"), ("and", "long"), ("sum", "longlong"),
               ("sum", "float"), ("max", "float"), ("prod", "float"), ("sum", "double"), ("min", "double"),
               ("prod", "double"), ("sum", "complexf"), ("prod", "complexf"), ("sum", "complexd"),
               ("prod", "complexd")]


@pytest.mark.parametrize("op,dtype", SHIFT_TYPES)
@pytest.mark.parametrize("nsrc", [1, 2, 3, 8])
def test_combine_shifted_sources(shm, dev, op, dtype, nsrc):
    """Target and sources at different 16-byte phases (every source at the
    same one): every value as the oracle's, NaN payloads included, for sizes
    around the vector boundaries (head peeled off the target, element tail)."""
    import gen_golden
    es = np.dtype(oracle.NP[dtype]).itemsize
    rng = np.random.default_rng(400 + nsrc)
    for doff, soff in SHIFT_PAIRS[es]:
        for n in (1, 7, 1000, 65537):
            srcs = [gen_golden.values(rng, op, dtype, n) for _ in range(nsrc)]
            ptrs = [_upload_at(dev, x, soff) for x in srcs]
            out = dev.empty(n * es + 32) + doff
            assert shm.combine(op, dtype, out, ptrs, n) == 0
            shm.sync()
            assert_match(shm.get(out, n, dtype), oracle.reduce_pe(op, dtype, srcs, 0), op, dtype,
                         ctx=f"target +{doff}, sources +{soff}, n={n}")
            dev.free()


@pytest.mark.parametrize("op,dtype", SHIFT_TYPES)
@pytest.mark.parametrize("nsrc", [2, 3, 8])
def test_combine_orders_shifted_sources(shm, dev, op, dtype, nsrc):
    """The every-member fold with its outputs at another 16-byte phase than
    its sources (the P2P schedule with target = &t[1], source = &s[0]): every
    member's reference result, with and without a skipped output."""
    import gen_golden
    es = np.dtype(oracle.NP[dtype]).itemsize
    rng = np.random.default_rng(500 + nsrc)
    for doff, soff in SHIFT_PAIRS[es]:
        for n, skip in ((7, ()), (4097, (1,)), (65537, ())):
            srcs = [gen_golden.values(rng, op, dtype, n) for _ in range(nsrc)]
            sp = [_upload_at(dev, x, soff) for x in srcs]
            dp = [None if q in skip else dev.empty(n * es + 32) + doff for q in range(nsrc)]
            assert shm.combine_orders(op, dtype, dp, sp, n) == 0
            shm.sync()
            for q in range(nsrc):
                if dp[q] is None:
                    continue
                assert_match(shm.get(dp[q], n, dtype), oracle.reduce_pe(op, dtype, srcs, q), op, dtype,
                             ctx=f"member {q}, target +{doff}, sources +{soff}, n={n}")
            dev.free()


LINE_TYPES = [("sum", "short"), ("xor", "int"), ("sum", "float"), ("max", "float"), ("sum", "double"),
              ("prod", "complexf"), ("sum", "complexd"), ("sum", "longdouble")]


@pytest.mark.parametrize("op,dtype", LINE_TYPES)
def test_targets_peeled_to_their_line(shm, dev, op, dtype):
    """Targets 16-112 bytes off a 128-byte line (a symmetric offset into the
    arrays): the fold, the every-member fold and the copy peel the target to
    its line (combine_kernels.h line_head, combine.hip seg_plan), folding or
    copying the head element-wise; sources on their line, at the target's
    offset, or (shifted loads) at another 16-byte phase. Sizes around the
    head: n below it (16-byte peel or element-wise), at it, just past it,
    one vector past it, many vectors."""
    import ctypes
    import gen_golden
    es = np.dtype(oracle.NP[dtype]).itemsize
    rng = np.random.default_rng(6100 + es)
    cases = [(16, 0), (48, 48), (112, 0), (64 + es, 0)] if es < 16 else [(16, 0), (112, 0), (48, 48)]
    for doff, soff in cases:
        h = ((128 - doff) & 127) // es
        for n in sorted({1, max(1, h - 1), h, h + 1, h + 16 // es + 1, 5000}):
            srcs = [gen_golden.values(rng, op, dtype, n) for _ in range(3)]
            ptrs = [_upload_at(dev, x, soff) for x in srcs]
            out = dev.empty(n * es + 128) + doff
            assert shm.combine(op, dtype, out, ptrs, n) == 0
            shm.sync()
            ctx = f"target +{doff}, sources +{soff}, n={n}"
            assert_match(shm.get(out, n, dtype), oracle.reduce_pe(op, dtype, srcs, 0), op, dtype, ctx=ctx)
            dp = [dev.empty(n * es + 128) + doff for _ in range(3)]
            assert shm.combine_orders(op, dtype, dp, ptrs, n) == 0
            shm.sync()
            for q in range(3):
                assert_match(shm.get(dp[q], n, dtype), oracle.reduce_pe(op, dtype, srcs, q), op, dtype,
                             ctx=f"member {q}, {ctx}")
            nb = n * es
            d = dev.empty(nb + 128) + doff
            dsts, sps, nbs = (ctypes.c_void_p * 1)(d), (ctypes.c_void_p * 1)(ptrs[0]), (ctypes.c_size_t * 1)(nb)
            assert shm.lib.mi355_copy_segments(dsts, sps, nbs, 1, None) == 0
            shm.sync()
            assert (shm.get(d, nb, np.uint8) == srcs[0].view(np.uint8)).all(), ctx
            dev.free()


@pytest.mark.parametrize("op,dtype", SHIFT_TYPES)
def test_combine_mixed_source_phases(shm, dev, op, dtype):
    """Sources at different 16-byte phases from each other (an offset into
    some of the arrays only): the fold and the every-member fold run as
    vectors with unaligned loads from every source (shift_head); targets on
    and off their phase. Every value as the oracle's."""
    import gen_golden
    es = np.dtype(oracle.NP[dtype]).itemsize
    rng = np.random.default_rng(700 + es)
    for nsrc in (2, 3, 8):
        soffs = [(k * es) % 16 + (16 if k % 3 == 2 else 0) for k in range(nsrc)]
        if len({o % 16 for o in soffs}) == 1:
            soffs[1] += 8   # 16-byte elements (complex double: 8-byte aligned in C)
        for doff in (0, es if es < 16 else 8, 48):
            for n in (5, 1000, 65537):
                srcs = [gen_golden.values(rng, op, dtype, n) for _ in range(nsrc)]
                sp = [_upload_at(dev, x, o) for x, o in zip(srcs, soffs)]
                ctx = f"sources +{soffs}, target +{doff}, n={n}"
                out = dev.empty(n * es + 64) + doff
                assert shm.combine(op, dtype, out, sp, n) == 0
                shm.sync()
                assert_match(shm.get(out, n, dtype), oracle.reduce_pe(op, dtype, srcs, 0), op, dtype, ctx=ctx)
                dp = [dev.empty(n * es + 64) + doff for _ in range(nsrc)]
                assert shm.combine_orders(op, dtype, dp, sp, n) == 0
                shm.sync()
                for q in range(nsrc):
                    assert_match(shm.get(dp[q], n, dtype), oracle.reduce_pe(op, dtype, srcs, q), op, dtype,
                                 ctx=f"member {q}, {ctx}")
                dev.free()


# ---------------------------------------------------------------------------
# NaN payloads: the golden_nan_* families (float, double and complex sum/prod
# on NaN-rich operands, outputs of the reference's compiled operators) through
# the fold, the every-member fold, their element-wise head/tail paths (offset
# pointers) and the multi-launch fold beyond 8 sources; bit for bit.
# ---------------------------------------------------------------------------
from test_oracle_golden import NAN_PAIRS, load_nan_cases  # noqa: E402


@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("op,dtype", NAN_PAIRS)
def test_nan_payloads_fold_every_pe(shm, dev, op, dtype, off):
    for npes, ins, outs in load_nan_cases(op, dtype):
        for me in range(npes):
            order = [me] + [i for i in range(npes) if i != me]
            got = gpu_fold(shm, dev, op, dtype, [ins[i] for i in order], offset_elems=off)
            assert_match(got, outs[me], op, dtype, strict=True, ctx=f"nan golden npes={npes} me={me} off={off}")
        dev.free()


@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("op,dtype", NAN_PAIRS)
def test_nan_payloads_every_member_fold(shm, dev, op, dtype, off):
    for npes, ins, outs in load_nan_cases(op, dtype):
        got = gpu_orders(shm, dev, op, dtype, [ins[i] for i in range(npes)], offset_elems=off)
        for me in range(npes):
            assert_match(got[me], outs[me], op, dtype, strict=True, ctx=f"nan golden npes={npes} me={me} off={off}")
        dev.free()


@pytest.mark.parametrize("op,dtype", NAN_PAIRS)
def test_nan_payloads_sparse_in_large_arrays(shm, dev, op, dtype):
    """Few NaNs among many ordinary values: the streaming kernels' fast form
    with the per-lane redo of only the chains that met a NaN (ops.h)."""
    import gen_golden
    rng = np.random.default_rng(4242)
    n, k = 300000, 8
    srcs = [gen_golden.values(rng, op, dtype, n) for _ in range(k)]
    specials = [gen_golden.nan_values(rng, dtype, 200) for _ in range(k)]
    for s, sp in zip(srcs, specials):
        s[rng.integers(0, n, 200)] = sp
    got = gpu_fold(shm, dev, op, dtype, srcs)
    assert_match(got, oracle.reduce_pe(op, dtype, srcs, 0), op, dtype, strict=True, ctx="fold")
    dev.free()
    got = gpu_orders(shm, dev, op, dtype, srcs)
    for q in range(k):
        assert_match(got[q], oracle.reduce_pe(op, dtype, srcs, q), op, dtype, strict=True, ctx=f"member {q}")


@pytest.mark.parametrize("dtype", ["float", "double"])
def test_nan_patch_copy_phases_and_flag(shm, dev, dtype):
    """mi355_nan_patch_copy (the two-member gather of reduce.c nan_pair):
    dst[i] = isnan(own[i]) ? quiet(own[i]) : peer[i] when the owner's NaN
    word is set (or absent), a plain copy of peer when it is clear; dst and
    peer at one 16-byte phase (a symmetric offset), own at the same or another
    one (the target offset against the source: own read unaligned)."""
    import ctypes
    import gen_golden
    from shmem_reduce import DTYPES
    L = shm.lib
    vp = ctypes.c_void_p
    L.mi355_nan_patch_copy.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_size_t, vp, vp]
    L.mi355_nan_patch_copy.restype = ctypes.c_int
    es = np.dtype(oracle.NP[dtype]).itemsize
    ut = np.uint32 if es == 4 else np.uint64
    quiet = ut(1 << 22) if es == 4 else ut(1 << 51)
    rng = np.random.default_rng(91)
    words = {v: _upload_at(dev, np.array([v], np.uint64), 0) for v in (0, 1)}
    # (48, 0), (72, 0): dst and peer off their 128-byte line, peeled to it
    for doff, ooff in ((0, 0), (es, 0), (0, 8), (8, es), (12 if es == 4 else 8, 4 if es == 4 else 0), (48, 0),
                       (72, 0)):
        for n in (1, 5, 1000, 70001):
            peer = gen_golden.values(rng, "sum", dtype, n)
            own = gen_golden.values(rng, "sum", dtype, n)
            pp, po = _upload_at(dev, peer, doff), _upload_at(dev, own, ooff)
            for flag in (None, 0, 1):
                d = dev.empty(n * es + 32) + doff
                rc = L.mi355_nan_patch_copy(DTYPES.index(dtype), d, pp, po, n, None if flag is None else words[flag],
                                            None)
                assert rc == 0, rc
                shm.sync()
                got = shm.get(d, n, dtype).view(ut)
                pb, ob = peer.view(ut), own.view(ut)
                want = pb if flag == 0 else np.where(np.isnan(own), ob | quiet, pb)
                assert (got == want).all(), (doff, ooff, n, flag, int(np.argmax(got != want)))
            dev.free()
            words = {v: _upload_at(dev, np.array([v], np.uint64), 0) for v in (0, 1)}
