// Round 2 x80.h (branchy general path): the FIXTURE of the x87 co-residency
// investigation. Built into tools/x80_lane_probe_r2 (tools/Makefile),
// it is the control of tests/test_gpu_x87_coresidency.py: its general kernels
// return wrong x87 results in waves that share a SIMD with another wave
// (profiles/r04/x80/). Not product code; never linked into the library.
// x80.h -- x87 80-bit extended ("long double" on x86-64 Linux) arithmetic on
// the GPU, for shmem_longdouble_{sum,prod,min,max}_to_all.
//
// The reference's element functions (src/reduce/reduce-op.c:99 and :158) are
// `a + b`, `a * b`, `a < b ? a : b`, `a > b ? a : b` on long double, which gcc
// executes on the x87 FPU with its Linux default control word 0x037F: 64-bit
// significand precision, round-to-nearest-even, every exception masked. The
// device has no such unit, so this header restates that arithmetic in integer
// code:
//   * 16-byte slot: bytes 0-7 significand (explicit integer bit 63),
//     bytes 8-9 sign (bit 15) and biased exponent (15 bits, bias 16383),
//     bytes 10-15 padding (not part of the value);
//   * add/mul: exact result, rounded once to 64 significant bits with
//     gradual underflow (denormals) and overflow to infinity;
//   * operands the 387+ rejects (unnormals, pseudo-infinities, pseudo-NaNs)
//     and invalid operations (inf - inf, 0 * inf) give the x87 "real
//     indefinite" QNaN (sign 1, exponent 0x7FFF, significand 0xC000...);
//   * NaN operands propagate quietened (the one with the larger significand
//     when both are NaN);
//   * min/max select an operand's bits unchanged; an unordered compare is
//     false, so the second operand is returned (as on the host).
#pragma once
#include <stdint.h>

struct x80 {
    uint64_t m;      // significand, explicit integer bit at bit 63
    uint16_t se;     // sign << 15 | biased exponent
    uint16_t pad[3];
};

namespace x80d {

constexpr int kBias = 16383;
constexpr int kEmaxField = 0x7FFF;
// value = m * 2^E with E = max(e,1) - 16446 (16446 = bias + 63)
constexpr int kEOff = kBias + 63;
constexpr int kEmin = 1 - kEOff;  // exponent of the denormal / pseudo-denormal class

struct u128 {
    uint64_t hi, lo;
};

__device__ __forceinline__ u128 mk(uint64_t hi, uint64_t lo) { return u128{hi, lo}; }
__device__ __forceinline__ bool is0(u128 a) { return (a.hi | a.lo) == 0; }
__device__ __forceinline__ u128 add(u128 a, u128 b) {
    u128 r;
    r.lo = a.lo + b.lo;
    r.hi = a.hi + b.hi + (r.lo < a.lo ? 1 : 0);
    return r;
}
__device__ __forceinline__ u128 sub(u128 a, u128 b) {
    u128 r;
    r.lo = a.lo - b.lo;
    r.hi = a.hi - b.hi - (a.lo < b.lo ? 1 : 0);
    return r;
}
__device__ __forceinline__ bool lt(u128 a, u128 b) {
    return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo);
}
__device__ __forceinline__ u128 shl(u128 a, int s) {  // 0 <= s < 128
    if (s == 0) return a;
    if (s >= 64) return mk(a.lo << (s - 64), 0);
    return mk((a.hi << s) | (a.lo >> (64 - s)), a.lo << s);
}
__device__ __forceinline__ u128 shr(u128 a, int s) {  // 0 <= s < 128
    if (s == 0) return a;
    if (s >= 64) return mk(0, a.hi >> (s - 64));
    return mk(a.hi >> s, (a.lo >> s) | (a.hi << (64 - s)));
}
// Bits of a below bit position s (s in [1,128]).
__device__ __forceinline__ u128 low_bits(u128 a, int s) {
    if (s >= 128) return a;
    if (s >= 64) return mk(a.hi & ((s == 64) ? 0 : ((~0ull) >> (128 - s))), a.lo);
    return mk(0, a.lo & ((~0ull) >> (64 - s)));
}
__device__ __forceinline__ int msb(u128 a) {  // a != 0
    return a.hi ? 127 - __builtin_clzll(a.hi) : 63 - __builtin_clzll(a.lo);
}

__device__ __forceinline__ int efield(const x80 &a) { return a.se & 0x7FFF; }
__device__ __forceinline__ int sign(const x80 &a) { return a.se >> 15; }
__device__ __forceinline__ bool jbit(const x80 &a) { return (a.m >> 63) != 0; }

// Encodings the 387 and later refuse as operands (invalid operation).
__device__ __forceinline__ bool unsupported(const x80 &a) {
    const int e = efield(a);
    return (e != 0 && !jbit(a));  // unnormal, pseudo-infinity, pseudo-NaN
}
__device__ __forceinline__ bool is_nan(const x80 &a) {
    return efield(a) == kEmaxField && jbit(a) && (a.m << 1) != 0;
}
__device__ __forceinline__ bool is_inf(const x80 &a) {
    return efield(a) == kEmaxField && a.m == 0x8000000000000000ull;
}
__device__ __forceinline__ bool is_zero(const x80 &a) { return efield(a) == 0 && a.m == 0; }

// c ? a : b as masks on the two 64-bit words: a select of structs (or of
// their fields, which the compiler turns back into a select of their
// addresses) keeps both operands in scratch memory -- two scratch stores per
// operation in the fold loops.
__device__ __forceinline__ x80 pick(bool c, const x80 &a, const x80 &b) {
    const uint64_t k = 0ull - (uint64_t)c;
    uint64_t ah, bh;
    __builtin_memcpy(&ah, &a.se, 8);  // sign/exponent and padding
    __builtin_memcpy(&bh, &b.se, 8);
    x80 r;
    r.m = (a.m & k) | (b.m & ~k);
    const uint64_t h = (ah & k) | (bh & ~k);
    __builtin_memcpy(&r.se, &h, 8);
    return r;
}

__device__ __forceinline__ x80 make(int s, int e, uint64_t m, const x80 &padsrc) {
    x80 r = padsrc;  // keep the accumulator's padding bytes
    r.m = m;
    r.se = (uint16_t)((s << 15) | e);
    return r;
}
__device__ __forceinline__ x80 indefinite(const x80 &padsrc) {
    return make(1, kEmaxField, 0xC000000000000000ull, padsrc);
}
__device__ __forceinline__ x80 quiet(x80 a) {
    a.m |= 0x4000000000000000ull;
    return a;
}
// NaN result of an operation with at least one NaN operand.
__device__ __forceinline__ x80 nan_result(const x80 &a, const x80 &b) {
    const bool na = is_nan(a), nb = is_nan(b);
    if (na && nb) {
        const uint64_t ma = a.m | 0x4000000000000000ull, mb = b.m | 0x4000000000000000ull;
        if (ma != mb) return quiet(pick(ma > mb, a, b));
        return quiet(pick(sign(a) == 0, a, b));
    }
    return quiet(pick(na, a, b));
}

__device__ __forceinline__ int exp_of(const x80 &a) {  // value = m * 2^E
    const int e = efield(a);
    return (e == 0 ? 1 : e) - kEOff;
}

// Round W * 2^Ew (+ sticky fraction below W's last bit) to 64 bits, RNE,
// with gradual underflow and overflow to infinity.
__device__ __forceinline__ x80 round_pack(int s, u128 W, int Ew, bool sticky, const x80 &padsrc) {
    const int L = msb(W);
    int E = Ew + L - 63;  // exponent with the leading bit at position 63
    int shift = L - 63;
    if (E < kEmin) {
        shift += kEmin - E;
        E = kEmin;
    }
    uint64_t m;
    if (shift <= 0) {
        m = shl(W, -shift).lo;  // exact (sticky bits, if any, are < half an ulp: round down)
    } else {
        u128 rem;
        if (shift >= 128) {
            m = 0;
            rem = W;
        } else {
            m = shr(W, shift).lo;
            rem = low_bits(W, shift);
        }
        bool up;
        if (shift > 128) {
            up = false;  // everything is below half an ulp
        } else {
            const u128 half = shl(mk(0, 1), shift - 1);
            if (lt(half, rem)) up = true;
            else if (lt(rem, half)) up = false;
            else up = sticky || (m & 1);  // tie: to even unless something lies beyond
        }
        if (up) {
            m += 1;
            if (m == 0) {  // carried out of 64 bits
                m = 0x8000000000000000ull;
                E += 1;
            }
        }
    }
    if (m == 0) return make(s, 0, 0, padsrc);
    if ((m >> 63) == 0) return make(s, 0, m, padsrc);  // denormal (E == kEmin)
    const int ef = E + kEOff;
    if (ef >= kEmaxField) return make(s, kEmaxField, 0x8000000000000000ull, padsrc);
    return make(s, ef, m, padsrc);
}

// Round-to-nearest-even of a 64-bit significand m with the 64 bits below it
// in rem (and a sticky bit beyond them): true when m must go up by one.
__device__ __forceinline__ bool round_up(uint64_t m, uint64_t rem, bool sticky) {
    constexpr uint64_t half = 0x8000000000000000ull;
    return rem > half || (rem == half && (sticky || (m & 1)));
}

// Fast path of add/mul: both operands normal with exponent fields in
// [1, kFastMax], so every result is normal or an exact zero and no rounding
// can overflow; the rest (zeros, denormals, infinities, NaNs, unsupported
// encodings, near-overflow exponents, alignment shifts beyond 64 bits,
// results that would be denormal) takes the general path. Both paths round
// the exact result once, so they agree bit for bit where both apply.
constexpr int kFastMax = kEmaxField - 3;
__device__ __forceinline__ bool fast_operand(const x80 &a) {
    const int e = efield(a);
    return e >= 1 && e <= kFastMax && jbit(a);
}

// The fast paths run when every active lane of the wave can take them (one
// vote, a uniform branch); otherwise the whole wave takes the general path.
// (Diverging per lane between the two paths gave nondeterministic one-ulp
// errors in the general path's results on gfx950 -- test_longdouble_
// random_encodings -- so the choice is per wave.)
__device__ __forceinline__ bool add_fast(const x80 &a, const x80 &b, x80 &r) {
    // One straight-line path for effective addition and subtraction (every
    // choice a select; a branchy form diverged per lane on the operands'
    // signs, carries and cancellations, and the every-member fold ran both
    // sides of every branch): B aligned under A = MA:0 in 128 bits, exactly;
    // A + B, or A + (~B + 1) when the signs differ (A >= B, so no borrow out);
    // then one normalization: right by one on a carry out of the addition,
    // left by the leading zeros after a subtraction; one rounding.
    const int ea = efield(a), eb = efield(b);
    const bool a_big = (ea > eb) | ((ea == eb) & (a.m >= b.m));
    const int EA = a_big ? ea : eb;
    const int d = a_big ? ea - eb : eb - ea;
    const uint64_t MA = a_big ? a.m : b.m, MB = a_big ? b.m : a.m;
    const int sa = sign(a), sb = sign(b);
    const int sA = a_big ? sa : sb;
    const bool sub = sa != sb;
    const int dd = d < 64 ? d : 64;
    const uint64_t Bh = dd == 64 ? 0 : MB >> (dd & 63);
    const uint64_t Bl = dd == 0 ? 0 : MB << ((64 - dd) & 63);  // dd = 64: MB << 0 = MB
    const uint64_t lo = sub ? 0 - Bl : Bl;
    const uint64_t hi = MA + (sub ? ~Bh + (Bl == 0 ? 1 : 0) : Bh);
    const bool carry = !sub & (hi < MA);
    const bool zero = sub & (hi == 0) & (lo == 0);  // exact cancellation: +0
    // leading zeros of hi:lo after a subtraction (0 after an addition)
    const int lz = !sub ? 0 : hi != 0 ? __builtin_clzll(hi) : 64 + (lo != 0 ? __builtin_clzll(lo) : 63);
    const int l = lz & 63;
    // hi:lo << lz (lz in [0, 127]) or >> 1 (carry: the 129th bit comes back in at the top)
    const uint64_t sh_hi = lz >= 64 ? lo << l : l == 0 ? hi : (hi << l) | (lo >> (64 - l));
    const uint64_t sh_lo = lz >= 64 ? 0 : lo << l;
    const uint64_t nhi = carry ? (hi >> 1) | 0x8000000000000000ull : sh_hi;
    const uint64_t nlo = carry ? (lo >> 1) | (hi << 63) : sh_lo;
    const bool sticky = carry & ((lo & 1) != 0);
    int E = EA + (carry ? 1 : 0) - lz;
    const bool up = round_up(nhi, nlo, sticky);
    uint64_t m = nhi + (up ? 1 : 0);
    const bool wrap = up & (m == 0);
    m = wrap ? 0x8000000000000000ull : m;
    E += wrap ? 1 : 0;
    const int fa = fast_operand(a), fb = fast_operand(b);  // ints: evaluated without branches
    const bool ok = fa & fb & (d <= 64) & (zero | (E >= 1));
    r = zero ? make(0, 0, 0, a) : make(sA, E, m, a);
    return ok;
}

__device__ __forceinline__ x80 add_general(const x80 &a, const x80 &b) {
    if (unsupported(a) || unsupported(b)) return indefinite(a);
    if (is_nan(a) || is_nan(b)) return nan_result(a, b);
    const int sa = sign(a), sb = sign(b);
    if (is_inf(a) || is_inf(b)) {
        if (is_inf(a) && is_inf(b) && sa != sb) return indefinite(a);
        return pick(is_inf(a), a, make(sb, kEmaxField, 0x8000000000000000ull, a));
    }
    if (is_zero(a) && is_zero(b)) return make(sa & sb, 0, 0, a);
    // order by magnitude: A >= B
    const int ea = exp_of(a), eb = exp_of(b);
    const bool a_big = (ea > eb) || (ea == eb && a.m >= b.m);
    const int EA = a_big ? ea : eb, EB = a_big ? eb : ea;
    const uint64_t MA = a_big ? a.m : b.m, MB = a_big ? b.m : a.m;
    const int sA = a_big ? sa : sb, sB = a_big ? sb : sa;
    const u128 WA = shl(mk(0, MA), 62);
    u128 WB = shl(mk(0, MB), 62);
    bool sticky = false;
    const int d = EA - EB;
    if (d > 0) {
        if (d >= 128) {
            sticky = !is0(WB);
            WB = mk(0, 0);
        } else {
            sticky = !is0(low_bits(WB, d));
            WB = shr(WB, d);
        }
    }
    u128 W;
    if (sA == sB) {
        W = add(WA, WB);
    } else {
        W = sub(WA, WB);
        if (sticky) W = sub(W, mk(0, 1));
    }
    if (is0(W) && !sticky) return make(0, 0, 0, a);  // exact cancellation: +0
    return round_pack(sA, W, EA - 62, sticky, a);
}

__device__ __forceinline__ x80 add(const x80 &a, const x80 &b) {
    x80 r = a;
    const bool ok = add_fast(a, b, r);
    if (__all(ok)) return r;
    return add_general(a, b);
}

__device__ __forceinline__ bool mul_fast(const x80 &a, const x80 &b, x80 &r) {
    // straight-line like add_fast: the 128-bit product's leading bit is at
    // 127 or 126 (one conditional left shift, as a select), one rounding
    const int E = efield(a) + efield(b) - kBias + 1;  // biased exponent, leading bit at 127
    const uint64_t hi = __umul64hi(a.m, b.m), lo = a.m * b.m;
    const bool low = (hi >> 63) == 0;  // leading bit at 126
    const uint64_t nhi = low ? (hi << 1) | (lo >> 63) : hi;
    const uint64_t nlo = low ? lo << 1 : lo;
    int Ef = E - (low ? 1 : 0);
    const bool up = round_up(nhi, nlo, false);
    uint64_t m = nhi + (up ? 1 : 0);
    const bool wrap = up & (m == 0);
    m = wrap ? 0x8000000000000000ull : m;
    Ef += wrap ? 1 : 0;
    const int fa = fast_operand(a), fb = fast_operand(b);  // ints: evaluated without branches
    r = make(sign(a) ^ sign(b), Ef, m, a);
    return fa & fb & (E >= 2) & (E <= kFastMax);
}

__device__ __forceinline__ x80 mul_general(const x80 &a, const x80 &b) {
    if (unsupported(a) || unsupported(b)) return indefinite(a);
    if (is_nan(a) || is_nan(b)) return nan_result(a, b);
    const int s = sign(a) ^ sign(b);
    const bool ia = is_inf(a), ib = is_inf(b);
    if (ia || ib) {
        if (is_zero(a) || is_zero(b)) return indefinite(a);
        return make(s, kEmaxField, 0x8000000000000000ull, a);
    }
    if (is_zero(a) || is_zero(b)) return make(s, 0, 0, a);
    const u128 P = mk(__umul64hi(a.m, b.m), a.m * b.m);
    return round_pack(s, P, exp_of(a) + exp_of(b), false, a);
}

__device__ __forceinline__ x80 mul(const x80 &a, const x80 &b) {
    x80 r = a;
    const bool ok = mul_fast(a, b, r);
    if (__all(ok)) return r;
    return mul_general(a, b);
}

// a < b on the x87 (false when unordered: NaN or an unsupported encoding).
// Branch-free: a value orders by sign, then by (exponent, significand) --
// zero lowest (E = kEmin, m = 0; denormals share kEmin with the smallest
// normals and order below them by their cleared integer bit), infinity
// highest -- except that the two zeros are equal. (An early-return form
// diverged per lane and ran the every-member max at 8 sources 3.8x slower
// than the plain fold.)
__device__ __forceinline__ bool less(const x80 &a, const x80 &b) {
    const int ua = unsupported(a), ub = unsupported(b), na = is_nan(a), nb = is_nan(b);  // ints: no branches
    const int za = is_zero(a), zb = is_zero(b);
    const bool unordered = ua | ub | na | nb;
    const bool both_zero = za & zb;
    const int sa = sign(a), sb = sign(b);
    const int ea = is_inf(a) ? 0x10000 : exp_of(a), eb = is_inf(b) ? 0x10000 : exp_of(b);
    const bool mag_lt = (ea < eb) | ((ea == eb) & (a.m < b.m));
    const bool mag_gt = (ea > eb) | ((ea == eb) & (a.m > b.m));
    const bool lt = sa != sb ? sa == 1 : (sa == 0 ? mag_lt : mag_gt);
    return !unordered & !both_zero & lt;
}

}  // namespace x80d

template <int OP>
__device__ __forceinline__ x80 x80_op(x80 a, x80 b) {
    if constexpr (OP == 0) return x80d::add(a, b);          // MI355_OP_SUM
    else if constexpr (OP == 1) return x80d::mul(a, b);     // MI355_OP_PROD
    else if constexpr (OP == 5) return x80d::pick(x80d::less(a, b), a, b);  // MI355_OP_MIN
    else return x80d::pick(x80d::less(b, a), a, b);                   // MI355_OP_MAX: a > b
}
