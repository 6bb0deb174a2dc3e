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
//   * NaN operands propagate quietened (when both are NaN: the quiet one
//     beside a signalling one, else the one with the larger significand);
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
    return (a.hi < b.hi) | ((a.hi == b.hi) & (a.lo < b.lo));
}
// Everything below is straight-line code (selects, no branches): the
// general path runs with whole waves, and its earlier branchy form -- early
// returns per encoding class, shifts with `if` per range -- gave
// nondeterministic one- and two-ulp errors on gfx950 in a kernel that ran it
// on every lane (tools/x80_lane_probe.hip: ~0.7 % of 3-operand x87 products
// of random encodings, varying from run to run, while the straight-line fast
// path matched the host x87 on every element).
__device__ __forceinline__ int clz64(uint64_t x) { return x == 0 ? 64 : __builtin_clzll(x); }
// a >> s, a << s and the bits of a below position s, for s in [0, 255]
__device__ __forceinline__ u128 shr(u128 a, int s) {
    const int k = s & 63;
    const uint64_t hk = a.hi >> k, lk = a.lo >> k;
    const uint64_t in = (a.hi << 1) << (63 - k);  // a.hi << (64 - k); 0 for k = 0
    const bool ge64 = s >= 64, ge128 = s >= 128;
    return mk(ge64 ? 0 : hk, ge128 ? 0 : ge64 ? hk : (lk | in));
}
__device__ __forceinline__ u128 shl(u128 a, int s) {
    const int k = s & 63;
    const uint64_t hk = a.hi << k, lk = a.lo << k;
    const uint64_t in = (a.lo >> 1) >> (63 - k);  // a.lo >> (64 - k); 0 for k = 0
    const bool ge64 = s >= 64, ge128 = s >= 128;
    return mk(ge128 ? 0 : ge64 ? lk : (hk | in), ge64 ? 0 : lk);
}
__device__ __forceinline__ u128 low_bits(u128 a, int s) {
    const int k = s & 63;
    const uint64_t m = (~0ull >> 1) >> (63 - k);  // the low k bits
    const bool ge64 = s >= 64, ge128 = s >= 128;
    return mk(ge128 ? a.hi : ge64 ? (a.hi & m) : 0, ge64 ? a.lo : (a.lo & m));
}
__device__ __forceinline__ int msb(u128 a) {  // -1 for 0
    return a.hi != 0 ? 127 - clz64(a.hi) : 63 - clz64(a.lo);
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
// NaN result of an operation with at least one NaN operand, by the 387's
// rule: one NaN -> it, quieted; a signalling and a quiet NaN -> the quiet one,
// whatever the significands; two of the same kind -> the larger significand
// (equal: the positive one), quieted. (Before round 4 a signalling/quiet pair
// took the larger quieted significand too: tests/native/x80_host_check.cpp's
// NaN-pair loop pins the rule against the host x87.)
__device__ __forceinline__ x80 nan_result(const x80 &a, const x80 &b) {
    const bool na = is_nan(a), nb = is_nan(b);
    const bool qa = ((a.m >> 62) & 1) != 0, qb = ((b.m >> 62) & 1) != 0;
    const uint64_t ma = a.m | 0x4000000000000000ull, mb = b.m | 0x4000000000000000ull;
    const bool take_a = (na & nb) ? (qa != qb ? qa : ma != mb ? ma > mb : sign(a) == 0) : na;
    return quiet(pick(take_a, a, b));
}

__device__ __forceinline__ int exp_of(const x80 &a) {  // value = m * 2^E
    const int e = efield(a);
    return (e == 0 ? 1 : e) - kEOff;
}

// Round W * 2^Ew (+ sticky fraction below W's last bit) to 64 bits, RNE,
// with gradual underflow and overflow to infinity. W != 0 on the lanes
// whose result is used (callers select a special result for the others).
__device__ __forceinline__ x80 round_pack(int s, u128 W, int Ew, bool sticky, const x80 &padsrc) {
    const int L = msb(W);
    int E = Ew + L - 63;  // exponent with the leading bit at position 63
    int shift = L - 63;
    const bool under = E < kEmin;
    shift += under ? kEmin - E : 0;
    E = under ? kEmin : E;
    // shift <= 0: exact (W < 2^64 there; sticky bits, if any, are below half an ulp)
    const uint64_t m_exact = W.lo << ((shift < 0 ? -shift : 0) & 63);
    // shift > 0: the bits shifted out decide; beyond 128 everything is below half an ulp
    const int rs = shift <= 0 ? 0 : shift > 255 ? 255 : shift;
    const u128 rem = low_bits(W, rs);
    const u128 half = shl(mk(0, 1), rs > 0 ? rs - 1 : 0);
    uint64_t m = shift > 0 ? shr(W, rs).lo : m_exact;
    const bool tie = (rem.hi == half.hi) & (rem.lo == half.lo);
    const bool up = (shift > 0) & (rs <= 128) & (lt(half, rem) | (tie & (sticky | ((m & 1) != 0))));
    m += up ? 1 : 0;
    const bool wrap = up & (m == 0);  // carried out of 64 bits
    m = wrap ? 0x8000000000000000ull : m;
    E += wrap ? 1 : 0;
    const int ef = E + kEOff;
    const bool zero = m == 0, denormal = (m >> 63) == 0;  // denormal: E == kEmin
    const bool ovf = !denormal & (ef >= kEmaxField);
    return make(s, (zero | denormal) ? 0 : ovf ? kEmaxField : ef, zero ? 0 : ovf ? 0x8000000000000000ull : m, padsrc);
}

// Round-to-nearest-even of a 64-bit significand m with the 64 bits below it
// in rem (and a sticky bit beyond them): true when m must go up by one.
__device__ __forceinline__ bool round_up(uint64_t m, uint64_t rem, bool sticky) {
    constexpr uint64_t half = 0x8000000000000000ull;
    return rem > half || (rem == half && (sticky || (m & 1)));
}

// Fast path of add/mul: both operands normal with exponent fields in
// [1, kFastMax], so no rounding can overflow; the rest (zeros, denormals,
// infinities, NaNs, unsupported encodings, near-overflow exponents,
// exponent differences of 63-65, differences that cancel more than 64 bits,
// round ups that wrap the significand, results that would be denormal) takes
// the general path. Both paths round the exact result once, so they agree
// bit for bit where both apply.
constexpr int kFastMax = kEmaxField - 3;
__device__ __forceinline__ bool fast_operand(const x80 &a) {
    const int e = efield(a);
    return e >= 1 && e <= kFastMax && jbit(a);
}

// The fast paths run when every active lane of the wave can take them (one
// vote, a uniform branch); otherwise the whole wave takes the general path.
// (Round 2 attributed nondeterministic one-ulp errors to lanes diverging
// between the two paths; round 3 found them in the then-branchy general path
// itself, which is now straight-line. The vote stays: it keeps the common
// case to the fast path's instructions only.)
// A value of the fast paths' domain, unpacked: significand, exponent field,
// sign as a mask (0 or -1). A chain of operations (the every-member fold)
// keeps its accumulator in this form and packs once at the end.
struct xu {
    uint64_t m;
    int e;
    int s;
};
__device__ __forceinline__ xu unpack(const x80 &a) {
    return xu{a.m, a.se & 0x7FFF, (int)(int16_t)a.se >> 15};
}
__device__ __forceinline__ x80 pack(const xu &u, const x80 &padsrc) {
    x80 r = padsrc;  // the padding bytes of the slot the result goes to
    r.m = u.m;
    r.se = (uint16_t)((u.s & 0x8000) | u.e);
    return r;
}

// nhi rounded to nearest even by the bits below it, nlo: up when nlo is
// above half, or at half with nhi odd -- (nlo | (nhi & 1)) > half, the carry
// out of its sum with half - 1, added into nhi by the same carry chain.
__device__ __forceinline__ uint64_t round_even(uint64_t nhi, uint64_t nlo) {
    const unsigned __int128 N = ((unsigned __int128)nhi << 64) | (nlo | (nhi & 1));
    return (uint64_t)((N + 0x7FFFFFFFFFFFFFFFull) >> 64);
}

// The operations of a chain of up to STEPS of them whose operands pass
// chain_operand<OP, STEPS> stay in the fast path's exponent range without a
// check per step. Sums: fields in [kChainLo, kFastMax - STEPS]; a sum's field
// exceeds the larger operand's by at most 1, and a difference's falls at most
// 61 below it (add_fast_u: at most 63 leading zeros in the high word, two
// bits of headroom). Products: unbiased exponents within +-L, L =
// (kFastMax - kBias - STEPS) / (STEPS + 1); a product's unbiased exponent is
// the operands' sum plus 0 or 1.
constexpr int kChainLo = 64;
template <int OP, int STEPS>
__device__ __forceinline__ bool chain_operand(const x80 &a) {
    const int e = efield(a);
    if constexpr (OP == 0) {
        return (e >= kChainLo) & (e <= kFastMax - STEPS) & jbit(a);
    } else {
        constexpr int L = (kFastMax - kBias - STEPS) / (STEPS + 1);
        return ((unsigned)(e - (kBias - L)) <= 2u * L) & jbit(a);
    }
}

// a + b for operands of the fast domain (the caller checks them:
// fast_operand); true when the result is in it too (RANGE: including its
// exponent range; false: the caller bounds it, chain_operand).
template <bool RANGE = true>
__device__ __forceinline__ bool add_fast_u(const xu &a, const xu &b, xu &r) {
    // Straight-line, in a 128-bit frame with two bits of headroom: A (the
    // larger magnitude) at bits 125..62, B aligned below it by the exponent
    // difference dd -- exact for dd <= 62; for dd >= 66 B is under a quarter
    // ulp of A and only its sign matters to the rounding, so it becomes a
    // sticky 1 at bit 0 (dd 63-65: general path). A + B cannot carry out of
    // the frame, and its high word has at least one leading zero; one left
    // shift by them normalizes the sum or difference (a difference whose high
    // word cancels entirely takes the general path), one round to nearest
    // even (a round up that wraps the significand takes the general path).
    const int d = a.e - b.e;
    const bool a_big = (d > 0) | ((d == 0) & (a.m >= b.m));
    const uint64_t MA = a_big ? a.m : b.m, MB = a_big ? b.m : a.m;
    const int EA = a.e > b.e ? a.e : b.e;
    const int dd = d < 0 ? -d : d;
    const int k = dd < 62 ? dd : 62;
    // A - B = A + ~B + 1: the sign difference as a mask and a carry in
    const uint32_t M32 = (uint32_t)(a.s ^ b.s);
    const uint64_t M = ((uint64_t)M32 << 32) | M32;
    const unsigned __int128 A = (unsigned __int128)MA << 62;
    const unsigned __int128 B = ((unsigned __int128)((MB >> 2) >> k) << 64) | (dd >= 66 ? 1 : MB << (62 - k));
    const unsigned __int128 R = A + (B ^ (((unsigned __int128)M << 64) | M)) + (M & 1);
    const uint64_t Rh = (uint64_t)(R >> 64), Rl = (uint64_t)R;
    const int lz = __builtin_clzg(Rh, 64);  // Rh == 0: not ok below
    __builtin_assume(lz >= 1);
    const uint64_t nhi = (Rh << lz) | (Rl >> (64 - lz)), nlo = Rl << lz;
    const uint64_t m = round_even(nhi, nlo);
    const int E = EA + 2 - lz;
    r.m = m;
    r.e = E;
    r.s = a_big ? a.s : b.s;
    const bool ok = ((dd <= 62) | (dd >= 66)) & (Rh != 0) & (m != 0);
    if constexpr (RANGE) return ok & ((unsigned)(E - 1) < (unsigned)kFastMax);
    return ok;
}

__device__ __forceinline__ bool add_fast(const x80 &a, const x80 &b, x80 &r) {
    xu u;
    const int ok = add_fast_u(unpack(a), unpack(b), u);  // ints: evaluated without branches
    const int fa = fast_operand(a), fb = fast_operand(b);
    r = pack(u, a);
    return ok & fa & fb;
}

// The general paths: every encoding class, straight-line -- the finite
// result is computed for every lane and the special cases (in the 387's
// priority: unsupported encoding, NaN, infinity, zeros) replace it by selects.
__device__ __forceinline__ x80 add_general(const x80 &a, const x80 &b) {
    const int sa = sign(a), sb = sign(b);
    const int ia = is_inf(a), ib = is_inf(b), na = is_nan(a), nb = is_nan(b);  // ints: evaluated without branches
    const int ua = unsupported(a), ub = unsupported(b), za = is_zero(a), zb = is_zero(b);
    // finite: order by magnitude, A >= B; align B under A with a sticky bit
    const int ea = exp_of(a), eb = exp_of(b);
    const bool a_big = (ea > eb) | ((ea == eb) & (a.m >= b.m));
    const int EA = a_big ? ea : eb, EB = a_big ? eb : ea;
    const uint64_t MA = a_big ? a.m : b.m, MB = a_big ? b.m : a.m;
    const int sA = a_big ? sa : sb, sB = a_big ? sb : sa;
    const u128 WA = shl(mk(0, MA), 62), WB0 = shl(mk(0, MB), 62);  // 2 guard bits above, 62 below
    const int d = EA - EB > 255 ? 255 : EA - EB;
    const int sticky = !is0(low_bits(WB0, d));
    const u128 WB = shr(WB0, d);
    const u128 dif = sub(WA, WB);
    const u128 W = sA == sB ? add(WA, WB) : sticky ? sub(dif, mk(0, 1)) : dif;
    x80 r = round_pack(sA, W, EA - 62, sticky, a);
    const int cancel = is0(W);
    r = pick(cancel & !sticky, make(0, 0, 0, a), r);                          // exact cancellation: +0
    r = pick(za & zb, make(sa & sb, 0, 0, a), r);
    const x80 inf_r = pick(ia, a, make(sb, kEmaxField, 0x8000000000000000ull, a));
    r = pick(ia | ib, pick(ia & ib & (sa != sb), indefinite(a), inf_r), r);  // inf - inf: invalid
    r = pick(na | nb, nan_result(a, b), r);
    return pick(ua | ub, indefinite(a), r);
}

__device__ __forceinline__ x80 add(const x80 &a, const x80 &b) {
    x80 r = a;
    const bool ok = add_fast(a, b, r);
    if (__all(ok)) return r;
    return add_general(a, b);
}

// The 128-bit product of two 64-bit significands from 32-bit limbs, each
// partial product a 32 x 32 -> 64 multiply-add whose 64-bit addend carries the
// previous one's upper half (no sum overflows 64 bits: (2^32-1)^2 + 2 (2^32-1)
// = 2^64 - 1); the low word is assembled from the partial products' halves.
// (__umul64hi next to a * b compiled to the same four multiply-adds plus two
// 32-bit multiplies and an add recomputing the low word's upper half.)
__device__ __forceinline__ void mul64x64(uint64_t a, uint64_t b, uint64_t &hi, uint64_t &lo) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t p01 = (uint64_t)a0 * b1 + (p00 >> 32);
    const uint64_t p10 = (uint64_t)a1 * b0 + (uint32_t)p01;
    const uint64_t p11 = (uint64_t)a1 * b1 + (p01 >> 32);
    hi = p11 + (p10 >> 32);
    lo = (p10 << 32) | (uint32_t)p00;
}

template <bool RANGE = true>
__device__ __forceinline__ bool mul_fast_u(const xu &a, const xu &b, xu &r) {
    // straight-line like add_fast_u: the 128-bit product's leading bit is at
    // 127 or 126 (one conditional left shift, as a select), one rounding (a
    // round up that wraps the significand takes the general path)
    const int E = a.e + b.e - kBias + 1;  // biased exponent, leading bit at 127
    uint64_t hi, lo;
    mul64x64(a.m, b.m, hi, lo);
    const bool low = (hi >> 63) == 0;  // leading bit at 126
    const uint64_t nhi = low ? (hi << 1) | (lo >> 63) : hi;
    const uint64_t nlo = low ? lo << 1 : lo;
    const uint64_t m = round_even(nhi, nlo);
    r.m = m;
    r.e = E - (low ? 1 : 0);
    r.s = a.s ^ b.s;
    const bool ok = m != 0;
    if constexpr (RANGE) return ok & (E >= 2) & (E <= kFastMax);
    return ok;
}

__device__ __forceinline__ bool mul_fast(const x80 &a, const x80 &b, x80 &r) {
    xu u;
    const int ok = mul_fast_u(unpack(a), unpack(b), u);  // ints: evaluated without branches
    const int fa = fast_operand(a), fb = fast_operand(b);
    r = pack(u, a);
    return ok & fa & fb;
}

__device__ __forceinline__ x80 mul_general(const x80 &a, const x80 &b) {
    const int s = sign(a) ^ sign(b);
    const int za = is_zero(a), zb = is_zero(b), ia = is_inf(a), ib = is_inf(b);  // ints: no branches
    const int na = is_nan(a), nb = is_nan(b), ua = unsupported(a), ub = unsupported(b);
    uint64_t phi, plo;
    mul64x64(a.m, b.m, phi, plo);
    const u128 P = mk(phi, plo);
    x80 r = round_pack(s, P, exp_of(a) + exp_of(b), false, a);
    r = pick(za | zb, make(s, 0, 0, a), r);
    const x80 inf_r = pick(za | zb, indefinite(a), make(s, kEmaxField, 0x8000000000000000ull, a));  // 0 x inf
    r = pick(ia | ib, inf_r, r);
    r = pick(na | nb, nan_result(a, b), r);
    return pick(ua | ub, indefinite(a), r);
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
