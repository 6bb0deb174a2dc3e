// x80_host_check.cpp -- osss-gasnet_amd/csrc/x80.h (the GPU's x87 long double
// arithmetic in integer code) compiled for the CPU and checked bit for bit
// against the host's own x87 `long double` + and * (what the reference's
// reduce-op.c:99 element functions execute), on pairs aimed at both of its
// paths and the boundaries between them: exponent differences 0-3 and 0-70,
// fields near 1 and near the top, exact and near cancellation, random fields,
// powers of two and all-ones significands against operands 60-73 fields
// below (the fast add's sticky operand), significands that round up to a
// carry (the wrap).
// Built and run by tests/test_x80_host.py (CPU). usage: x80_host_check [pairs per case]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

#define __device__
#define __forceinline__ inline
#define __all(x) (x)
#define __builtin_clzg(x, z) ((x) != 0 ? __builtin_clzll(x) : (z))
#define __builtin_assume(c) ((void)0)
static inline uint64_t __umul64hi(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }
#include "x80.h"

static bool same(const x80 &a, long double v) {
    unsigned char w[10];
    memcpy(w, &v, 10);
    return memcmp(&a, w, 10) == 0;
}

int main(int argc, char **argv) {
    const long per = argc > 1 ? atol(argv[1]) : 1000000;
    std::mt19937_64 g(7);
    long bad = 0, n = 0;
    auto mk = [&](int e, int s) {
        x80 r;
        memset(&r, 0, sizeof r);
        r.m = g() | (1ull << 63);
        r.se = (uint16_t)((s << 15) | e);
        return r;
    };
    for (int round = 0; round < 8; ++round)
        for (long i = 0; i < per; ++i) {
            int ea, eb;
            switch (round) {
            case 0: ea = 100 + (int)(g() % 32500); eb = ea + (int)(g() % 7) - 3; break;
            case 1: ea = 16000 + (int)(g() % 800); eb = ea - (int)(g() % 71); break;
            case 2: ea = 1 + (int)(g() % 80); eb = 1 + (int)(g() % 80); break;
            case 3: ea = 0x7FF8 + (int)(g() % 7); eb = 0x3F80 + (int)(g() % 256); break;
            case 4: ea = 1 + (int)(g() % 0x7FFE); eb = 1 + (int)(g() % 0x7FFE); break;
            case 5: ea = 16383 + (int)(g() % 5); eb = ea; break;
            case 6: ea = 16000 + (int)(g() % 800); eb = ea - 60 - (int)(g() % 14); break;
            default: ea = 16383 + (int)(g() % 3); eb = ea - (int)(g() % 3); break;
            }
            if (eb < 1) eb = 1;
            if (eb > 0x7FFE) eb = 0x7FFE;
            x80 a = mk(ea, (int)(g() & 1)), b = mk(eb, (int)(g() & 1));
            if (round == 5) {  // b = -a with the low significand bits perturbed
                b.m = (a.m ^ (g() & 0xFFF)) | (1ull << 63);
                b.se = a.se ^ 0x8000;
            }
            if (round == 6) a.m = g() & 1 ? 1ull << 63 : ~0ull;
            if (round == 7) {  // all-ones high bits: sums and products that round up to 2^64
                a.m |= ~0ull << (g() % 20);
                b.m |= ~0ull << (g() % 20);
            }
            long double la, lb;
            memset(&la, 0, sizeof la);
            memset(&lb, 0, sizeof lb);
            memcpy(&la, &a, 10);
            memcpy(&lb, &b, 10);
            volatile long double s = la + lb, p = la * lb;
            ++n;
            if (!same(x80d::add(a, b), s)) {
                if (bad < 5) printf("add mismatch: case %d fields %d %d\n", round, ea, eb);
                ++bad;
            }
            if (!same(x80d::mul(a, b), p)) {
                if (bad < 5) printf("mul mismatch: case %d fields %d %d\n", round, ea, eb);
                ++bad;
            }
        }
    printf("%ld pairs, %ld mismatches\n", n, bad);
    // x80d::less against the host's x87 `<` (unordered -- NaN or an encoding
    // the 387 refuses -- compares false), over every encoding class: zeros,
    // denormals, pseudo-denormals, normals with near and far exponents and
    // equal significands, infinities, quiet/signalling NaNs, unnormals,
    // pseudo-infinities and pseudo-NaNs
    auto any = [&](int e0) {
        x80 r;
        memset(&r, 0, sizeof r);
        const int cls = (int)(g() % 11);
        int e = e0;
        uint64_t m = g() | (1ull << 63);
        switch (cls) {
        case 0: e = 0; m = 0; break;                                          // zero
        case 1: e = 0; m = g() >> (1 + g() % 63); break;                      // denormal
        case 2: e = 0; break;                                                 // pseudo-denormal
        case 3: e = 0x7FFF; m = 1ull << 63; break;                            // infinity
        case 4: e = 0x7FFF; m = (1ull << 63) | (g() >> 1) | 1; break;         // NaN, quiet or signalling
        case 5: e = 1 + (int)(g() % 0x7FFE); m = g() >> 1; break;             // unnormal
        case 6: e = 0x7FFF; m = g() >> 1; break;                              // pseudo-inf / pseudo-NaN
        default: break;                                                       // normal near e0
        }
        r.m = m;
        r.se = (uint16_t)(((g() & 1) << 15) | e);
        return r;
    };
    long nc = 0, badc = 0;
    for (long i = 0; i < per; ++i) {
        const int e0 = 1 + (int)(g() % 0x7FFE);
        x80 a = any(e0), b = any(e0 + (int)(g() % 3) - 1 < 1 ? 1 : e0);
        if (g() % 4 == 0) b = a;                                             // equal values
        if (g() % 8 == 0) { b = a; b.se ^= 0x8000; }                          // opposite signs, +-0
        long double la, lb;
        memset(&la, 0, sizeof la);
        memset(&lb, 0, sizeof lb);
        memcpy(&la, &a, 10);
        memcpy(&lb, &b, 10);
        const bool want = la < lb, want2 = lb < la;
        ++nc;
        if (x80d::less(a, b) != want || x80d::less(b, a) != want2) {
            if (badc < 5) printf("less mismatch: fields %04x %016llx vs %04x %016llx\n", a.se,
                                 (unsigned long long)a.m, b.se, (unsigned long long)b.m);
            ++badc;
        }
    }
    printf("compare: %ld pairs, %ld mismatches\n", nc, badc);
    // the general paths (x80d::add_general / mul_general, straight-line) on
    // operands of every encoding class, against the host's x87 + and *
    long ng = 0, badg = 0;
    for (long i = 0; i < per; ++i) {
        const int e0 = 1 + (int)(g() % 0x7FFE);
        x80 a = any(e0), b = any(g() % 2 ? e0 + (int)(g() % 140) - 70 : 1 + (int)(g() % 0x7FFE));
        if (b.se == 0 && b.m == 0 && g() % 2) b = a;
        long double la, lb;
        memset(&la, 0, sizeof la);
        memset(&lb, 0, sizeof lb);
        memcpy(&la, &a, 10);
        memcpy(&lb, &b, 10);
        volatile long double s = la + lb, p = la * lb;
        ++ng;
        if (!same(x80d::add_general(a, b), s) || !same(x80d::mul_general(a, b), p)) {
            if (badg < 5)
                printf("general mismatch: %04x %016llx, %04x %016llx\n", a.se, (unsigned long long)a.m, b.se,
                       (unsigned long long)b.m);
            ++badg;
        }
    }
    printf("general: %ld pairs, %ld mismatches\n", ng, badg);
    // two NaN operands (the 387's rule: two quiet or two signalling NaNs give
    // the larger significand, a signalling and a quiet NaN give the quiet one,
    // whatever the significands), quiet bits, signs and significands picked so
    // that the quieted significands are often equal or ordered either way;
    // and one NaN against a number, an infinity or a zero
    long nn = 0, badn = 0;
    for (long i = 0; i < per / 4; ++i) {
        const uint64_t base = (1ull << 63) | (g() >> 2) | 1;
        auto nan = [&](void) {
            x80 r;
            memset(&r, 0, sizeof r);
            uint64_t m = g() % 3 ? base : (1ull << 63) | (g() >> 2) | 1;
            m ^= (g() % 4 == 0) ? (g() & 0xFF) & ~1ull : 0;
            m |= (g() & 1) ? (1ull << 62) : 0;                                // quiet or signalling
            r.m = m;
            r.se = (uint16_t)(((g() & 1) << 15) | 0x7FFF);
            return r;
        };
        x80 a = nan(), b = g() % 4 ? nan() : any(1 + (int)(g() % 0x7FFE));
        if (g() % 2) { x80 t = a; a = b; b = t; }
        long double la, lb;
        memset(&la, 0, sizeof la);
        memset(&lb, 0, sizeof lb);
        memcpy(&la, &a, 10);
        memcpy(&lb, &b, 10);
        volatile long double s = la + lb, p = la * lb;
        ++nn;
        if (!same(x80d::add_general(a, b), s) || !same(x80d::mul_general(a, b), p)) {
            if (badn < 5)
                printf("NaN-pair mismatch: %04x %016llx, %04x %016llx\n", a.se, (unsigned long long)a.m, b.se,
                       (unsigned long long)b.m);
            ++badn;
        }
    }
    printf("NaN pairs: %ld pairs, %ld mismatches\n", nn, badn);
    return bad != 0 || badc != 0 || badg != 0 || badn != 0;
}
