// ops.h -- the reference's element operators on the GPU, shared by the
// combine kernels (combine.hip) and the fused small-message kernel (fused.hip).
// See combine.hip for the numerics notes (reduce-op.c:79-158).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "mi355_reduce.h"
#include "x80.h"

namespace mi355 {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct cplxf { float re, im; };
struct cplxd { double re, im; };

// ---------------------------------------------------------------------------
// element operators (reduce-op.c:79-158)
// ---------------------------------------------------------------------------
template <int OP, typename T>
__device__ __forceinline__ T int_op(T a, T b) {
    // 32-bit unsigned arithmetic for short/int, 64-bit for long/long long:
    // defined wrap-around, identical bits to gcc's add/imul on the host.
    using W = typename std::conditional<(sizeof(T) <= 4), uint32_t, uint64_t>::type;
    if constexpr (OP == MI355_OP_SUM) return (T)((W)a + (W)b);
    else if constexpr (OP == MI355_OP_PROD) return (T)((W)a * (W)b);
    else if constexpr (OP == MI355_OP_AND) return (T)(a & b);
    else if constexpr (OP == MI355_OP_OR) return (T)(a | b);
    else if constexpr (OP == MI355_OP_XOR) return (T)(a ^ b);
    else if constexpr (OP == MI355_OP_MIN) return a < b ? a : b;
    else return a > b ? a : b;
}

// The reference's float/double arithmetic is x86-64 SSE code (gcc -O2):
// `acc + src` is `addsd src, acc` with the accumulator as the FIRST source.
// Where a NaN comes out, SSE returns the first NaN operand, quieted, and an
// invalid operation (inf - inf, 0 * inf) gives the "real indefinite" QNaN,
// whose sign bit is SET. gfx950 propagates NaNs with its own operand choice
// (the compiler may commute) and produces +QNaN for invalid operations, so
// every NaN result is rewritten to SSE's: bit-exact NaN payloads and signs.
template <typename R> struct X86Nan;
template <> struct X86Nan<float> {
    using U = uint32_t;
    static constexpr U quiet = 0x00400000u, indefinite = 0xFFC00000u;
};
template <> struct X86Nan<double> {
    using U = uint64_t;
    static constexpr U quiet = 0x0008000000000000ull, indefinite = 0xFFF8000000000000ull;
};

// r = a <op> b computed by the GPU; the value SSE's `a <op> b` gives
template <typename R>
__device__ __forceinline__ R x86_result(R r, R a, R b) {
    using N = X86Nan<R>;
    using U = typename N::U;
    if (!__builtin_isnan(r)) return r;
    const U u = __builtin_isnan(a)   ? __builtin_bit_cast(U, a) | N::quiet
                : __builtin_isnan(b) ? __builtin_bit_cast(U, b) | N::quiet
                                     : N::indefinite;
    return __builtin_bit_cast(R, u);
}
template <typename R>
__device__ __forceinline__ R x86_indefinite_if_nan(R r) {
    return __builtin_isnan(r) ? __builtin_bit_cast(R, X86Nan<R>::indefinite) : r;
}

template <int OP, typename T>
__device__ __forceinline__ T fp_op(T a, T b) {
    if constexpr (OP == MI355_OP_SUM) return x86_result(a + b, a, b);
    else if constexpr (OP == MI355_OP_PROD) return x86_result(a * b, a, b);
    else if constexpr (OP == MI355_OP_MIN) return a < b ? a : b;
    else return a > b ? a : b;
}

// libgcc __muldc3/__mulsc3 (C99 Annex G.5.1) as compiled in this image (GCC
// 11, /lib/x86_64-linux-gnu/libgcc_s.so.1 and libgcc.a disassemble the same):
// ac = a*c, bd = b*d, ad = a*d, bc = c*b (c first), x = ac - bd, y = ad + bc,
// each an SSE scalar op (x86_result); then the recovery of infinities when
// both parts came out NaN. The recomputation's operands are never NaN (the
// recovery replaced them), so any NaN it makes is the invalid-operation QNaN.
// gcc's inline `a * b` calls this function whenever its own product has a NaN
// part (oracle o_prod_complex*, reduce-op.c:93-101), so these are the
// reference's bits in every case.
template <typename R>
__device__ __forceinline__ void cmul(R a, R b, R c, R d, R &x, R &y) {
    const R ac = x86_result(a * c, a, c), bd = x86_result(b * d, b, d);
    const R ad = x86_result(a * d, a, d), bc = x86_result(c * b, c, b);
    x = x86_result(ac - bd, ac, bd);
    y = x86_result(ad + bc, ad, bc);
    if (__builtin_isnan(x) && __builtin_isnan(y)) {
        bool recalc = false;
        const R inf = __builtin_inf();
        if (__builtin_isinf(a) || __builtin_isinf(b)) {
            a = __builtin_copysign(__builtin_isinf(a) ? R(1) : R(0), a);
            b = __builtin_copysign(__builtin_isinf(b) ? R(1) : R(0), b);
            if (__builtin_isnan(c)) c = __builtin_copysign(R(0), c);
            if (__builtin_isnan(d)) d = __builtin_copysign(R(0), d);
            recalc = true;
        }
        if (__builtin_isinf(c) || __builtin_isinf(d)) {
            c = __builtin_copysign(__builtin_isinf(c) ? R(1) : R(0), c);
            d = __builtin_copysign(__builtin_isinf(d) ? R(1) : R(0), d);
            if (__builtin_isnan(a)) a = __builtin_copysign(R(0), a);
            if (__builtin_isnan(b)) b = __builtin_copysign(R(0), b);
            recalc = true;
        }
        if (!recalc && (__builtin_isinf(ac) || __builtin_isinf(bd) ||
                        __builtin_isinf(ad) || __builtin_isinf(bc))) {
            if (__builtin_isnan(a)) a = __builtin_copysign(R(0), a);
            if (__builtin_isnan(b)) b = __builtin_copysign(R(0), b);
            if (__builtin_isnan(c)) c = __builtin_copysign(R(0), c);
            if (__builtin_isnan(d)) d = __builtin_copysign(R(0), d);
            recalc = true;
        }
        if (recalc) {
            x = x86_indefinite_if_nan(inf * (a * c - b * d));
            y = x86_indefinite_if_nan(inf * (a * d + b * c));
        }
    }
}

// Complex sum as gcc compiles reduce-op.c's `a + b` here: for double complex
// re = a.re + b.re, im = a.im + b.im; for float complex the imaginary add has
// the INCOMING operand first, im = b.im + a.im (`addss` order in the oracle's
// o_sum_complexf and in the golden build's fold, oracle/_ref/ref_ops.o) --
// which matters only for which NaN payload comes out.
template <int OP, typename C>
__device__ __forceinline__ C cplx_op(C a, C b) {
    C r;
    if constexpr (OP == MI355_OP_SUM) {
        r.re = x86_result(a.re + b.re, a.re, b.re);
        if constexpr (std::is_same<C, cplxf>::value) r.im = x86_result(b.im + a.im, b.im, a.im);
        else r.im = x86_result(a.im + b.im, a.im, b.im);
    } else {
        cmul(a.re, a.im, b.re, b.im, r.re, r.im);
    }
    return r;
}

// The reference's operator, bit for bit (NaN payloads included).
template <int OP, typename T>
__device__ __forceinline__ T apply(T a, T b) {
    if constexpr (std::is_same<T, cplxf>::value || std::is_same<T, cplxd>::value)
        return cplx_op<OP>(a, b);
    else if constexpr (std::is_same<T, x80>::value)
        return x80_op<OP>(a, b);
    else if constexpr (std::is_floating_point<T>::value)
        return fp_op<OP>(a, b);
    else
        return int_op<OP>(a, b);
}

// The streaming kernels' form: float/double/complex sum and product as the
// plain hardware operations (complex product without Annex G's recovery).
// A chain of these equals the chain of apply() unless a NaN comes out: a NaN
// operand or part stays NaN through every later plain add or product, so a
// chain whose result has no NaN part took no NaN, recovery or payload path
// at any step. redo_needed() tests that on the chain's result; a lane where it
// holds redoes its chain with apply() (rare and divergent: the other lanes
// skip the branch). Every other (op, type) is apply() itself.
template <int OP, typename T>
constexpr bool has_fast_form() {
    constexpr bool fp = std::is_same<T, float>::value || std::is_same<T, double>::value ||
                        std::is_same<T, cplxf>::value || std::is_same<T, cplxd>::value;
    return fp && (OP == MI355_OP_SUM || OP == MI355_OP_PROD);
}

template <int OP, typename T>
__device__ __forceinline__ T apply_fast(T a, T b) {
    if constexpr (!has_fast_form<OP, T>()) {
        return apply<OP>(a, b);
    } else if constexpr (std::is_floating_point<T>::value) {
        return OP == MI355_OP_SUM ? a + b : a * b;
    } else {
        T r;
        if constexpr (OP == MI355_OP_SUM) {
            r.re = a.re + b.re;
            r.im = a.im + b.im;
        } else {
            r.re = a.re * b.re - a.im * b.im;
            r.im = a.re * b.im + a.im * b.re;
        }
        return r;
    }
}

template <int OP, typename T>
__device__ __forceinline__ bool redo_needed(const T &r) {
    if constexpr (!has_fast_form<OP, T>()) return false;
    else if constexpr (std::is_floating_point<T>::value) return __builtin_isnan(r);
    else return __builtin_isnan(r.re) | __builtin_isnan(r.im);
}

// Which (op, type) pairs exist: reduce-op.c:405-448.
template <int OP, typename T>
constexpr bool valid_pair() {
    constexpr bool is_int = std::is_integral<T>::value;
    constexpr bool is_real = std::is_floating_point<T>::value || std::is_same<T, x80>::value;
    constexpr bool is_cplx = std::is_same<T, cplxf>::value || std::is_same<T, cplxd>::value;
    if (OP == MI355_OP_SUM || OP == MI355_OP_PROD) return is_int || is_real || is_cplx;
    if (OP == MI355_OP_AND || OP == MI355_OP_OR || OP == MI355_OP_XOR) return is_int;
    return is_int || is_real;  // min/max
}

template <typename T>
union Pack {
    u32x4 v;
    T e[16 / sizeof(T)];
};

}  // namespace mi355
