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

template <int OP, typename T>
__device__ __forceinline__ T fp_op(T a, T b) {
    if constexpr (OP == MI355_OP_SUM) return a + b;
    else if constexpr (OP == MI355_OP_PROD) return a * b;
    else if constexpr (OP == MI355_OP_MIN) return a < b ? a : b;
    else return a > b ? a : b;
}

// libgcc __muldc3/__mulsc3 (C99 Annex G.5.1): plain products, then recovery
// of infinities when both parts came out NaN.
template <typename R>
__device__ __forceinline__ void cmul(R a, R b, R c, R d, R &x, R &y) {
    R ac = a * c, bd = b * d, ad = a * d, bc = b * c;
    x = ac - bd;
    y = ad + bc;
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
            x = inf * (a * c - b * d);
            y = inf * (a * d + b * c);
        }
    }
}

template <int OP, typename C>
__device__ __forceinline__ C cplx_op(C a, C b) {
    C r;
    if constexpr (OP == MI355_OP_SUM) {
        r.re = a.re + b.re;
        r.im = a.im + b.im;
    } else {
        cmul(a.re, a.im, b.re, b.im, r.re, r.im);
    }
    return r;
}

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
