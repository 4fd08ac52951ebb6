// yavo_fp64.h -- correctly rounded FP64 division and square root without the range handling the compiler's
// sequences carry for operands that need none.
//
// For a / b the compiler emits (gfx950, IEEE division):
//   s = v_div_scale(b), n = v_div_scale(a)             [both: the operand itself unless it must be rescaled]
//   r = v_rcp(s); e = fma(-s, r, 1); r = fma(r, e, r); e = fma(-s, r, 1); r = fma(r, e, r)
//   q = n * r; rem = fma(-s, q, n); q = v_div_fmas(rem, r, q)   [= fma(rem, r, q) when no operand was rescaled]
//   result = v_div_fixup(q, b, a)                       [= q unless an operand or the quotient is special]
// v_div_scale rescales only for a zero, denormal or near-overflow operand, an exponent gap of 768 or more, or a
// numerator below 2^-969; v_div_fixup changes q only for NaN / infinite / zero operands and over- / underflowing
// quotients.  With 2^-300 <= |a|, |b| < 2^301 none of these can happen, so the sequence below -- the same operations
// without the no-op scaling and fixup -- returns the compiler's result bit for bit; everything else takes the
// compiler's division.  The refined reciprocal r depends on b alone, so divisions by one denominator share it
// (Rcp64).  sqrt(x) likewise: the compiler's sequence rescales x < 2^-767 and passes 0 / +inf through a class test;
// for 2^-700 <= x < 2^1001 it is rsq + the two Goldschmidt / Newton corrections below.  tests/test_gpu_fp64.py
// compares every form with the compiler's operators on random and boundary operands (yv_debug_fp64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace yavo {
namespace fp64 {

// biased exponent field of x in [1023 - 300, 1023 + 300] (sign ignored): 2^-300 <= |x| < 2^301
__device__ __forceinline__ bool mid(double x) {
    const uint32_t e = ((uint32_t)__double2hiint(x) >> 20) & 0x7ffu;
    return e - 723u <= 600u;
}
// positive x with biased exponent in [323, 2023]: 2^-700 <= x < 2^1001
__device__ __forceinline__ bool sqrt_ok(double x) {
    const uint32_t e = (uint32_t)__double2hiint(x) >> 20;  // sign bit included: negative x fails
    return e - 323u <= 1700u;
}

__device__ __forceinline__ double rcp_refined(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    e = fma(-b, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ double div_r(double a, double b, double r) {
    const double q = a * r;
    const double rem = fma(-b, q, a);
    return fma(rem, r, q);
}

// a / b, bit-identical to the operator
__device__ __forceinline__ double div(double a, double b) {
    if (mid(a) && mid(b)) return div_r(a, b, rcp_refined(b));
    return a / b;
}
// 1 / b
__device__ __forceinline__ double rcp(double b) {
    if (mid(b)) return div_r(1.0, b, rcp_refined(b));
    return 1.0 / b;
}

// several divisions by one denominator: the refined reciprocal once
struct Rcp64 {
    double b = 1.0, r = 0.0;
    bool ok = false;
    Rcp64() = default;
    __device__ __forceinline__ explicit Rcp64(double den) : b(den), r(0.0), ok(mid(den)) {
        if (ok) r = rcp_refined(den);
    }
    __device__ __forceinline__ double div(double a) const {
        if (ok && mid(a)) return div_r(a, b, r);
        return a / b;
    }
};

// sqrt(x), bit-identical to the library's correctly rounded sqrt
__device__ __forceinline__ double sqrt(double x) {
    if (!sqrt_ok(x)) return ::sqrt(x);
    const double y = __builtin_amdgcn_rsq(x);
    double h = x * y, g = y * 0.5;
    const double e = fma(-g, h, 0.5);
    h = fma(h, e, h);
    g = fma(g, e, g);
    double d = fma(-h, h, x);
    h = fma(d, g, h);
    d = fma(-h, h, x);
    return fma(d, g, h);
}

}  // namespace fp64
}  // namespace yavo
