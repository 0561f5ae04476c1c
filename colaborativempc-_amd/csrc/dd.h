// Double-double arithmetic (value = hi + lo, |lo| <= ulp(hi)/2) built from error-free
// transformations: fma-based TwoProd and Knuth's TwoSum.  Used by the Riccati kernel's
// high-precision regime (mpc_riccati.hip), mirrored by oracle/cmpc_oracle.c (dd_t).
//
// Every function disables floating-point contraction: TwoSum/QuickTwoSum are exact only if
// each addition is rounded on its own, and a product fused into a later addition would
// break the TwoProd error term.
#pragma once
#include <hip/hip_runtime.h>

namespace cmpc {

struct dd {
    double hi, lo;
};

__device__ __forceinline__ dd dd_of(double a) { return {a, 0.0}; }

// |a| >= |b| (or a == 0): s + e == a + b exactly
__device__ __forceinline__ dd dd_qts(double a, double b) {
#pragma clang fp contract(off)
    const double s = a + b;
    return {s, b - (s - a)};
}

__device__ __forceinline__ dd dd_ts(double a, double b) {
#pragma clang fp contract(off)
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}

__device__ __forceinline__ dd dd_add(dd x, dd y) {
#pragma clang fp contract(off)
    const dd s = dd_ts(x.hi, y.hi);
    return dd_qts(s.hi, s.lo + x.lo + y.lo);
}

__device__ __forceinline__ dd dd_sub(dd x, dd y) { return dd_add(x, {-y.hi, -y.lo}); }

__device__ __forceinline__ dd dd_mul(dd x, dd y) {
#pragma clang fp contract(off)
    const double p = x.hi * y.hi;
    double e = __builtin_fma(x.hi, y.hi, -p);
    e = __builtin_fma(x.hi, y.lo, __builtin_fma(x.lo, y.hi, e));
    return dd_qts(p, e);
}

__device__ __forceinline__ dd dd_muld(dd x, double y) {
#pragma clang fp contract(off)
    const double p = x.hi * y;
    double e = __builtin_fma(x.hi, y, -p);
    e = __builtin_fma(x.lo, y, e);
    return dd_qts(p, e);
}

// acc + x*y
__device__ __forceinline__ dd dd_fma(dd acc, dd x, dd y) { return dd_add(acc, dd_mul(x, y)); }
__device__ __forceinline__ dd dd_fmad(dd acc, dd x, double y) { return dd_add(acc, dd_muld(x, y)); }
// acc + x*y for doubles x, y (exact product)
__device__ __forceinline__ dd dd_fmadd(dd acc, double x, double y) {
#pragma clang fp contract(off)
    const double p = x * y;
    return dd_add(acc, dd_qts(p, __builtin_fma(x, y, -p)));
}

__device__ __forceinline__ dd dd_div(dd x, dd y) {
#pragma clang fp contract(off)
    const double q1 = x.hi / y.hi;
    dd r = dd_sub(x, dd_muld(y, q1));
    const double q2 = r.hi / y.hi;
    r = dd_sub(r, dd_muld(y, q2));
    const double q3 = r.hi / y.hi;
    return dd_add(dd_qts(q1, q2), dd_of(q3));
}

__device__ __forceinline__ dd dd_sqrt(dd x) {
#pragma clang fp contract(off)
    const double s = __builtin_sqrt(x.hi);
    const dd r = dd_sub(x, dd_mul(dd_of(s), dd_of(s)));
    return dd_qts(s, r.hi / (2.0 * s));
}

// LDS storage: element i of a dd array lives at (p[2i], p[2i+1])
__device__ __forceinline__ dd ld_dd(const double* p, int i) { return {p[2 * i], p[2 * i + 1]}; }
__device__ __forceinline__ void st_dd(double* p, int i, dd v) {
    p[2 * i] = v.hi;
    p[2 * i + 1] = v.lo;
}

}  // namespace cmpc
