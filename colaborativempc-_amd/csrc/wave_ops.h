// Wave-level helpers shared by the solver kernels (one 64-lane wavefront = one agent).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace cmpc {

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void bar() { __syncthreads(); }

// One-wavefront workgroups: a wave's LDS operations execute in order, so an LDS hand-off
// between lanes needs only this compiler fence (no s_barrier, no counter drain — outstanding
// global prefetches stay in flight).
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    asm volatile("" ::: "memory");
}

// ... and a hand-off through global memory (stores by one lane, loads by another) drains the
// vector-memory counter first.
__device__ __forceinline__ void gsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Broadcast lane `lane` (must be wave-uniform) of a double to every lane (two v_readlane_b32).
__device__ __forceinline__ double readlane_d(double v, int lane) {
    long long i = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(i & 0xffffffffll), lane);
    int hi = __builtin_amdgcn_readlane((int)(i >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// NaN-propagating max: a NaN residual must never look converged (fmax drops NaNs).
__device__ __forceinline__ double nmax(double a, double b) { return (a > b || a != a) ? a : b; }

// Cross-lane reductions without LDS (a __shfl_xor of a double is two ds_bpermute plus a full
// lgkmcnt wait per step): DPP row rotations within a row of 16 lanes, then the permlane
// row swaps across rows.  Every stage combines commutatively, so all lanes end with the
// bit-identical value (the solver's wave-uniform decisions rely on it).
template <int N>
__device__ __forceinline__ double ror16(double x) {
    return __builtin_amdgcn_update_dpp(0.0, x, 0x120 + N, 0xF, 0xF, true);  // row_ror:N
}
template <class Op>
__device__ __forceinline__ double row_reduce(double v, Op op) {
    v = op(v, ror16<8>(v));
    v = op(v, ror16<4>(v));
    v = op(v, ror16<2>(v));
    return op(v, ror16<1>(v));
}
__device__ __forceinline__ double add_(double a, double b) { return a + b; }
__device__ __forceinline__ double min_(double a, double b) { return fmin(a, b); }
__device__ __forceinline__ double nmax_(double a, double b) { return nmax(a, b); }

__device__ __forceinline__ unsigned long long clock64_() { return __builtin_amdgcn_s_memtime(); }

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Lane J of each row of 16 lanes, broadcast to the whole row: one v_mov_b64_dpp row_newbcast:J
// (no SGPR round trip, unlike v_readlane).  Every lane reads a valid source lane, so the old
// value is dead: bound_ctrl with old = 0 lets the compiler drop the copy of x it otherwise
// makes into the destination first.  Call it with the whole wave active (never inside a
// divergent branch or select arm): a disabled source lane reads as 0.
template <int J>
__device__ __forceinline__ double bcast16(double x) {
    static_assert(J >= 0 && J < 16, "row_newbcast lane");
    return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + J, 0xF, 0xF, true);
}

// 1/sqrt(x) to full double precision: hardware estimate + two Newton steps.
__device__ __forceinline__ double rsqrt_d(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = y * fma(-0.5 * x, y * y, 1.5);
    y = y * fma(-0.5 * x, y * y, 1.5);
    return y;
}

// 1/x to full double precision: hardware estimate + two Newton steps (no IEEE divide sequence).
__device__ __forceinline__ double rcp_d(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    r = fma(r, fma(-x, r, 1.0), r);
    return r;
}

// CDNA4 row exchanges on doubles (one instruction per dword):
//  swap_half: lanes 32..63 of a <-> lanes 0..31 of b   (v_permlane32_swap)
//  swap_odd:  odd 16-lane rows of a <-> even rows of b  (v_permlane16_swap)
__device__ __forceinline__ void swap_half(double& a, double& b) {
    const unsigned long long ua = __builtin_bit_cast(unsigned long long, a);
    const unsigned long long ub = __builtin_bit_cast(unsigned long long, b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    a = __builtin_bit_cast(double, (unsigned long long)lo[0] | ((unsigned long long)hi[0] << 32));
    b = __builtin_bit_cast(double, (unsigned long long)lo[1] | ((unsigned long long)hi[1] << 32));
}
__device__ __forceinline__ void swap_odd(double& a, double& b) {
    const unsigned long long ua = __builtin_bit_cast(unsigned long long, a);
    const unsigned long long ub = __builtin_bit_cast(unsigned long long, b);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    a = __builtin_bit_cast(double, (unsigned long long)lo[0] | ((unsigned long long)hi[0] << 32));
    b = __builtin_bit_cast(double, (unsigned long long)lo[1] | ((unsigned long long)hi[1] << 32));
}

// over the 4 rows (lanes sharing l & 15)
template <class Op>
__device__ __forceinline__ double rows_reduce(double v, Op op) {
    double a = v, b = v;
    swap_odd(a, b);  // a: rows (0,0,2,2), b: rows (1,1,3,3)
    v = op(a, b);
    a = v;
    b = v;
    swap_half(a, b);  // a: rows (0,1,0,1), b: rows (2,3,2,3)
    return op(a, b);
}
__device__ __forceinline__ double wave_max(double v) { return rows_reduce(row_reduce(v, nmax_), nmax_); }
__device__ __forceinline__ double wave_min(double v) { return rows_reduce(row_reduce(v, min_), min_); }
__device__ __forceinline__ double wave_sum(double v) { return rows_reduce(row_reduce(v, add_), add_); }
// sum over the 16 lanes that share (lane >> 4)
__device__ __forceinline__ double sum16(double v) { return row_reduce(v, add_); }
// sum over the 4 lanes that share (lane & 15)
__device__ __forceinline__ double sum_groups(double v) { return rows_reduce(v, add_); }

// 4x4 transpose of (register, 16-lane row): on return r[t] holds, in row k, what r[k] held in
// row t.  With lane c carrying column c of a 4 x 64 matrix M in r[0..3], r[t] becomes the
// f64 16x16x4 MFMA fragment of the columns 16t..16t+15 (lane i + 16k: M[k][16t + i]).
__device__ __forceinline__ void transpose_rows4(double& r0, double& r1, double& r2, double& r3) {
    swap_half(r0, r2);
    swap_half(r1, r3);
    swap_odd(r0, r1);
    swap_odd(r2, r3);
}

}  // namespace cmpc
