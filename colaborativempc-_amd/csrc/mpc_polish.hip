// Active-set polish of condensed solves that stop at the rounding floor (CMPC_FLAG_POLISH).
//
// The reference solves every agent-QP with OSQP and `polish=True` (LPV_Planner.py:233): after the
// ADMM iterations, OSQP guesses the active set from the multipliers, solves the equality-
// constrained QP on it (a reduced KKT system) and keeps that point when its residuals are lower.
// This is the same step for the interior-point iterate.  A condensed kernel (mpc_ipm3.hip,
// mpc_ipm.hip) whose Newton matrix breaks down at the rounding floor (theta = lambda / t ~ 1e18 on
// the active rows: the merit is below 1e3 tol but not below tol, status 2) leaves its iterate in
// the rescue image (hand_doubles, internal.h) with flag 2 and its best merit in slot 1.  This
// kernel — one 256-thread workgroup per agent, every other workgroup returns at once — takes
// A = {r : lambda_r > t_r} as exact and solves
//     min f(U) + sum Qs sigma^2   s.t.   row_r(U, sigma) = w_r   (r in A)
// by Newton steps on its linear KKT system, in the range-space form:
//     H  = the condensed Hessian of f alone (2Q stage weights, 2R, 2dR; no theta: well conditioned),
//          H = L L' (LDS);
//     Y  = L^-1 G_A'  (G_A: the active rows as functions of U, c_r' Gamma_{k+1} or +-e_i, formed by
//          one adjoint recursion per row, psi_{j} = A_j' psi_{j+1}, g_j = B_j' psi_{j+1});
//     S  = Y'Y + E    (E: the slack coupling sign_r sign_r' / 2Qs_j within a slack group), S = M M';
//     z  = L^-1 rU,  S dlam = rA' - Y'z,  dU = -L^-T (z + Y dlam),
//     dsig = -(rsig + sign' dlam) / 2Qs,   rA' = rA - sign rsig / 2Qs.
// The polished point (t = 0 and lambda = max(lambda_A, 0) on A; t = max(w - row, 0) and lambda = 0
// elsewhere) replaces the returned solution when its merit max(res, 1e4 mu) is below the best
// merit the interior-point method reached — status 1 when below tol.  A second pass drops rows
// with a negative multiplier and adds violated ones (kPolishPasses).  oracle/cmpc_oracle.c
// restates it (polish_one) and the GPU tests compare the two.
#include "internal.h"
#include "wave_ops.h"

namespace cmpc {
namespace {

constexpr int kPT = 256;           // threads per workgroup (four waves)
constexpr int kPolishMaxActive = 96;
constexpr int kPolishSteps = 3;    // Newton steps on the (linear) KKT system: one solve, refinements while above tol
constexpr int kPolishPasses = 2;
constexpr int kLdG = 72;           // row stride of the H build's Gamma / 2Q Gamma images (2-way LDS banks)

struct PolLayout {
    int cst, Lh, Y, S, sA, sB, sC, sp, U, sig, Uc, sc, Ub, sb, X, ybar, w, lamp, tp, rp, rd, gU, rsig, zv,
        gz, rdH, rdS, lA, rA, dl, red, in, Ar;
    int amax, total;
};

__host__ __device__ inline PolLayout pol_layout_for(const MpcConst& c, int amax) {
    PolLayout L{};
    int o = 0;
    auto take = [&](int cnt) {
        const int at = o;
        o += (cnt + 1) & ~1;  // 16-byte alignment
        return at;
    };
    const int n = c.n, nx = c.nx, N = c.N, ns = c.ns, m = c.m;
    L.amax = amax;
    L.cst = take(mpc_const_used_doubles(c));
    const int mc = c.mc, nu = c.nu;
    L.Lh = take(n * (n + 1) / 2);                       // packed lower triangle
    L.Y = take(amax * (n | 1));  // rows at an odd stride (LDS banks)
    // S; also Gamma and 2Q Gamma while H is built (4 x KR x kLdG), and the one-wave Cholesky's scratch while
    // H is factored (wave_chol64: 4 x 272 + 3 x 272)
    const int sG = 4 * ((nx + 3) & ~3) * kLdG, sS = amax * (amax + 1) / 2;
    const int sS2 = sG > 8 * 272 ? sG : 8 * 272;  // (8 x 272: also the blocked Y solve's D_J and tiles)
    L.S = take(sS > sS2 ? sS : sS2);
    L.sA = take(N * nx * nx);                           // the agent's stage data, staged once
    L.sB = take(N * nx * nu);
    L.sC = take(N * mc * nx);
    L.sp = take((N + 1) * nx);
    L.U = take(n);
    L.sig = take(N * ns);
    L.Uc = take(n);
    L.sc = take(N * ns);
    L.Ub = take(n);
    L.sb = take(N * ns);
    L.X = take((N + 1) * nx);
    L.ybar = take((N + 1) * nx);
    L.w = take(m);
    L.lamp = take(m);
    L.tp = take(m);
    L.rp = take(m);
    L.rd = take(n);
    L.gU = take(n);
    L.rsig = take(N * ns);
    L.zv = take(n);
    L.gz = take(n);
    L.rdH = take(n);
    L.rdS = take(amax);
    L.lA = take(amax);
    L.rA = take(amax);
    L.dl = take(amax);
    L.red = take(16);
    L.in = take((m + 1) / 2);      // int flags
    L.Ar = take((amax + 1) / 2);   // int row indices
    L.total = o;
    return L;
}

__host__ __device__ inline PolLayout pol_layout(const MpcConst& c) {
    int amax = c.m < kPolishMaxActive ? c.m : kPolishMaxActive;
    PolLayout L = pol_layout_for(c, amax);
    while (amax > 8 && (size_t)L.total * sizeof(double) + 1024 > kMaxLdsBytes) {  // 1 KB: static LDS
        amax -= 8;
        L = pol_layout_for(c, amax);
    }
    return L;
}

// the (I, J) of lower 16 x 16 tile t in row-major order (I >= J)
__device__ __forceinline__ void tile_ij(int t, int& I, int& J) {
    I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    J = t - I * (I + 1) / 2;
}

// NaN-propagating block reductions over the four waves (scratch: 4 doubles)
__device__ double block_nmax(double v, double* red) {
    v = wave_max(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return nmax(nmax(red[0], red[1]), nmax(red[2], red[3]));
}
__device__ double block_sum(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[4 + (threadIdx.x >> 6)] = v;
    __syncthreads();
    return (red[4] + red[5]) + (red[6] + red[7]);
}

// In-place Cholesky of a packed lower n x n matrix, n <= 64, by wave 0 alone in the MFMA accumulator layout
// (the v3 kernel's factorisation, mpc_ipm3.hip): 16 x 16 tiles, padding rows the identity; each 16 x 16
// diagonal factor by DPP row broadcasts and rsq + Newton steps, the panel substitution in the accumulator
// layout, the trailing update on V_MFMA_F64_16X16X4_F64.  L overwrites M; rd receives 1 / L_ii.  Scratch: 7 x 272
// doubles of LDS.  Returns false when a pivot is not positive.  (Was the workgroup's four-column blocked
// factorisation, block_chol_packed, two barriers per block: 0.14 M clocks at n = 60.)
// (Out of line, so its registers stay out of the kernel's other sections; the operands are cast to the LDS
// address space, or the call's generic pointers would make every access a flat one.)
typedef __attribute__((address_space(3))) double lds_f64;
template <int T>  // 16 x 16 tiles per side: n <= 16 T
__device__ __attribute__((noinline)) bool wave_chol64(double* M_, double* rd_, int n, double* scratch) {
    const int l = threadIdx.x & 63;
    lds_f64* M = (lds_f64*)M_;
    lds_f64* rd = (lds_f64*)rd_;
    lds_f64* Ld = (lds_f64*)scratch;  // T x 16 x 17: the factored diagonal blocks
    lds_f64* SP = Ld + T * 272;       // (T - 1) x 16 x 17: the panel, for the transposed MFMA operands
    auto pk = [](int i, int j) { return i * (i + 1) / 2 + j; };
    v4d acc[T * (T + 1) / 2];
#pragma unroll
    for (int I = 0; I < T; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * I + (l >> 4) + 4 * r, col = 16 * J + (l & 15);
                const int a = row > col ? row : col, b2 = row > col ? col : row;
                const double v = M[pk(a < n ? a : 0, b2 < n ? b2 : 0)];
                acc[I * (I + 1) / 2 + J][r] = (row < n && col < n) ? v : (row == col ? 1.0 : 0.0);
            }
    bool ok = true;
#pragma unroll
    for (int J = 0; J < T; ++J) {
        const int JJ = J * (J + 1) / 2 + J;
        lds_f64* S0 = Ld + J * 272;
#pragma unroll
        for (int r = 0; r < 4; ++r) S0[((l >> 4) + 4 * r) * 17 + (l & 15)] = acc[JJ][r];
        wsync();
        double rw[16];
#pragma unroll
        for (int cc = 0; cc < 16; ++cc) rw[cc] = S0[(l & 15) * 17 + cc];
        {
            double dn = 0.0;
            static_for<0, 16>([&](auto jc) __attribute__((always_inline)) {
                constexpr int j = decltype(jc)::value;
                const double djj = bcast16<j>(j == 0 ? rw[0] : dn);
                if (!(djj > 0.0)) ok = false;
                const double y = rsqrt_d(djj);
                const double lj = rw[j] * y;
                rw[j] = lj;
                if constexpr (j + 1 < 16) dn = fma(-lj, lj, rw[j + 1]);
                static_for<j + 1, 16>([&](auto cc) __attribute__((always_inline)) {
                    constexpr int c2 = decltype(cc)::value;
                    rw[c2] = fma(-lj, bcast16<c2>(lj), rw[c2]);
                });
            });
        }
        if (l < 16) {
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) S0[l * 17 + cc] = (cc <= l) ? rw[cc] : 0.0;
        }
        wsync();
        if (J + 1 < T) {
            // panel: L_IJ = K_IJ L_JJ^-T (lane l: column l & 15 of every panel tile; unscaled form)
            const int i16 = l & 15;
            const double inv_own = 1.0 / S0[i16 * 17 + i16];
            static_for<0, 16>([&](auto jc) __attribute__((always_inline)) {
                constexpr int cc = decltype(jc)::value;
                const double dcc = bcast16<cc>(inv_own);
                const double lcc = (i16 > cc) ? rw[cc] * dcc : 0.0;
#pragma unroll
                for (int I = J + 1; I < T; ++I)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const double v = acc[I * (I + 1) / 2 + J][r];
                        acc[I * (I + 1) / 2 + J][r] = fma(-bcast16<cc>(v), lcc, v);
                    }
            });
#pragma unroll
            for (int I = J + 1; I < T; ++I)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[I * (I + 1) / 2 + J][r] *= inv_own;
#pragma unroll
            for (int I = J + 1; I < T; ++I)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    SP[((I - J - 1) * 16 + (l >> 4) + 4 * r) * 17 + (l & 15)] = acc[I * (I + 1) / 2 + J][r];
            wsync();
            // trailing update K_IK -= L_IJ L_KJ' (I >= K > J)
#pragma unroll
            for (int q = 0; q < 16; q += 4) {
                double fr[T];
#pragma unroll
                for (int I = J + 1; I < T; ++I) fr[I] = SP[((I - J - 1) * 16 + (l & 15)) * 17 + q + (l >> 4)];
#pragma unroll
                for (int I = J + 1; I < T; ++I)
#pragma unroll
                    for (int K2 = J + 1; K2 <= I; ++K2)
                        acc[I * (I + 1) / 2 + K2] =
                            __builtin_amdgcn_mfma_f64_16x16x4f64(-fr[I], fr[K2], acc[I * (I + 1) / 2 + K2], 0, 0, 0);
            }
            wsync();
        }
    }
    // L back into the packed storage: the off-diagonal tiles from the accumulators, the diagonal blocks from Ld
#pragma unroll
    for (int I = 1; I < T; ++I)
#pragma unroll
        for (int J = 0; J < I; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * I + (l >> 4) + 4 * r, col = 16 * J + (l & 15);
                if (row < n) M[pk(row, col)] = acc[I * (I + 1) / 2 + J][r];
            }
    for (int e = l; e < T * 256; e += kWave) {
        const int J = e >> 8, i = (e >> 4) & 15, j = e & 15, row = 16 * J + i, col = 16 * J + j;
        if (row < n && col <= row) M[pk(row, col)] = Ld[J * 272 + i * 17 + j];
    }
    wsync();
    for (int i = l; i < n; i += kWave) rd[i] = 1.0 / M[pk(i, i)];
    return ok;
}

// in-place Cholesky of an n x n matrix by the whole workgroup (packed lower storage, rows contiguous),
// blocked by four columns: wave 0 factors the four-column panel (compiler fences only), then the
// workgroup applies its rank-4 update to the trailing triangle as (row, 8-column chunk) items — two
// barriers per block instead of three per column.  Returns false when a pivot is not positive.
// (Tried: unblocked with three barriers per column, 1.6x slower; one wave with fences; the column
// in registers with readlane broadcasts, 2.4x slower still.)
// (Now only S beyond 64 active rows, or without room for wave_chol64's scratch.)
__device__ bool block_chol_packed(double* M, int n, int* flag) {
    const int tid = threadIdx.x;
    auto idx = [](int i, int j) { return i * (i + 1) / 2 + j; };
    for (int jb = 0; jb < n; jb += 4) {
        const int bw = n - jb < 4 ? n - jb : 4;
        if (tid < kWave) {  // panel: columns jb .. jb + bw - 1, rows jb .. n - 1
            int ok = 1;
            for (int j = jb; j < jb + bw; ++j) {
                const double d = M[idx(j, j)];
                if (!(d > 0.0)) {
                    ok = 0;
                    break;
                }
                const double sq = sqrt(d);
                const double inv = 1.0 / sq;
                wsync();
                if (tid == 0) M[idx(j, j)] = sq;
                for (int i = j + 1 + tid; i < n; i += kWave) M[idx(i, j)] *= inv;
                wsync();
                for (int i = j + 1 + tid; i < n; i += kWave) {  // the panel's later columns only
                    const double lij = M[idx(i, j)];
                    for (int p = j + 1; p < jb + bw && p <= i; ++p) M[idx(i, p)] -= lij * M[idx(p, j)];
                }
                wsync();
            }
            if (tid == 0) *flag = ok;
        }
        __syncthreads();
        if (!*flag) return false;  // uniform
        // trailing update: M[i][p] -= sum_c L[i][c] L[p][c], c in the panel, i >= p >= jb + bw
        const int j0 = jb + bw, rows = n - j0, chunks = (rows + 7) >> 3;
        for (int item = tid; item < rows * chunks; item += kPT) {
            const int i = j0 + item / chunks, p0 = j0 + 8 * (item % chunks);
            if (p0 > i) continue;
            double li[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) li[cc] = cc < bw ? M[idx(i, jb + cc)] : 0.0;
            double* r = M + idx(i, 0);
            const int pe = i + 1 < p0 + 8 ? i + 1 : p0 + 8;
            for (int p = p0; p < pe; ++p) {
                const double* lp = M + idx(p, jb);
                double v = r[p];
#pragma unroll
                for (int cc = 0; cc < 4; ++cc)
                    if (cc < bw) v -= li[cc] * lp[cc];
                r[p] = v;
            }
        }
        __syncthreads();
    }
    return true;
}

// forward substitution L x = b in place, wave 0 only: lane l holds x_l and x_{l+64}; the solved entry is
// broadcast by readlane (no LDS round trip in the chain); rd = the reciprocal diagonal.  The factor's
// entries and rd of eight pivots are loaded ahead of their eight chain steps (one LDS latency per group
// instead of one per pivot; the same operations in the same order).
template <class Idx>
__device__ void wave_fsub(const double* M, const double* rd, int n, Idx idx, double* x) {
    const int l = threadIdx.x & (kWave - 1);
    double x0 = l < n ? x[l] : 0.0, x1 = l + kWave < n ? x[l + kWave] : 0.0;
    for (int p0 = 0; p0 < n; p0 += 8) {
        double m0[8], m1[8], rp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int p = p0 + u;
            rp[u] = rd[p < n ? p : 0];
            m0[u] = (l > p && l < n) ? M[idx(l, p)] : 0.0;
            m1[u] = (l + kWave > p && l + kWave < n) ? M[idx(l + kWave, p)] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int p = p0 + u;
            if (p < n) {
                const double xp = (p < kWave ? readlane_d(x0, p) : readlane_d(x1, p - kWave)) * rp[u];
                if (l == p) x0 = xp;
                if (l + kWave == p) x1 = xp;
                if (l > p && l < n) x0 -= m0[u] * xp;
                if (l + kWave > p && l + kWave < n) x1 -= m1[u] * xp;
            }
        }
    }
    if (l < n) x[l] = x0;
    if (l + kWave < n) x[l + kWave] = x1;
}
// backward substitution L' x = b in place, wave 0 only (as above; row p of the factor is contiguous)
template <class Idx>
__device__ void wave_bsub(const double* M, const double* rd, int n, Idx idx, double* x) {
    const int l = threadIdx.x & (kWave - 1);
    double x0 = l < n ? x[l] : 0.0, x1 = l + kWave < n ? x[l + kWave] : 0.0;
    for (int p0 = n - 1; p0 >= 0; p0 -= 8) {
        double m0[8], m1[8], rp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int p = p0 - u;
            rp[u] = rd[p >= 0 ? p : 0];
            m0[u] = (l < p) ? M[idx(p, l)] : 0.0;
            m1[u] = (l + kWave < p) ? M[idx(p, l + kWave)] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int p = p0 - u;
            if (p >= 0) {
                const double xp = (p < kWave ? readlane_d(x0, p) : readlane_d(x1, p - kWave)) * rp[u];
                if (l == p) x0 = xp;
                if (l + kWave == p) x1 = xp;
                if (l < p) x0 -= m0[u] * xp;
                if (l + kWave < p) x1 -= m1[u] * xp;
            }
        }
    }
    if (l < n) x[l] = x0;
    if (l + kWave < n) x[l + kWave] = x1;
}

struct PolCtx {
    const MpcConst& c;
    int nx, nu;  // the state and input dimensions (compile-time constants in the NX / NU instantiations)
    const PolLayout& L;
    double* sm;
    const double* A;
    const double* B;
    const double* x0;
    const double* up;
    const double* pl;
    const double* C;
};

// n <= 64 forms of the two substitutions (H's factor, every condensed shape): x in one register, no branch
// on the pivot's register; the same operations in the same order as wave_fsub / wave_bsub.
template <class Idx>
__device__ void wave_fsub64(const double* M, const double* rd, int n, Idx idx, double* x) {
    const int l = threadIdx.x & (kWave - 1);
    double x0 = l < n ? x[l] : 0.0;
    for (int p0 = 0; p0 < n; p0 += 8) {
        double m0[8], rp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int p = p0 + u;
            rp[u] = rd[p < n ? p : 0];
            m0[u] = (l > p && l < n) ? M[idx(l, p)] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int p = p0 + u;
            if (p < n) {
                const double xp = readlane_d(x0, p) * rp[u];
                if (l == p) x0 = xp;
                if (l > p && l < n) x0 -= m0[u] * xp;
            }
        }
    }
    if (l < n) x[l] = x0;
}
template <class Idx>
__device__ void wave_bsub64(const double* M, const double* rd, int n, Idx idx, double* x) {
    const int l = threadIdx.x & (kWave - 1);
    double x0 = l < n ? x[l] : 0.0;
    for (int p0 = n - 1; p0 >= 0; p0 -= 8) {
        double m0[8], rp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int p = p0 - u;
            rp[u] = rd[p >= 0 ? p : 0];
            m0[u] = (l < p) ? M[idx(p, l)] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int p = p0 - u;
            if (p >= 0) {
                const double xp = readlane_d(x0, p) * rp[u];
                if (l == p) x0 = xp;
                if (l < p) x0 -= m0[u] * xp;
            }
        }
    }
    if (l < n) x[l] = x0;
}

// The stage recursions below run on wave 0 with the state (or costate) in lanes 0..nx-1 of a register and
// its entries broadcast by readlane: no LDS round trip or fence in the chain.  The next stage's A / B
// entries are loaded while a stage computes (two register sets, the loop unrolled by two), and each
// nx-term product runs as three partial sums (terms t = 0, 3, 6, ...; 1, 4, 7, ...; 2, 5, 8, ...) so
// the dependent chain is a third as long.  (Was an LDS form, one load latency inside every 9-term chain:
// 0.7 k clocks per stage.)

// the three partial sums of sum_t a[t] * v[t], t < nx, added in a fixed order
template <int M>
__device__ __forceinline__ double dot3(const double (&a)[M], const double (&v)[M], int nx) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int t = 0; t < M; t += 3) {
        if (t < nx) s0 = fma(a[t], v[t], s0);
        if (t + 1 < M && t + 1 < nx) s1 = fma(a[t + 1], v[t + 1], s1);
        if (t + 2 < M && t + 2 < nx) s2 = fma(a[t + 2], v[t + 2], s2);
    }
    return (s0 + s1) + s2;
}

// X = simulation of (x0, U) (wave 0; the other waves wait at the caller's barrier)
__device__ __forceinline__ void pol_fwd(const PolCtx& q, const double* U, double* X) {
    const MpcConst& c = q.c;
    const int nx = q.nx, nu = q.nu, N = c.N, l = threadIdx.x;
    if (l >= kWave) return;
    const int lr = l < nx ? l : 0;
    struct Set {
        double a[CMPC_MAX_NX], bu[CMPC_MAX_NU], u[CMPC_MAX_NU];
    };
    auto load = [&](Set& S, int k) {
        const int kk = k < N ? k : N - 1;  // (a clamped dummy past the horizon)
        const double* Ak = q.A + ((size_t)kk * nx + lr) * nx;
        const double* Bk = q.B + ((size_t)kk * nx + lr) * nu;
#pragma unroll
        for (int t = 0; t < CMPC_MAX_NX; ++t) S.a[t] = t < nx ? Ak[t] : 0.0;
#pragma unroll
        for (int i = 0; i < CMPC_MAX_NU; ++i) {
            S.bu[i] = i < nu ? Bk[i] : 0.0;
            S.u[i] = i < nu ? U[kk * nu + i] : 0.0;
        }
    };
    double x = q.x0[lr];
    if (l < nx) X[l] = x;
    auto stage = [&](const Set& S, int k) {
        double xs[CMPC_MAX_NX];
#pragma unroll
        for (int t = 0; t < CMPC_MAX_NX; ++t) xs[t] = t < nx ? readlane_d(x, t) : 0.0;
        double v = dot3(S.a, xs, nx);
#pragma unroll
        for (int i = 0; i < CMPC_MAX_NU; ++i)
            if (i < nu) v = fma(S.bu[i], S.u[i], v);
        x = v;
        if (l < nx) X[(k + 1) * nx + l] = v;
    };
    Set S0, S1;
    load(S0, 0);
    for (int k = 0; k < N; k += 2) {
        load(S1, k + 1);
        stage(S0, k);
        if (k + 1 >= N) break;
        load(S0, k + 2);
        stage(S1, k + 1);
    }
    wsync();
}

// out_k = B_k' psi_{k+1}, psi_N = y_N, psi_k = y_k + A_k' psi_{k+1} (wave 0; psi kept in y's slots,
// y is overwritten)
__device__ __forceinline__ void pol_adjoint(const PolCtx& q, double* y, double* out) {
    const MpcConst& c = q.c;
    const int nx = q.nx, nu = q.nu, N = c.N, l = threadIdx.x;
    if (l >= kWave) return;
    const int lr = l < nx ? l : 0, lb = l < nu ? l : 0;
    struct Set {
        double a[CMPC_MAX_NX], bc[CMPC_MAX_NX], yk;
    };
    auto load = [&](Set& S, int k) {
        const int kk = k >= 0 ? k : 0;
        const double* Ak = q.A + (size_t)kk * nx * nx;
        const double* Bk = q.B + (size_t)kk * nx * nu;
#pragma unroll
        for (int s2 = 0; s2 < CMPC_MAX_NX; ++s2) {
            S.a[s2] = s2 < nx ? Ak[s2 * nx + lr] : 0.0;
            S.bc[s2] = s2 < nx ? Bk[s2 * nu + lb] : 0.0;
        }
        S.yk = y[kk * nx + lr];
    };
    double psi = y[N * nx + lr];
    auto stage = [&](const Set& S, int k) {
        double ps[CMPC_MAX_NX];
#pragma unroll
        for (int s2 = 0; s2 < CMPC_MAX_NX; ++s2) ps[s2] = s2 < nx ? readlane_d(psi, s2) : 0.0;
        const double vo = dot3(S.bc, ps, nx);
        if (l < nu) out[k * nu + l] = vo;
        if (k > 0) {
            psi = S.yk + dot3(S.a, ps, nx);
            if (l < nx) y[k * nx + l] = psi;
        }
    };
    Set S0, S1;
    load(S0, N - 1);
    for (int k = N - 1; k >= 0; k -= 2) {
        load(S1, k - 1);
        stage(S0, k);
        if (k - 1 < 0) break;
        load(S0, k - 2);
        stage(S1, k - 1);
    }
    wsync();
}

// both residual adjoints of pol_residuals in one sweep: chain 0 (lanes 0..31) as pol_adjoint on y (out0 = gU),
// chain 1 (lanes 32..63) on y2 = y + C' lam on stages 1..N, formed as it goes (out1 = rd).
__device__ __forceinline__ void pol_adjoint2(const PolCtx& q, double* y, double* out0, double* out1, const double* lam) {
    const MpcConst& c = q.c;
    const int nx = q.nx, nu = q.nu, N = c.N, mc = c.mc, l = threadIdx.x;
    if (l >= kWave) return;
    const int ch = l >> 5, j = l & 31;
    const int lr = j < nx ? j : 0, lb = j < nu ? j : 0;
    auto y2 = [&](int k) {  // this lane's entry of y (chain 0) or y2 (chain 1) at stage k >= 1
        double v = y[k * nx + lr];
        if (ch)
            for (int r = 0; r < mc; ++r) v += lam[(k - 1) * mc + r] * q.C[((size_t)(k - 1) * mc + r) * nx + lr];
        return v;
    };
    struct Set {
        double a[CMPC_MAX_NX], bc[CMPC_MAX_NX], yk;
    };
    auto load = [&](Set& S, int k) {
        const int kk = k >= 0 ? k : 0;
        const double* Ak = q.A + (size_t)kk * nx * nx;
        const double* Bk = q.B + (size_t)kk * nx * nu;
#pragma unroll
        for (int s2 = 0; s2 < CMPC_MAX_NX; ++s2) {
            S.a[s2] = s2 < nx ? Ak[s2 * nx + lr] : 0.0;
            S.bc[s2] = s2 < nx ? Bk[s2 * nu + lb] : 0.0;
        }
        S.yk = kk > 0 ? y2(kk) : 0.0;
    };
    double psi = y2(N);
    auto stage = [&](const Set& S, int k) {
        double ps[CMPC_MAX_NX];
#pragma unroll
        for (int s2 = 0; s2 < CMPC_MAX_NX; ++s2) {
            const double p0 = s2 < nx ? readlane_d(psi, s2) : 0.0, p1 = s2 < nx ? readlane_d(psi, 32 + s2) : 0.0;
            ps[s2] = ch ? p1 : p0;
        }
        const double vo = dot3(S.bc, ps, nx);
        if (j < nu) (ch ? out1 : out0)[k * nu + j] = vo;
        if (k > 0) psi = S.yk + dot3(S.a, ps, nx);
    };
    Set S0, S1;
    load(S0, N - 1);
    for (int k = N - 1; k >= 0; k -= 2) {
        load(S1, k - 1);
        stage(S0, k);
        if (k - 1 < 0) break;
        load(S0, k - 2);
        stage(S1, k - 1);
    }
    wsync();
}

__device__ __forceinline__ double pol_row(const PolCtx& q, const double* X, const double* U, const double* sg, int r) {
    const MpcConst& c = q.c;
    const int nx = q.nx, mc = c.mc, ms = c.ms;
    if (r < ms) {
        const int k = r / mc, rr = r - k * mc;
        const double* cr = q.C + (size_t)r * nx;
        double v = 0.0;
        for (int s = 0; s < nx; ++s) v += cr[s] * X[(k + 1) * nx + s];
        const int j = c.row_slack[rr];
        if (j >= 0) v += c.row_sign[rr] * sg[k * c.ns + j];
        return v;
    }
    const int qq = r - ms;
    return (qq & 1) ? -U[qq >> 1] : U[qq >> 1];
}

// The interior-point residuals at (U, sigma, t, lambda) into rd / rsig / rp (cmpc_oracle.c merit_at);
// X is re-simulated when `sim` (otherwise X already holds U's states).  With `full`, returns the merit
// max(res, 1e4 mu) and *kkt = max(res, mu).
__device__ __forceinline__ double pol_residuals(const PolCtx& q, const double* U, const double* sg, const double* t,
                                const double* lam, const int* act_w, bool full, bool sim, double* kkt) {
    const MpcConst& c = q.c;
    const PolLayout& L = q.L;
    double* sm = q.sm;
    const int nx = q.nx, nu = q.nu, N = c.N, ns = c.ns, mc = c.mc, ms = c.ms, m = c.m, n = c.n;
    const int tid = threadIdx.x;
    double *X = sm + L.X, *ybar = sm + L.ybar, *rd = sm + L.rd, *gU = sm + L.gU, *rsig = sm + L.rsig,
           *rp = sm + L.rp, *red = sm + L.red;
    if (sim) {
        pol_fwd(q, U, X);
        __syncthreads();
    }
    auto ucost = [&](int k, int i) {
        double v = 0.0;
        for (int j = 0; j < nu; ++j) {
            const double du_k = U[k * nu + j] - (k ? U[(k - 1) * nu + j] : q.up[j]);
            const double du_n = (k + 1 < N) ? U[(k + 1) * nu + j] - U[k * nu + j] : 0.0;
            v += 2.0 * c.R[i * nu + j] * U[k * nu + j] + 2.0 * c.dR[i * nu + j] * (du_k - du_n);
        }
        return v;
    };
    double gscale = 1.0;
    if (full) {
        for (int e = tid; e < (N + 1) * nx; e += kPT) {
            const int k = e / nx, s = e - k * nx;
            double v = 2.0 * q.pl[e];
            for (int t2 = 0; t2 < nx; ++t2) v += 2.0 * c.Q[s * nx + t2] * X[k * nx + t2];
            ybar[e] = v;
        }
        __syncthreads();
        pol_adjoint2(q, ybar, gU, rd, lam);
        __syncthreads();
        double g_l = 0.0;
        for (int e = tid; e < n; e += kPT) g_l = nmax(g_l, fabs(gU[e] + ucost(e / nu, e % nu)));
        gscale = nmax(1.0, block_nmax(g_l, red));
    }
    for (int e = tid; e < (N + 1) * nx && !full; e += kPT) {
        const int k = e / nx, s = e - k * nx;
        double v = 2.0 * q.pl[e];
        for (int t2 = 0; t2 < nx; ++t2) v += 2.0 * c.Q[s * nx + t2] * X[k * nx + t2];
        if (k > 0)
            for (int r = 0; r < mc; ++r) v += lam[(k - 1) * mc + r] * q.C[((size_t)(k - 1) * mc + r) * nx + s];
        ybar[e] = v;
    }
    if (!full) {
        __syncthreads();
        pol_adjoint(q, ybar, rd);
        __syncthreads();
    }
    for (int e = tid; e < n; e += kPT) {
        const int k = e / nu, i = e - k * nu, r = ms + 2 * e;
        rd[e] += ucost(k, i) + lam[r] - lam[r + 1];
    }
    for (int e = tid; e < N * ns; e += kPT) {
        const int k = e / ns, j = e - k * ns;
        double v = 2.0 * c.Qs[j] * sg[e];
        for (int r = 0; r < mc; ++r)
            if (c.row_slack[r] == j) v += c.row_sign[r] * lam[k * mc + r];
        rsig[e] = v;
    }
    double nrp = 0.0, mu = 0.0, sp = 1.0, cnt = 0.0;
    for (int r = tid; r < m; r += kPT) {
        if (!(act_w[r] & 1)) { rp[r] = 0.0; continue; }
        const double w = sm[L.w + r];
        rp[r] = pol_row(q, X, U, sg, r) + t[r] - w;
        nrp = nmax(nrp, fabs(rp[r]));
        mu += t[r] * lam[r];
        sp = fmax(sp, fabs(w));
        cnt += 1.0;
    }
    __syncthreads();
    if (!full) return 0.0;
    double nrd = 0.0, nrs = 0.0;
    for (int e = tid; e < n; e += kPT) nrd = nmax(nrd, fabs(rd[e]));
    for (int e = tid; e < N * ns; e += kPT) nrs = nmax(nrs, fabs(rsig[e]));
    nrd = block_nmax(nrd, red);
    nrs = block_nmax(nrs, red);
    nrp = block_nmax(nrp, red);
    const double scale_p = block_nmax(sp, red);
    const double mact = block_sum(cnt, red);
    mu = block_sum(mu, red);
    mu = mact > 0.0 ? mu / mact : 0.0;
    const double res = nmax(nmax(nrd / gscale, nrs / c.qs_max), nrp / scale_p);
    if (tid == 0) {  // diagnostics (the stamps of mpc_polish_kernel)
        red[8] = nrd / gscale;
        red[9] = nrs / c.qs_max;
        red[10] = nrp / scale_p;
    }
    *kkt = nmax(res, mu);
    return nmax(res, 1e4 * mu);
}

// NXT, NUT: the state and input dimensions as compile-time constants (0: the runtime c.nx, c.nu)
template <int NXT, int NUT>
__global__ __launch_bounds__(kPT) void mpc_polish_kernel(const MpcConst c_arg, const MpcPtrs P) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    // with the compacted list (polish_list_kernel): workgroup i polishes the i-th flagged agent, so the
    // flagged agents start on distinct CUs at once instead of queueing behind each other
    int b = blockIdx.x;
    if (P.plist) {
        if (b >= P.plist[gridDim.x]) return;
        b = P.plist[b];
    }
    double* hd = P.ws + (size_t)b * c_arg.ws_stride;
    // flag 2: a final exit short of tol; flag 1: a condensed breakdown handed over to the Riccati
    // rescue — polished first, and handed over only when that does not reach tol
    const double flag = hd[0];
    if (flag != 2.0 && flag != 1.0) return;
    const int tid = threadIdx.x;
    const PolLayout L = pol_layout(c_arg);
    {
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&c_arg);
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(sm + L.cst);
        for (int i = tid; i < mpc_const_used_doubles(c_arg); i += kPT) dst[i] = src[i];
    }
    __syncthreads();
    const MpcConst& c = *reinterpret_cast<const MpcConst*>(sm + L.cst);
    const int nx = NXT ? NXT : c.nx, nu = NUT ? NUT : c.nu, N = c.N, ns = c.ns, mc = c.mc, ms = c.ms, m = c.m, n = c.n;
    const int amax = L.amax, ldY = n | 1;
    // the stage data (A, B, C rows, linear cost) staged in LDS once: every recursion below reads it
    {
        const double* gA = P.A + (size_t)b * N * nx * nx;
        const double* gB = P.B + (size_t)b * N * nx * nu;
        const double* gC = P.C + (size_t)b * N * mc * nx;
        const double* gp = P.p + (size_t)b * (N + 1) * nx;
        for (int i = tid; i < N * nx * nx; i += kPT) sm[L.sA + i] = gA[i];
        for (int i = tid; i < N * nx * nu; i += kPT) sm[L.sB + i] = gB[i];
        for (int i = tid; i < N * mc * nx; i += kPT) sm[L.sC + i] = gC[i];
        for (int i = tid; i < (N + 1) * nx; i += kPT) sm[L.sp + i] = gp[i];
    }
    const PolCtx q{c, nx, nu, L, sm, sm + L.sA, sm + L.sB, P.x0 + (size_t)b * nx, P.up + (size_t)b * nu, sm + L.sp, sm + L.sC};
    const double* hC = P.h + (size_t)b * N * mc;
    const double best_m = flag == 2.0 ? hd[1] : c_arg.tol;  // (flag 1: slot 1 holds the iterations done)
    const int ht = (int)hand_t(c);
    double *Lh = sm + L.Lh, *Y = sm + L.Y, *Sm = sm + L.S, *U = sm + L.U, *sig = sm + L.sig, *Uc = sm + L.Uc,
           *sc = sm + L.sc, *Ub = sm + L.Ub, *sb = sm + L.sb, *w = sm + L.w, *lamp = sm + L.lamp,
           *tp = sm + L.tp, *rp = sm + L.rp, *rd = sm + L.rd, *rsig = sm + L.rsig, *zv = sm + L.zv, *gz = sm + L.gz,
           *lA = sm + L.lA, *rA = sm + L.rA, *dl = sm + L.dl;
    int* in = reinterpret_cast<int*>(sm + L.in);
    int* Ar = reinterpret_cast<int*>(sm + L.Ar);
    // act flags: kept in the low bit of in[] (bit 1: in A)
    for (int r = tid; r < m; r += kPT) {
        double wr;
        if (r < ms) {
            wr = hC[r];
        } else {
            const int qq = r - ms, i = (qq >> 1) % nu;
            wr = (qq & 1) ? -c.u_lb[i] : c.u_ub[i];
        }
        const int act = isfinite(wr) ? 1 : 0;
        w[r] = act ? wr : 0.0;
        const double tr = hd[ht + r], lr = hd[ht + m + r];
        in[r] = act | ((act && lr > tr) ? 2 : 0);
    }
    for (int i = tid; i < n; i += kPT) U[i] = hd[2 + i];
    for (int i = tid; i < N * ns; i += kPT) sig[i] = hd[2 + n + i];
    for (int i = tid; i < n * (n + 1) / 2; i += kPT) Lh[i] = 0.0;
    int& nA_s = *reinterpret_cast<int*>(sm + L.red + 12);
    __syncthreads();
    // the active list (ascending rows), wave 0 by ballot; nA_s = |A| (rows past amax are not listed)
    auto active_list = [&]() {
        if (tid < kWave) {
            int base = 0;
            for (int r0 = 0; r0 < m; r0 += kWave) {
                const int r = r0 + tid;
                const bool f = r < m && (in[r] & 2);
                const unsigned long long msk = __ballot(f);
                const int pos = base + __popcll(msk & ((1ull << tid) - 1ull));
                if (f && pos < amax) Ar[pos] = r;
                base += __popcll(msk);
            }
            if (tid == 0) nA_s = base;
        }
        __syncthreads();
    };
    // pass 0's rows of G_A are formed in the H build below (c_r' Gamma_{k+1} at stage k, as
    // cmpc_oracle.c polish_one); the bound rows +-e_i here
    active_list();
    const int nA0 = nA_s;
    if (nA0 <= amax) {
        for (int e = tid; e < nA0 * ldY; e += kPT) {
            const int qa = e / ldY, i = e - qa * ldY, r = Ar[qa];
            double v = 0.0;
            if (r >= ms && i == ((r - ms) >> 1)) v = ((r - ms) & 1) ? -1.0 : 1.0;
            Y[e] = v;
        }
    }
    __syncthreads();
    // diagnostic section clocks (MpcPtrs::stamps slots 8..14, thread 0): init, H build, H factor,
    // G_A rows, Y, S build + factor + the Newton steps' linear algebra, the residual sweeps (simulation,
    // adjoints, reductions) of the Newton steps and evaluations; slot 4 bits 1..: Newton steps run
    // (slot 15 stays the solver's iteration count, kStampSlots - 1)
    unsigned long long tsum[7] = {0, 0, 0, 0, 0, 0, 0}, t_a = P.stamps ? clock64_() : 0;
#define PSTAMP(slot)                         \
    if (P.stamps && tid == 0) {              \
        const unsigned long long t_b = clock64_(); \
        tsum[slot] += t_b - t_a;             \
        t_a = t_b;                           \
    }
    PSTAMP(0);
#ifdef CMPC_POL_LAB  // lab: the clocks of a chosen region in slot 8 (CMPC_POL_LAB_REGION)
    unsigned long long lab_fwd = 0;
#endif
    // ---- H = sum_k Gamma_{k+1}' (2Q Gamma_{k+1}) + the 2R / 2dR band (lower triangle), H = L L' ----
    // (cmpc_oracle.c polish_one's build.)  Gamma_{k+1} = A_k Gamma_k + B_k E_k (nx x n, zero beyond column
    // (k + 1) nu) and W = 2Q Gamma_{k+1} are formed stage by stage in LDS ping-pong buffers (thread: column
    // l, rows wave + 4 i); the 16 x 16 lower tiles of H accumulate Gamma' W on V_MFMA_F64_16X16X4_F64 over
    // the nx rows (padded to 4), a wave holding up to three tiles in its accumulators through the horizon;
    // tiles whose Gamma columns are still zero are skipped.  (Was wave 0 alone: the backward recursion
    // S_k = 2Q + A_k' S_{k+1} A_k, then one lane per row of H carrying B_i' S_{i+1} A_i ... back over the
    // stages: 0.165 M clocks.)
    {
        const int KR = (nx + 3) & ~3;
        double* Gb = Sm;                      // Gamma_k, Gamma_{k+1}: 2 x KR x kLdG
        double* Wb = Sm + 2 * KR * kLdG;      // 2Q Gamma_{k+1}: KR x kLdG
        for (int i = tid; i < 4 * KR * kLdG; i += kPT) Sm[i] = 0.0;
        int qptr = 0;  // the first active row of pass 0 not yet formed (Ar ascending: stage by stage)
        const int T = (n + 15) >> 4, NT = T * (T + 1) / 2;
        const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;  // (wave-uniform)
        int tI[3], tJ[3];
#pragma unroll
        for (int sl = 0; sl < 3; ++sl) tile_ij(wv + 4 * sl < NT ? wv + 4 * sl : 0, tI[sl], tJ[sl]);
        v4d acc[3];
#pragma unroll
        for (int sl = 0; sl < 3; ++sl) acc[sl] = v4d{0.0, 0.0, 0.0, 0.0};
        // a diagonal Q (the reference's agent, the double integrators): the MFMA's B fragment is 2 Q_ss Gamma,
        // formed as it is loaded (the same rounding as the W sum, whose other terms are zeros) — no W phase
        bool qd_l = true;
        for (int i = l; i < nx * nx; i += kWave)
            if (i / nx != i % nx && c.Q[i] != 0.0) qd_l = false;
        const bool qd = __ballot(!qd_l) == 0ull;  // (wave-uniform; every wave reads the same Q)
        double qv[3];
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            const int s2 = 4 * ks + (l >> 4);
            qv[ks] = s2 < nx ? 2.0 * c.Q[s2 * nx + s2] : 0.0;
        }
        // Gamma_{k+1} from Gamma_k (ping-pong buffer k & 1 -> (k + 1) & 1; thread: column l, rows wv + 4 i)
        auto gamma_step = [&](int k) {
            const double* Gc = Gb + (k & 1) * KR * kLdG;
            double* Gn = Gb + ((k + 1) & 1) * KR * kLdG;
            const int ncol = (k + 1) * nu, j = l;
            if (j < ncol) {
                const double* Ak = q.A + k * nx * nx;
                const double* Bk = q.B + k * nx * nu;
                double gc[CMPC_MAX_NX];
#pragma unroll
                for (int t2 = 0; t2 < CMPC_MAX_NX; ++t2) gc[t2] = t2 < nx ? Gc[t2 * kLdG + j] : 0.0;
#pragma unroll
                for (int i = 0; i < 3; ++i) {  // rows wv, wv + 4, wv + 8: three independent chains
                    const int s2 = wv + 4 * i;
                    if (s2 < nx) {
                        double v = 0.0;
                        if (j >= k * nu) {
                            v = Bk[s2 * nu + (j - k * nu)];
                        } else {
#pragma unroll
                            for (int t2 = 0; t2 < CMPC_MAX_NX; ++t2)
                                if (t2 < nx) v += Ak[s2 * nx + t2] * gc[t2];
                        }
                        Gn[s2 * kLdG + j] = v;
                    }
                }
            }
        };
        __syncthreads();
        gamma_step(0);
        __syncthreads();
        // one barrier per stage: stage k's MFMAs and G_A rows read Gamma_{k+1} while the same phase forms
        // Gamma_{k+2} into the other buffer (Gamma_k's, read by nobody after the previous barrier)
        for (int k = 0; k < N; ++k) {
            const double* Gn = Gb + ((k + 1) & 1) * KR * kLdG;
            const int ncol = (k + 1) * nu, j = l;
            if (!qd) {  // W = 2Q Gamma_{k+1} (one buffer: the previous stage's MFMAs finished before the barrier)
                if (j < ncol) {
                    double gn[CMPC_MAX_NX];
#pragma unroll
                    for (int t2 = 0; t2 < CMPC_MAX_NX; ++t2) gn[t2] = t2 < nx ? Gn[t2 * kLdG + j] : 0.0;
                    for (int s2 = wv; s2 < nx; s2 += 4) {
                        double v = 0.0;
#pragma unroll
                        for (int t2 = 0; t2 < CMPC_MAX_NX; ++t2)
                            if (t2 < nx) v += 2.0 * c.Q[s2 * nx + t2] * gn[t2];
                        Wb[s2 * kLdG + j] = v;
                    }
                }
                __syncthreads();
            }
            // every fragment loaded first, then the next stage's Gamma, then the three tiles' MFMA chains
            double fa[3][3], fb[3][3];
            const double* Bsrc = qd ? Gn : Wb;
#pragma unroll
            for (int sl = 0; sl < 3; ++sl)
#pragma unroll
                for (int ks = 0; ks < 3; ++ks) {
                    const int row = (4 * ks + (l >> 4)) * kLdG;
                    const bool ld = wv + 4 * sl < NT && 16 * tI[sl] < ncol && 4 * ks < KR;
                    fa[sl][ks] = ld ? Gn[row + 16 * tI[sl] + (l & 15)] : 0.0;
                    fb[sl][ks] = ld ? Bsrc[row + 16 * tJ[sl] + (l & 15)] : 0.0;
                }
            if (k + 1 < N) gamma_step(k + 1);
            if (nA0 <= amax) {  // pass 0's active rows of stage k: g = c_r' Gamma_{k+1}
                // (this stage's rows follow qptr in Ar: counted by ballot over the next 64, every wave alike;
                // a stage holds at most mc <= 64 rows)
                const int qn = qptr + l;
                const bool at_k = qn < nA0 && Ar[qn] < ms && Ar[qn] / mc == k;
                const int q1 = qptr + __popcll(__ballot(at_k));
                for (int qa = qptr + wv; qa < q1; qa += kPT / kWave) {
                    if (j < ncol) {
                        const double* cr = q.C + (size_t)Ar[qa] * nx;
                        double v = 0.0;
#pragma unroll
                        for (int t2 = 0; t2 < CMPC_MAX_NX; ++t2)
                            if (t2 < nx) v += cr[t2] * Gn[t2 * kLdG + j];
                        Y[(size_t)qa * ldY + j] = v;
                    }
                }
                qptr = q1;
            }
            if (qd) {
#pragma unroll
                for (int sl = 0; sl < 3; ++sl)
#pragma unroll
                    for (int ks = 0; ks < 3; ++ks) fb[sl][ks] *= qv[ks];
            }
            // (unconditional: a tile or k-step without data has zero operands and adds zeros — no exec-mask
            // branches around the MFMAs, whose accumulators then stay in place)
#pragma unroll
            for (int ks = 0; ks < 3; ++ks)
#pragma unroll
                for (int sl = 0; sl < 3; ++sl)
                    acc[sl] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[sl][ks], fb[sl][ks], acc[sl], 0, 0, 0);
            __syncthreads();
        }
#pragma unroll
        for (int sl = 0; sl < 3; ++sl) {
            if (wv + 4 * sl < NT) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * tI[sl] + (l >> 4) + 4 * r, col = 16 * tJ[sl] + (l & 15);
                    if (row < n && col <= row) Lh[row * (row + 1) / 2 + col] = acc[sl][r];
                }
            }
        }
        __syncthreads();
        for (int ci = tid; ci < n; ci += kPT) {
            const int k = ci / nu, i = ci - k * nu;
            for (int j = 0; j < nu; ++j) {
                const int cj = k * nu + j;
                const double d = 2.0 * c.R[i * nu + j] + 2.0 * c.dR[i * nu + j] * (k + 1 < N ? 2.0 : 1.0);
                if (cj <= ci) Lh[ci * (ci + 1) / 2 + cj] += d;
                if (k > 0) Lh[ci * (ci + 1) / 2 + (k - 1) * nu + j] += -2.0 * c.dR[i * nu + j];
            }
        }
        __syncthreads();
    }
    PSTAMP(1);
    auto ih = [](int i, int j) { return i * (i + 1) / 2 + j; };
    auto is = [](int i, int j) { return i * (i + 1) / 2 + j; };
    int& flag_s = *reinterpret_cast<int*>(sm + L.red + 14);
    if (tid < kWave) {  // one wave, in the accumulators (n <= 64: every polished condensed shape)
        const bool ok = n <= 32 ? wave_chol64<2>(Lh, sm + L.rdH, n, Sm) : wave_chol64<4>(Lh, sm + L.rdH, n, Sm);
        if (tid == 0) flag_s = ok ? 1 : 0;
    }
    __syncthreads();
    const bool h_ok = flag_s != 0;
    PSTAMP(2);
    __syncthreads();
    double best = INFINITY, best_kkt = INFINITY;
    int passes = 0, nsteps = 0;
    for (int pass = 0; pass < kPolishPasses && h_ok; ++pass) {
        passes = pass + 1;
        if (pass) active_list();
        const int nA = nA_s;
        if (nA > amax) break;
        // later passes: G_A rows by adjoint recursions (one thread a row)
        for (int qa = pass ? tid : nA; qa < nA; qa += kPT) {
            const int r = Ar[qa];
            double* g = Y + (size_t)qa * ldY;
            for (int i = 0; i < n; ++i) g[i] = 0.0;
            if (r < ms) {
                const int k = r / mc;
                double psi[CMPC_MAX_NX], nps[CMPC_MAX_NX];
                for (int s = 0; s < nx; ++s) psi[s] = q.C[r * nx + s];
                for (int j = k; j >= 0; --j) {
                    const double* Bj = q.B + j * nx * nu;
                    for (int i = 0; i < nu; ++i) {
                        double v = 0.0;
                        for (int s = 0; s < nx; ++s) v += Bj[s * nu + i] * psi[s];
                        g[j * nu + i] = v;
                    }
                    if (j > 0) {
                        const double* Aj = q.A + j * nx * nx;
                        for (int t2 = 0; t2 < nx; ++t2) {
                            double v = 0.0;
                            for (int s = 0; s < nx; ++s) v += Aj[s * nx + t2] * psi[s];
                            nps[t2] = v;
                        }
                        for (int s = 0; s < nx; ++s) psi[s] = nps[s];
                    }
                }
            } else {
                const int qq = r - ms;
                g[qq >> 1] = (qq & 1) ? -1.0 : 1.0;
            }
        }
        __syncthreads();
        PSTAMP(3);
        // Y = G_A L^-T in place, blocked by 16 on V_MFMA_F64_16X16X4_F64: with D_J = L_JJ^-1 (the diagonal
        // 16 x 16 blocks' inverses, lane (J, c) substituting column c of block J; rows past n the identity),
        //     Y_J = (G_J - sum_{K<J} Y_K L_JK') D_J'
        // for each 16-row tile of the active rows (wave w: tiles w, w + 4, ...), J = 0 .. T-1.  S's region
        // is free until S is built: D_J at Sm (T x 16 x 17), each wave's staging tile after it.
        // (Was wave-level forward substitution of each row, 60 readlane-chained steps: 60 k clocks at |A| ~ 20;
        // before that one thread per row: 0.17 M.)
        {
            const int T = (n + 15) >> 4, RT = (nA + 15) >> 4;
            const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
            double* Dj = Sm;
            double* Ts = Sm + 4 * 272 + wv * 272;
            const double* rdH = sm + L.rdH;
            if (tid < kWave) {
                const int J = l >> 4, cc = l & 15;
                if (J < T) {
                    double x[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int gi = 16 * J + i;
                        double v = (i == cc) ? 1.0 : 0.0;
#pragma unroll
                        for (int p2 = 0; p2 < i; ++p2) {
                            const double lv = gi < n ? Lh[gi * (gi + 1) / 2 + 16 * J + p2] : 0.0;
                            v -= lv * x[p2];
                        }
                        x[i] = v * (gi < n ? rdH[gi] : 1.0);
                    }
#pragma unroll
                    for (int i = 0; i < 16; ++i) Dj[J * 272 + i * 17 + cc] = x[i];
                }
            }
            __syncthreads();
            for (int I = wv; I < RT; I += kPT / kWave) {
                for (int J = 0; J < T; ++J) {
                    v4d acc;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = 16 * I + (l >> 4) + 4 * r, col = 16 * J + (l & 15);
                        acc[r] = (row < nA && col < n) ? Y[(size_t)row * ldY + col] : 0.0;
                    }
                    for (int K = 0; K < J; ++K) {
                        double fa[4], fb[4];
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2) {
                            const int ra = 16 * I + (l & 15), rb = 16 * J + (l & 15), kc = 16 * K + 4 * s2 + (l >> 4);
                            fa[s2] = ra < nA ? -Y[(size_t)ra * ldY + kc] : 0.0;
                            fb[s2] = rb < n ? Lh[rb * (rb + 1) / 2 + kc] : 0.0;
                        }
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[s2], fb[s2], acc, 0, 0, 0);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) Ts[((l >> 4) + 4 * r) * 17 + (l & 15)] = acc[r];
                    wsync();
                    v4d yj = {0.0, 0.0, 0.0, 0.0};
                    {
                        double fa[4], fb[4];
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2) {
                            fa[s2] = Ts[(l & 15) * 17 + 4 * s2 + (l >> 4)];
                            fb[s2] = Dj[J * 272 + (l & 15) * 17 + 4 * s2 + (l >> 4)];
                        }
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2) yj = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[s2], fb[s2], yj, 0, 0, 0);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = 16 * I + (l >> 4) + 4 * r, col = 16 * J + (l & 15);
                        if (row < nA && col < n) Y[(size_t)row * ldY + col] = yj[r];
                    }
                    wsync();
                }
            }
        }
        __syncthreads();
        PSTAMP(4);
        // S = Y Y' + E (packed lower): the active rows' Gram matrix on V_MFMA_F64_16X16X4_F64.  16 x 16
        // tiles (I, J), I >= J, over nA padded to 16, dealt round-robin to the four waves, two tiles in
        // flight per wave (independent accumulator chains); k-steps of 4 over the n columns.  Both
        // operands of a k-step are the same fragment pattern: lane l holds Y[16 I + (l & 15)][4 s + (l >> 4)]
        // (A: 16 x 4 row block of Y; B: its transpose); D[i][j] sits at lane j + 16 (i & 3), register i >> 2.
        // (Was one thread per packed entry with an n-term LDS dot product: 0.15 M clocks at nA ~ 80.)
        {
            const int TA = (nA + 15) >> 4, NTt = TA * (TA + 1) / 2, KS = (n + 3) >> 2;
            const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63, i16 = l & 15, kq = l >> 4;
            auto frag = [&](int blk, int s) {
                const int row = 16 * blk + i16, col = 4 * s + kq;
                const double v = Y[(size_t)(row < nA ? row : 0) * ldY + (col < n ? col : 0)];
                return (row < nA && col < n) ? v : 0.0;
            };
            auto store = [&](int I, int J, const v4d& acc) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int a = 16 * I + kq + 4 * r, b2 = 16 * J + i16;
                    if (a < nA && b2 <= a) {
                        double v = acc[r];
                        const int ra = Ar[a], rb = Ar[b2];
                        if (ra < ms && rb < ms && ra / mc == rb / mc) {
                            const int j = c.row_slack[ra % mc];
                            if (j >= 0 && c.row_slack[rb % mc] == j)
                                v += c.row_sign[ra % mc] * c.row_sign[rb % mc] / (2.0 * c.Qs[j]);
                        }
                        Sm[a * (a + 1) / 2 + b2] = v;
                    }
                }
            };
            for (int t0 = 2 * wv; t0 < NTt; t0 += 2 * (kPT / kWave)) {
                int I0, J0, I1, J1;
                tile_ij(t0, I0, J0);
                const bool two = t0 + 1 < NTt;
                tile_ij(two ? t0 + 1 : t0, I1, J1);
                v4d a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
                for (int s = 0; s < KS; ++s) {
                    const double yi0 = frag(I0, s), yj0 = frag(J0, s), yi1 = frag(I1, s), yj1 = frag(J1, s);
                    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(yi0, yj0, a0, 0, 0, 0);
                    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(yi1, yj1, a1, 0, 0, 0);
                }
                store(I0, J0, a0);
                if (two) store(I1, J1, a1);
            }
        }
        __syncthreads();
        if (nA <= 64 && (amax - nA) * ldY >= 7 * 272) {  // (Y is live: the scratch is its rows past nA)
            if (tid < kWave) {
                double* chs = Y + (size_t)nA * ldY;
                const bool ok = nA <= 32 ? wave_chol64<2>(Sm, sm + L.rdS, nA, chs) : wave_chol64<4>(Sm, sm + L.rdS, nA, chs);
                if (tid == 0) flag_s = ok ? 1 : 0;
            }
        } else {
            const bool ok = block_chol_packed(Sm, nA, &flag_s);
            if (tid == 0) flag_s = ok ? 1 : 0;
            if (ok)
                for (int i = tid; i < nA; i += kPT) sm[L.rdS + i] = 1.0 / Sm[is(i, i)];
        }
        __syncthreads();
        PSTAMP(5);
        if (!flag_s) break;
        // Newton steps from (U, sigma, lambda_A)
        for (int i = tid; i < n; i += kPT) Uc[i] = U[i];
        for (int i = tid; i < N * ns; i += kPT) sc[i] = sig[i];
        for (int r = tid; r < m; r += kPT) {
            lamp[r] = 0.0;
            tp[r] = 0.0;
        }
        for (int qa = tid; qa < nA; qa += kPT) lA[qa] = hd[ht + m + Ar[qa]];
        __syncthreads();
        double mp = INFINITY, kk = INFINITY;
        for (int step = 0; step < kPolishSteps; ++step) {
            for (int r = tid; r < m; r += kPT) tp[r] = 0.0;
            for (int qa = tid; qa < nA; qa += kPT) lamp[Ar[qa]] = lA[qa];
            __syncthreads();
            double kk0;
            // t = 0: rp = row - w on A (X: Uc's states after the first step, left by the evaluation below)
            PSTAMP(5);
            pol_residuals(q, Uc, sc, tp, lamp, in, false, step == 0, &kk0);
            PSTAMP(6);
            for (int qa = tid; qa < nA; qa += kPT) {
                const int r = Ar[qa];
                double ra = rp[r];
                if (r < ms) {
                    const int j = c.row_slack[r % mc];
                    if (j >= 0) ra -= c.row_sign[r % mc] * rsig[(r / mc) * ns + j] / (2.0 * c.Qs[j]);
                }
                rA[qa] = ra;
            }
            for (int i = tid; i < n; i += kPT) zv[i] = rd[i];
            __syncthreads();
            if (tid < kWave) wave_fsub64(Lh, sm + L.rdH, n, ih, zv);  // z = L^-1 rU
            __syncthreads();
            for (int qa = tid; qa < nA; qa += kPT) {
                double v = rA[qa];
                for (int i = 0; i < n; ++i) v -= Y[(size_t)qa * ldY + i] * zv[i];
                dl[qa] = v;
            }
            __syncthreads();
            if (tid < kWave) {
                if (nA <= 64) {
                    wave_fsub64(Sm, sm + L.rdS, nA, is, dl);
                    wave_bsub64(Sm, sm + L.rdS, nA, is, dl);
                } else {
                    wave_fsub(Sm, sm + L.rdS, nA, is, dl);
                    wave_bsub(Sm, sm + L.rdS, nA, is, dl);
                }
            }
            __syncthreads();
            for (int i = tid; i < n; i += kPT) {  // z + Y dlam
                double v = zv[i];
                for (int qa = 0; qa < nA; ++qa) v += Y[(size_t)qa * ldY + i] * dl[qa];
                gz[i] = v;
            }
            __syncthreads();
            if (tid < kWave) wave_bsub64(Lh, sm + L.rdH, n, ih, gz);  // H^-1 (rU + G_A' dlam)
            __syncthreads();
            for (int i = tid; i < n; i += kPT) Uc[i] -= gz[i];
            for (int e = tid; e < N * ns; e += kPT) {
                const int k = e / ns, j = e - k * ns;
                double v = rsig[e];
                for (int qa = 0; qa < nA; ++qa) {
                    const int r = Ar[qa];
                    if (r < ms && r / mc == k && c.row_slack[r % mc] == j) v += c.row_sign[r % mc] * dl[qa];
                }
                sc[e] -= v / (2.0 * c.Qs[j]);
            }
            for (int qa = tid; qa < nA; qa += kPT) lA[qa] += dl[qa];
            __syncthreads();
            // the polished point as an interior-point iterate: t = 0 and lambda = max(lambda_A, 0) on A,
            // t = max(w - row, 0) and lambda = 0 elsewhere; one Newton step normally reaches tol, a
            // refinement step follows only when it does not
            PSTAMP(5);
#if defined(CMPC_POL_LAB) && CMPC_POL_LAB == 2
            const unsigned long long t_f0 = clock64_();
#endif
            pol_fwd(q, Uc, sm + L.X);
            __syncthreads();
#if defined(CMPC_POL_LAB) && CMPC_POL_LAB == 2
            lab_fwd = clock64_() - t_f0;
#endif
            PSTAMP(6);
            for (int r = tid; r < m; r += kPT) {
                lamp[r] = 0.0;
                tp[r] = ((in[r] & 1) && !(in[r] & 2)) ? fmax(w[r] - pol_row(q, sm + L.X, Uc, sc, r), 0.0) : 1.0;
            }
            __syncthreads();  // the active rows' entries below overwrite the defaults above
            for (int qa = tid; qa < nA; qa += kPT) {
                lamp[Ar[qa]] = fmax(lA[qa], 0.0);
                tp[Ar[qa]] = 0.0;
            }
            __syncthreads();
            PSTAMP(5);
            mp = pol_residuals(q, Uc, sc, tp, lamp, in, true, false, &kk);  // (X: pol_fwd above)
            PSTAMP(6);
            ++nsteps;
            if (mp < c.tol) break;
        }
        PSTAMP(5);
        if (mp < best) {
            best = mp;
            best_kkt = kk;
            for (int i = tid; i < n; i += kPT) Ub[i] = Uc[i];
            for (int i = tid; i < N * ns; i += kPT) sb[i] = sc[i];
        }
        // the next pass's active set: violated rows join it, negative multipliers leave it (X: Uc's)
        int ch = 0;
        for (int r = tid; r < m; r += kPT)
            if ((in[r] & 1) && !(in[r] & 2) && w[r] - pol_row(q, sm + L.X, Uc, sc, r) < 0.0) ch = 1;
        for (int qa = tid; qa < nA; qa += kPT)
            if (lA[qa] < 0.0) ch = 1;
        const int changed = __syncthreads_or(ch);
        if (!changed) break;
        for (int r = tid; r < m; r += kPT)
            if ((in[r] & 1) && !(in[r] & 2) && w[r] - pol_row(q, sm + L.X, Uc, sc, r) < 0.0) in[r] |= 2;
        __syncthreads();  // (the loop above reads the active bits the one below clears)
        for (int qa = tid; qa < nA; qa += kPT)
            if (lA[qa] < 0.0) in[Ar[qa]] &= ~2;
        __syncthreads();
    }
    __syncthreads();
    // diagnostics (MpcPtrs::stamps, tools/polish_diag.py, tools/polish_stamps.py): [passes run, |A| of the
    // last, polished merit, the method's best merit, H factored | Newton steps << 1, three reductions, the
    // section clocks]; slot 15 (the solver's iteration count) is left alone
    if (P.stamps && tid == 0) {
        unsigned long long* st = P.stamps + (size_t)b * kStampSlots;
        st[0] = (unsigned long long)passes;
        st[1] = (unsigned long long)nA_s;
        st[2] = (unsigned long long)__double_as_longlong(best);
        st[3] = (unsigned long long)__double_as_longlong(best_m);
        st[4] = (h_ok ? 1ull : 0ull) | ((unsigned long long)nsteps << 1);
        for (int i = 0; i < 3; ++i) st[5 + i] = (unsigned long long)__double_as_longlong(sm[L.red + 8 + i]);
#ifdef CMPC_POL_LAB
        st[7] = lab_fwd;
#endif
        for (int i = 0; i < 7; ++i) st[8 + i] = tsum[i];
    }
    // kept only when it beats the method's best AND lands at the rounding floor at least (stop_status's
    // 1e3 tol): below tol it is solved (1), below the floor solved-inaccurate (2).  A polish of a solve
    // that ended far from the floor (a cold-pass stall, a max-iteration exit) never turns it into a 2,
    // which the reference would count as feasible (LPV_Planner.py:243-249): status and z stay as they were
    if (!(best < best_m) || !(best < 1e3 * c.tol)) {
        if (tid == 0 && flag == 2.0) hd[0] = 0.0;  // (flag 1 stays: the Riccati rescue takes the agent)
        return;
    }
    // ---- output in the reference layout (the condensed kernels' expansion) ----
    double* X = sm + L.X;
    pol_fwd(q, Ub, X);
    __syncthreads();
    const int nxe = nx + ns;
    const size_t nz = (size_t)nxe * (N + 1) + 2 * (size_t)n;
    double* z = P.z + (size_t)b * nz;
    for (int i = tid; i < (N + 1) * nx; i += kPT) {
        const int kk = i / nx, s = i - kk * nx;
        z[(size_t)kk * nxe + s] = X[i];
    }
    for (int i = tid; i < (N + 1) * ns; i += kPT) {
        const int kk = i / ns, j = i - kk * ns;
        z[(size_t)kk * nxe + nx + j] = kk ? sb[(kk - 1) * ns + j] : 0.0;
    }
    for (int i = tid; i < n; i += kPT) {
        const int kk = i / nu, j = i - kk * nu;
        z[(size_t)(N + 1) * nxe + i] = Ub[i];
        z[(size_t)(N + 1) * nxe + n + i] = Ub[i] - (kk ? Ub[(kk - 1) * nu + j] : q.up[j]);
    }
    if (tid == 0) {
        if (P.kkt) P.kkt[b] = best_kkt;
        if (P.status) P.status[b] = best < c.tol ? CMPC_SOLVED : CMPC_SOLVED_INACCURATE;
        hd[0] = 0.0;
    }
}

}  // namespace

// The polish launch's compacted agent list: list[0 .. count) = the agents whose rescue image carries flag 1 or 2
// (ascending), list[batch] = count.  One 1024-thread workgroup: a ballot per wave, the waves' counts summed
// through LDS, 1024 agents per step.
__global__ __launch_bounds__(1024) void polish_list_kernel(const double* __restrict__ ws, unsigned long long stride,
                                                         int batch, int* __restrict__ list) {
    __shared__ int cnt[16];
    const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
    int base = 0;
    for (int b0 = 0; b0 < batch; b0 += 1024) {
        const int b = b0 + tid;
        double f = 0.0;
        if (b < batch) f = ws[(size_t)b * stride];
        const bool on = f == 1.0 || f == 2.0;
        const unsigned long long msk = __ballot(on);
        if (l == 0) cnt[wv] = __popcll(msk);
        __syncthreads();
        int off = base;
        for (int w = 0; w < wv; ++w) off += cnt[w];
        if (on) list[off + __popcll(msk & ((1ull << l) - 1ull))] = b;
        for (int w = 0; w < 16; ++w) base += cnt[w];
        __syncthreads();
    }
    if (tid == 0) list[batch] = base;
}

size_t mpc_polish_lds_bytes(const MpcConst& c) { return sizeof(double) * (size_t)pol_layout(c).total; }
int mpc_polish_max_active(const MpcConst& c) { return pol_layout(c).amax; }

template <int NXT, int NUT>
static hipError_t polish_launch_t(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, size_t lds) {
    hipError_t e = hipFuncSetAttribute((const void*)mpc_polish_kernel<NXT, NUT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((mpc_polish_kernel<NXT, NUT>), dim3(batch), dim3(kPT), lds, s, c, p);
    return hipGetLastError();
}

hipError_t mpc_polish_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    const size_t lds = mpc_polish_lds_bytes(c);
    if (lds > kMaxLdsBytes) return hipErrorInvalidValue;
    if (p.plist) {
        hipLaunchKernelGGL(polish_list_kernel, dim3(1), dim3(1024), 0, s, p.ws, c.ws_stride, batch, p.plist);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    switch (c.nx) {  // the reference's agent (9), the BASELINE double-integrator families (4, 6)
        case 9: return c.nu == 2 ? polish_launch_t<9, 2>(c, p, batch, s, lds) : polish_launch_t<9, 0>(c, p, batch, s, lds);
        case 4: return c.nu == 2 ? polish_launch_t<4, 2>(c, p, batch, s, lds) : polish_launch_t<4, 0>(c, p, batch, s, lds);
        case 6: return c.nu == 3 ? polish_launch_t<6, 3>(c, p, batch, s, lds) : polish_launch_t<6, 0>(c, p, batch, s, lds);
        default: return polish_launch_t<0, 0>(c, p, batch, s, lds);
    }
}

}  // namespace cmpc
