// Batched condensed IPM, v3: the production solver for the PlannerLPV row pattern
// (stage rows [v <= ; v + s0 <= ; e + s1 <= ; -e + s1 <= ; planes - s2 <=], reference
// planner/lib/plan_lib/distributedPlanner/LPV_Planner.py:251-380) with N <= 32.
// Same QP, same interior-point method, same safeguards and termination as the generic
// kernel (mpc_ipm.hip) and the C oracle (oracle/cmpc_oracle.c).
//
// Laid out so that nothing spills (the v2 kernel needed 512 registers and spilled
// 0.9 KB/lane to scratch on its latency-critical chains):
//  * one 64-lane wavefront per agent, one wavefront per workgroup.  LDS operations of
//    one wave execute in order, so intra-wave LDS hand-offs need only a compiler fence
//    (wsync), never s_barrier or a full lgkmcnt drain;
//  * lanes 0..31 own the constraint rows of stage k+1 (k = lane), lanes 32..63 the input
//    rows of u_k: RX = max(MC, 2 NU) register rows per lane; the slack groups of a stage
//    stay lane-local;
//  * batch-shared weights live in LDS, not in kernel-argument SGPRs;
//  * K = sum_k Gamma_{k+1}' W_{k+1} Gamma_{k+1}: lane c carries column c of Gamma_k in
//    registers through the recursion Gamma_{k+1} = A_k Gamma_k + [0 .. B_k], forms
//    W Gamma in registers, moves both to the MFMA fragment layout by an in-register row
//    transpose (v_permlane32_swap / v_permlane16_swap) and accumulates with V_MFMA_F64_16X16X4_F64 only on the tiles that are nonzero for the
//    stage (static per horizon segment: no data-dependent branch around an MFMA);
//  * K is factored in the accumulators (blocked right-looking Cholesky: 16x16 diagonal
//    factor, panel substitution, trailing SYRK on MFMA); the diagonal factors L_JJ are
//    kept in LDS for the triangular solves.
#include <cmath>

#include "di_rows.h"
#include "internal.h"
#include "wave_ops.h"

namespace cmpc {

namespace {

// Intra-wave LDS ordering: the hardware keeps one wave's LDS operations in order; this
// only stops the compiler from moving LDS accesses across the hand-off point.

// PlannerLPV row pattern: row 0 no slack; 1 -> s0 (+); 2,3 -> s1 (+); 4.. -> s2 (-)
__host__ __device__ constexpr int slk(int r) { return r == 0 ? -1 : (r == 1 ? 0 : (r < 4 ? 1 : 2)); }
__host__ __device__ constexpr double sgn(int r) { return r < 4 ? 1.0 : -1.0; }

struct Lds3 {
    int cst, A, B, C, H, Pq, x0, up, W, Gb, Yb, X, dX, yb, U, dU, rd, vb, thin, bU, Ld, red, stamps, Phi, Pst, total;
    // two-wave mode (W2): the fields from W to stamps are each wave's private copy (wave 1's at + psz);
    // exchange areas: wave 1's K tiles (xk), the predictor's rho and vb (xr, xv), dU of the two passes
    // (xu0, xu1), flags (xf)
    int psz, xk, xr, xv, xu0, xu1, xf;
};

// Two-wave mode (W2, the DS instantiation at <= 2 agents per CU): the K build's MFMA tiles split between
// the waves (the VALU Gamma recursion runs on both); wave 1 hands its tiles to wave 0.  Wave 0 owns the
// tiles below (balanced by the number of stages that touch each tile: 70 of 140 MFMAs at cfg3).
__host__ __device__ constexpr bool w2_own0(int T, int ti, int tj) {
    return T >= 4 ? (ti == 0 || (ti == 1 && tj == 0) || (ti == 3 && tj < 3))
                  : (T == 3 ? (ti == 0 || (ti == 1 && tj == 0)) : ti == 0);
}
#ifndef CMPC_W2_RHS
#define CMPC_W2_RHS 1
#endif
constexpr bool kW2Rhs = CMPC_W2_RHS != 0;  // (lab switch: the predictor right-hand side on wave 1)
__host__ __device__ constexpr int w2_tiles1(int T) {
    int c = 0;
    for (int ti = 0; ti < T; ++ti)
        for (int tj = 0; tj <= ti; ++tj) c += w2_own0(T, ti, tj) ? 0 : 1;
    return c;
}
// slot of wave-1 tile (ti, tj) in the exchange (tiles in ascending (ti, tj) order)
__host__ __device__ constexpr int w2_slot1(int T, int ti, int tj) {
    int c = 0;
    for (int a = 0; a < T; ++a)
        for (int b = 0; b <= a; ++b) {
            if (a == ti && b == tj) return c;
            c += w2_own0(T, a, b) ? 0 : 1;
        }
    return c;
}

// LS (the reference's own agent, nx 9 / nu 2, built by lpv_build.hip): the model's structure is
// fixed by LPV_Planner.py:493-585 and :279-380, and the images shrink to it —
//   A_k = I + D_k with D_k nonzero only in columns 0..2 (vx, vy, wz drive every state)   N x 9 x 3
//   B_k nonzero only in rows 0..2                                                          N x 3 x 2
//   rows: -vx, vx, ey, -ey, then a_x X + a_y Y per plane: their coefficients only          N x (4 + 2 nb)
//   W_k = 2Q + the rows' weights (Q diagonal): diagonal except the (X, Y) block; the entries
//   on vx, ey and the (X, Y) block per stage                                               N x 5
// 39 KB of LDS at N = 30 instead of 78 KB: four agents per CU, so 1024 agents run at once.
constexpr int kLsW = 5;  // LS stage weights: w(vx,vx), w(ey,ey), w(X,X), w(X,Y), w(Y,Y)
template <int NB>
__host__ __device__ constexpr int ls_cw() { return 4 + 2 * NB; }

// DS (the synthetic 2-D double integrator's fused round, x = [p_x p_y v_x v_y], rows built by
// di_rows.h inside the launch): rows 0..3 are -v_x, v_x, p_y, -p_y (constant coefficients), the planes
// a_x p_x + a_y p_y, Q diagonal.  The images shrink to the planes' coefficients (N x 2 nb) and the
// six entries of W_k that are not exactly zero (w_xx, w_xy, w_yx, w_yy on (p_x, p_y), w_vx, w_vy);
// every product and sum is the dense form's, in its order, without the exact zeros: same bits.
// Bit equality with the dense instantiation also needs the same fma contraction in both: the
// backend's cross-statement contraction (-ffp-contract=fast) decides per use count of a product and
// so differs between the two instantiations; this file is built with -ffp-contract=on (Makefile).
constexpr int kDsW = 6;
template <int NB>
__host__ __device__ constexpr int ds_cw() { return NB > 0 ? 2 * NB : 2; }

// Segmented (parallel-in-time) forward simulation: the horizon's N stages split into four
// segments [a_q, a_{q+1}), one per row of 16 lanes.  Each row runs its segment's recursion from a
// zero state (row 0 from x_0); a two-step chain then carries the true state across the segment
// starts, x_{a_{q+1}} = x^loc_{a_{q+1}} + Phi_{a_{q+1}} x_{a_q}, and one parallel pass adds
// Phi_k x_{a_q} to every stage of segments 1..3.  Phi_k = A_{k-1} .. A_{a_q}, the transition from
// the segment start, depends on A only: built once per solve (phi_build).  The serial chain drops
// from N stage steps to ceil(N / 4) + 2.  For the small-state instantiations (NX <= 4: the LDS image
// has room for Phi) with T >= 2 tiles and NU <= 2, i.e. N > 8: every segment is non-empty.
__host__ __device__ constexpr int seg_a(int q, int N) { return (q * N + 3) / 4; }
// ... and of the adjoint over the stages k = 1..N: [b_q, b_{q+1}), b_0 = 1, b_4 = N + 1
__host__ __device__ constexpr int seg_b(int q, int N) { return 1 + (q * N + 3) / 4; }
template <int T, int NX, int NU, bool LS>
__host__ __device__ constexpr bool seg_on() {
    return !LS && NX <= 4 && NU <= 2 && T >= 2;
}

template <int T, int NX, int NU, int NB, bool LS = false, bool DS = false, bool W2 = false>
__host__ __device__ inline Lds3 lds3_layout(int N) {
    constexpr int NP = 16 * T, MC = 4 + NB;
    Lds3 L{};
    int o = 0;
    auto take = [&](int cnt) {
        int r = o;
        o += (cnt + 1) & ~1;
        return r;
    };
    L.cst = take(NX * NX + 2 * NU * NU + 3 + 2 * NU);
    L.A = take(LS ? N * NX * 3 : N * NX * NX);
    L.B = take(LS ? N * 3 * NU : N * NX * NU);
    L.C = take(LS ? N * ls_cw<NB>() : (DS ? N * ds_cw<NB>() : N * MC * NX));
    L.H = take(N * MC);
    L.Pq = take((N + 1) * NX);
    L.x0 = take(NX);
    L.up = take(NU);
    // segmented forward simulation (kSeg): the transitions Phi_k of stages (a_1, N] (fwd3seg); 352
    // doubles at N = 30, NX = 4
    L.Phi = take(seg_on<T, NX, NU, LS>() ? (N - seg_a(1, N)) * NX * NX : 0);
    // ... and the transposed transitions Psi'_k of the segmented adjoint (psi3seg): 352 doubles at N = 30
    L.Pst = take(seg_on<T, NX, NU, LS>() ? (seg_b(3, N) - 1) * NX * NX : 0);
    const int pbeg = o;
    // the Cholesky panel scratch ((T-1) x 16 x 17) aliases W | dX | yb after the K build (the stage
    // weights are consumed by then, and the residuals' adjoints are done while the passes' have not
    // begun); Gb extends them only where they are smaller than that (short horizons, small NX).  At
    // NX = 9 the extra 12 KB it used to take halved the agents per CU (90 KB -> 78 KB); at cfg3 the
    // dX | yb alias makes room for the segmented recursions' transitions within 40 KB.
    const int wsz = LS ? N * kLsW : (DS ? N * kDsW : N * NX * NX);
    L.W = take(wsz);
    L.dX = take((N + 1) * NX);
    L.yb = take((N + 1) * NX);
    const int sp_need = (T - 1) * 16 * 17 - (L.yb + (((N + 1) * NX + 1) & ~1) - L.W);
    L.Gb = take(sp_need > 0 ? sp_need : 0);
    L.Yb = L.Gb;
    L.X = take((N + 1) * NX);
    L.U = take(NP);
    L.dU = take(NP);
    L.rd = take(NP);
    L.vb = take(NP);
    L.thin = take(NP);
    L.bU = take(NP);
    L.Ld = take(T * 16 * 17);
    L.red = take(16);
    L.stamps = take(kStampSlots);
    L.psz = o - pbeg;
    if (W2) {
        constexpr int RX = (4 + NB) > 2 * NU ? (4 + NB) : 2 * NU;
        o += L.psz;  // wave 1's private copy
        L.xk = take(w2_tiles1(T) * 256);
        L.xr = take(64 * RX);
        L.xv = take(NP);
        L.xu0 = take(NP);
        L.xu1 = take(NP);
        L.xf = take(2);
    }
    L.total = o;
    return L;
}

// x_0 = x0 (LDS, or 0), x_{k+1} = A_k x_k + B_k u_k.  Lane (l & 15) = s < NX of every row of
// 16 carries x_s (the rows are duplicates; lanes with s >= NX duplicate x_0); x_t reaches the
// row by DPP row_newbcast.  A stage's A row and B u term are fetched two stages ahead into
// rotating register sets (unrolled by three: no copies, no branches; the fetch index is clamped
// instead of guarded).  Every lane stores: duplicates write equal values.
template <int NX, int NU, bool LS = false>
__device__ __forceinline__ void fwd3(int l, int N, const double* A, const double* B, const double* x0,
                                     const double* U, double* X) {
    static_assert(NX <= 16, "row broadcast");
    constexpr int NA = LS ? 3 : NX;  // columns of the stage image (LS: D_k, A_k = I + D_k)
    const int s = (l & 15) < NX ? (l & 15) : 0;
    double xr = x0 ? x0[s] : 0.0;
    X[s] = xr;
    if (N <= 0) return;
    // B_k u_k of every stage first, in parallel (off the chain), into X_{k+1}'s slot; the
    // recursion then adds A_k x_k to it in place (the slot is fetched before it is overwritten)
    for (int i = l; i < N * NX; i += 64) {
        const int k = i / NX, r = i - k * NX;
        double v = 0.0;
        if constexpr (LS) {
            const int rr = r < 3 ? r : 0;
#pragma unroll
            for (int j = 0; j < NU; ++j) v = fma(B[(k * 3 + rr) * NU + j], U[k * NU + j], v);
            v = r < 3 ? v : 0.0;
        } else {
#pragma unroll
            for (int j = 0; j < NU; ++j) v = fma(B[(k * NX + r) * NU + j], U[k * NU + j], v);
        }
        X[NX + i] = v;
    }
    wsync();
    auto fetch = [&](int k, double* av, double* bv) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < NA; ++t) av[t] = A[(k * NX + s) * NA + t];
        bv[0] = X[(k + 1) * NX + s];
    };
    auto step = [&](int k, const double* av, const double* bv) __attribute__((always_inline)) {
        double v0 = bv[0], v1 = 0.0;
        static_for<0, NA>([&](auto t) __attribute__((always_inline)) {
            constexpr int tt = decltype(t)::value;
            if constexpr (tt & 1) v1 = fma(av[tt], bcast16<tt>(xr), v1);
            else v0 = fma(av[tt], bcast16<tt>(xr), v0);
        });
        if constexpr (LS) xr = (v0 + v1) + xr;  // x_{k+1} = x_k + D_k x_k + B_k u_k
        else xr = v0 + v1;
        X[(k + 1) * NX + s] = xr;
    };
    // three register sets, fetched two stages ahead (unrolled by three: no copies; fetch indices
    // clamped, not guarded): a stage's LDS latency hides behind two stages of the chain
    double a0[NA], a1[NA], a2[NA], b0[1], b1[1], b2[1];
    fetch(0, a0, b0);
    fetch(1 < N ? 1 : N - 1, a1, b1);
    int k = 0;
    // (scheduling barriers keep the machine scheduler from sinking the loads towards their use)
    for (; k + 2 < N; k += 3) {
        fetch(k + 2, a2, b2);
        __builtin_amdgcn_sched_barrier(0);
        step(k, a0, b0);
        fetch(k + 3 < N ? k + 3 : N - 1, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        step(k + 1, a1, b1);
        fetch(k + 4 < N ? k + 4 : N - 1, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        step(k + 2, a2, b2);
    }
    if (k < N) step(k, a0, b0);
    if (k + 1 < N) step(k + 1, a1, b1);
}

// Phi_k for k in (a_1, N] (see seg_a): rows 1..3 build their segment's transitions in parallel, lane
// s of the row holding row s of Phi (Phi_{a_q} = I, Phi_{k+1} = A_k Phi_k); stored at slot k - a_1 - 1.
template <int NX>
__device__ __forceinline__ void phi_build(int l, int N, const double* A, double* Phi) {
    const int q = l >> 4, s = (l & 15) < NX ? (l & 15) : 0;
    const int a1 = seg_a(1, N), a = seg_a(q, N), e = seg_a(q + 1, N);
    double ph[NX];
#pragma unroll
    for (int t = 0; t < NX; ++t) ph[t] = (s == t) ? 1.0 : 0.0;
    for (int i = 0; i < a1; ++i) {  // a_1 = the longest segment
        const int k = a + i;
        const bool valid = q >= 1 && k < e;
        const int kc = valid ? k : a1;
        double ar[NX], nw[NX];
#pragma unroll
        for (int t = 0; t < NX; ++t) ar[t] = A[(kc * NX + s) * NX + t];
        static_for<0, NX>([&](auto c_c) __attribute__((always_inline)) {
            constexpr int cc = decltype(c_c)::value;
            double v = 0.0;
            static_for<0, NX>([&](auto t_c) __attribute__((always_inline)) {
                constexpr int tt = decltype(t_c)::value;
                v = fma(ar[tt], bcast16<tt>(ph[cc]), v);
            });
            nw[cc] = v;
        });
#pragma unroll
        for (int c = 0; c < NX; ++c) ph[c] = valid ? nw[c] : ph[c];
        if (valid && (l & 15) < NX) {
#pragma unroll
            for (int c = 0; c < NX; ++c) Phi[((k - a1) * NX + s) * NX + c] = ph[c];
        }
    }
}

// x += Phi x_a (the correction of a stage state, and the segment-start chain: same operation order)
template <int NX>
__device__ __forceinline__ double phi_apply(const double* phr, const double* xa, double v) {
#pragma unroll
    for (int t = 0; t < NX; ++t) v = fma(phr[t], xa[t], v);
    return v;
}

// fwd3 (x_0 = x0 or 0, x_{k+1} = A_k x_k + B_k u_k) by segments (seg_a, phi_build); X, U, A, B as fwd3.
template <int NX, int NU>
__device__ __forceinline__ void fwd3seg(int l, int N, const double* A, const double* B, const double* x0,
                                        const double* U, double* X, const double* Phi) {
    static_assert(NX <= 16, "row broadcast");
    const int q = l >> 4, s = (l & 15) < NX ? (l & 15) : 0;
    const int a1 = seg_a(1, N), a = seg_a(q, N), e = seg_a(q + 1, N);
    // each row its segment, from x^loc_{a_q} = 0 (row 0: x_0); B_k u_k is formed beside the chain. A
    // finished row repeats its last stage without changing its state (clamped fetch, select, equal store)
    double xr = (q == 0 && x0) ? x0[s] : 0.0;
    if (q == 0) X[s] = xr;
    auto fetch = [&](int i, double* av) __attribute__((always_inline)) {
        const int k = a + i < e ? a + i : e - 1;
#pragma unroll
        for (int t = 0; t < NX; ++t) av[t] = A[(k * NX + s) * NX + t];
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            av[NX + j] = B[(k * NX + s) * NU + j];
            av[NX + NU + j] = U[k * NU + j];
        }
    };
    auto step = [&](int i, const double* av) __attribute__((always_inline)) {
        const int k = a + i < e ? a + i : e - 1;
        double v0 = 0.0, v1 = 0.0;
#pragma unroll
        for (int j = 0; j < NU; ++j) v0 = fma(av[NX + j], av[NX + NU + j], v0);
        static_for<0, NX>([&](auto t) __attribute__((always_inline)) {
            constexpr int tt = decltype(t)::value;
            if constexpr (tt & 1) v1 = fma(av[tt], bcast16<tt>(xr), v1);
            else v0 = fma(av[tt], bcast16<tt>(xr), v0);
        });
        xr = (a + i < e) ? v0 + v1 : xr;
        X[(k + 1) * NX + s] = xr;
    };
    // two register sets, one stage ahead (the rows' chains are ceil(N / 4) steps long)
    double p0[NX + 2 * NU], p1[NX + 2 * NU];
    fetch(0, p0);
    int i = 0;
    for (; i + 1 < a1; i += 2) {
        fetch(i + 1, p1);
        __builtin_amdgcn_sched_barrier(0);
        step(i, p0);
        fetch(i + 2, p0);
        __builtin_amdgcn_sched_barrier(0);
        step(i + 1, p1);
    }
    if (i < a1) step(i, p0);
    wsync();
    // segment starts: x_{a_1} is exact (segment 0 began at x_0); x_{a_{q+1}} = x^loc + Phi x_{a_q}
    // (every row runs the chain; row q keeps x_{a_q} for its own stages)
    double xq[NX];
    {
        double xa[NX], ph[NX];
        double v = X[a1 * NX + s];
#pragma unroll
        for (int qq = 2; qq < 5; ++qq) {
            static_for<0, NX>([&](auto t) __attribute__((always_inline)) {
                constexpr int tt = decltype(t)::value;
                xa[tt] = bcast16<tt>(v);
            });
#pragma unroll
            for (int t = 0; t < NX; ++t) xq[t] = (q == qq - 1) ? xa[t] : xq[t];
            if (qq == 4) break;
            const int aq = seg_a(qq, N);
#pragma unroll
            for (int t = 0; t < NX; ++t) ph[t] = Phi[((aq - a1 - 1) * NX + s) * NX + t];
            v = phi_apply<NX>(ph, xa, X[aq * NX + s]);
        }
    }
    // row q >= 1 corrects its segment's stages (a_q, a_{q+1}]: x_k = x^loc_k + Phi_k x_{a_q}; at most
    // 2 x 16 entries per row (segments of <= 8 stages, NX <= 4)
    if (q >= 1) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = (l & 15) + 16 * h, k = a + 1 + j / NX, r = j % NX;
            if (k <= e) {
                double ph[NX];
#pragma unroll
                for (int t = 0; t < NX; ++t) ph[t] = Phi[((k - a1 - 1) * NX + r) * NX + t];
                X[k * NX + r] = phi_apply<NX>(ph, xq, X[k * NX + r]);
            }
        }
    }
}

// Psi'_k (transposed) for k in [1, b_3): x_{b_{q+1}} = Psi_k x_k, the transition of stages k ..
// b_{q+1} - 1 of segment q (seg_b); rows 0..2 build their segment's in parallel from the top
// (Psi'_k = A_k' Psi'_{k+1}), lane s holding row s; stored at slot k - 1.
template <int NX>
__device__ __forceinline__ void psi_build(int l, int N, const double* A, double* Pst) {
    const int q = l >> 4, s = (l & 15) < NX ? (l & 15) : 0;
    const int b = seg_b(q, N), e = seg_b(q + 1, N), len = seg_b(1, N) - 1;
    double tr[NX];
#pragma unroll
    for (int c = 0; c < NX; ++c) tr[c] = (s == c) ? 1.0 : 0.0;
    for (int i = 0; i < len; ++i) {
        const int k = e - 1 - i;
        const bool valid = q <= 2 && k >= b;
        const int kc = valid ? k : 1;
        double at[NX], nw[NX];
#pragma unroll
        for (int t = 0; t < NX; ++t) at[t] = A[(kc * NX + t) * NX + s];
        static_for<0, NX>([&](auto c_c) __attribute__((always_inline)) {
            constexpr int cc = decltype(c_c)::value;
            double v = 0.0;
            static_for<0, NX>([&](auto t_c) __attribute__((always_inline)) {
                constexpr int tt = decltype(t_c)::value;
                v = fma(at[tt], bcast16<tt>(tr[cc]), v);
            });
            nw[cc] = v;
        });
#pragma unroll
        for (int c = 0; c < NX; ++c) tr[c] = valid ? nw[c] : tr[c];
        if (valid && (l & 15) < NX) {
#pragma unroll
            for (int c = 0; c < NX; ++c) Pst[((k - 1) * NX + s) * NX + c] = tr[c];
        }
    }
}

// psi3 (psi_N = y_N, psi_k = y_k + A_k' psi_{k+1}, k = N-1 .. 1, over y in place) by segments: each row
// runs its segment from psi^loc = 0 above it (the top one from psi_N = y_N), a two-step chain carries
// psi down the segment tops, each row corrects its stages, psi_k = psi^loc_k + Psi'_k psi_{b_{q+1}}.
template <int NX>
__device__ __forceinline__ void psi3seg(int l, int N, const double* A, double* y, const double* Pst) {
    const int q = l >> 4, j = l & 15, s = j < NX ? j : 0;
    const int b = seg_b(q, N), e = seg_b(q + 1, N), len = seg_b(1, N) - 1;
    double pr = 0.0;  // psi^loc_{k+1}: zero above the segment
    auto fetch = [&](int i, double* av) __attribute__((always_inline)) {
        const int k = e - 1 - i >= b ? e - 1 - i : b;
        const int ka = k < N ? k : N - 1;  // psi_N = y_N: A_N does not exist (pr = 0 there)
#pragma unroll
        for (int t = 0; t < NX; ++t) av[t] = A[(ka * NX + t) * NX + s];
        av[NX] = y[k * NX + s];
    };
    auto step = [&](int i, const double* av) __attribute__((always_inline)) {
        const int k = e - 1 - i >= b ? e - 1 - i : b;
        double p0 = av[NX], p1 = 0.0;
        static_for<0, NX>([&](auto t) __attribute__((always_inline)) {
            constexpr int tt = decltype(t)::value;
            if constexpr (tt & 1) p1 = fma(av[tt], bcast16<tt>(pr), p1);
            else p0 = fma(av[tt], bcast16<tt>(pr), p0);
        });
        pr = (e - 1 - i >= b) ? p0 + p1 : pr;
        y[k * NX + s] = pr;
    };
    double a0[NX + 1], a1[NX + 1];
    fetch(0, a0);
    int i = 0;
    for (; i + 1 < len; i += 2) {
        fetch(i + 1, a1);
        __builtin_amdgcn_sched_barrier(0);
        step(i, a0);
        fetch(i + 2, a0);
        __builtin_amdgcn_sched_barrier(0);
        step(i + 1, a1);
    }
    if (i < len) step(i, a0);
    wsync();
    // segment tops, from above: psi_{b_3} is exact (the top segment began at psi_N); row q keeps
    // psi_{b_{q+1}} for its stages
    double pq[NX];
    {
        double xa[NX], ph[NX];
        double v = y[seg_b(3, N) * NX + s];
#pragma unroll
        for (int qq = 2; qq >= 0; --qq) {
            static_for<0, NX>([&](auto t) __attribute__((always_inline)) {
                constexpr int tt = decltype(t)::value;
                xa[tt] = bcast16<tt>(v);
            });
#pragma unroll
            for (int t = 0; t < NX; ++t) pq[t] = (q == qq) ? xa[t] : pq[t];
            if (qq == 0) break;
            const int bb = seg_b(qq, N);
#pragma unroll
            for (int t = 0; t < NX; ++t) ph[t] = Pst[((bb - 1) * NX + s) * NX + t];
            v = phi_apply<NX>(ph, xa, y[bb * NX + s]);
        }
    }
    // rows 0..2 correct their stages [b_q, b_{q+1}): at most 8 stages x NX entries, 2 per lane
    if (q <= 2) {
#pragma unroll
        for (int h = 0; h < (8 * NX + 15) / 16; ++h) {
            const int idx = j + 16 * h, k = b + idx / NX, r = idx % NX;
            if (k < e) {
                double ph[NX];
#pragma unroll
                for (int t = 0; t < NX; ++t) ph[t] = Pst[((k - 1) * NX + r) * NX + t];
                y[k * NX + r] = phi_apply<NX>(ph, pq, y[k * NX + r]);
            }
        }
    }
}

// The adjoint's serial part only: psi_N = y_N, psi_k = y_k + A_k' psi_{k+1} for k = N-1 .. 1,
// written over y in place (rows 0,1 of the wave on y0, rows 2,3 on y1; y_k is fetched before
// psi_k overwrites it).  The products o_k = B_k' psi_{k+1} are independent of one another and
// are formed afterwards by the lanes that own u_k (bpsi3), off the recursion's chain.  The
// operation order is the fused recursion's (even/odd partial sums), so the bits are unchanged.
template <int NX, bool LS = false>
__device__ __forceinline__ void psi3(int l, int N, const double* A, double* y0, double* y1) {
    static_assert(NX <= 16, "row broadcast");
    const int h = l >> 5, s = l & 15;
    const int sx = s < NX ? s : 0;
    double* y = h ? y1 : y0;
    double pr = y[N * NX + sx];
    if (N <= 1) return;
    // LS: (A_k' psi)[s] = psi[s] + (s < 3 ? sum_t D_k[t][s] psi[t] : 0); lanes s >= 3 read column 0
    // of D and discard it (branch-free)
    const int sd = sx < 3 ? sx : 0;
    const double dmask = sx < 3 ? 1.0 : 0.0;
    auto fetch = [&](int k, double* av, double& yv) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < NX; ++t) av[t] = LS ? A[(k * NX + t) * 3 + sd] : A[(k * NX + t) * NX + sx];
        yv = y[k * NX + sx];
    };
    auto step = [&](int k, const double* av, double yk) __attribute__((always_inline)) {
        double ps[NX];
        static_for<0, NX>([&](auto t) __attribute__((always_inline)) {
            constexpr int tt = decltype(t)::value;
            ps[tt] = bcast16<tt>(pr);
        });
        double p0 = LS ? 0.0 : yk, p1 = 0.0;
#pragma unroll
        for (int t = 0; t < NX; ++t) {
            if (t & 1) p1 = fma(av[t], ps[t], p1);
            else p0 = fma(av[t], ps[t], p0);
        }
        if constexpr (LS) pr = fma(dmask, p0 + p1, yk + pr);
        else pr = p0 + p1;
        y[k * NX + sx] = pr;
    };
    // three register sets fetched two stages ahead; fetch indices clamped to stage 1
    double a0[NX], y0k, a1[NX], y1k, a2[NX], y2k;
    fetch(N - 1, a0, y0k);
    fetch(N >= 3 ? N - 2 : 1, a1, y1k);
    int k = N - 1;
    for (; k >= 3; k -= 3) {
        fetch(k - 2, a2, y2k);
        __builtin_amdgcn_sched_barrier(0);
        step(k, a0, y0k);
        fetch(k >= 4 ? k - 3 : 1, a0, y0k);
        __builtin_amdgcn_sched_barrier(0);
        step(k - 1, a1, y1k);
        fetch(k >= 5 ? k - 4 : 1, a1, y1k);
        __builtin_amdgcn_sched_barrier(0);
        step(k - 2, a2, y2k);
    }
    if (k >= 1) step(k, a0, y0k);
    if (k >= 2) step(k - 1, a1, y1k);
}

// o = B_k[:, i]' psi_{k+1} (psi as left in place by psi3): even/odd partial sums, as before
template <int NX, int NU, bool LS = false>
__device__ __forceinline__ double bpsi3(const double* B, const double* psi, int k, int i) {
    constexpr int NB_ = LS ? 3 : NX;  // LS: B_k is nonzero only in rows 0..2
    double v0 = 0.0, v1 = 0.0;
#pragma unroll
    for (int t = 0; t < NB_; ++t) {
        const double bt = B[(k * NB_ + t) * NU + i], pt = psi[(k + 1) * NX + t];
        if (t & 1) v1 = fma(bt, pt, v1);
        else v0 = fma(bt, pt, v0);
    }
    return v0 + v1;
}

}  // namespace

// L5 (with LS): Q's diagonal is zero on states 1, 2, 5, 6 (the reference's Q = diag(10, 0, 0, 25, 10, 0, 0,
// 0, 0), config_LPV.py:7), so W_k = 2Q + the rows' weights is nonzero only on states {0, 3, 4, 7, 8}: the
// K build's MFMA contraction runs over those five (two k-steps of 4) instead of all nine (three).
// W2: two wavefronts per agent (a 128-lane workgroup, one wave per SIMD, two agents per CU): for batches
// that leave SIMDs idle at one wave per agent (<= 512 agents on 256 CUs: BASELINE cfg4's shard).  Both waves
// run the whole iteration on private copies of the mutable images (the same arithmetic in the same order, so
// they hold bit-identical values and take the same wave-uniform decisions), except:
//   * the K build's MFMAs: each wave accumulates its own tiles (w2_own0); wave 1 hands its tiles to wave 0
//     through LDS (each tile keeps its accumulation order: bit-identical to one wave);
//   * while wave 0 factors K and inverts the diagonal blocks, wave 1 forms the predictor's right-hand side
//     (rho, C' rho~, the adjoint recursion, vb) and hands rho and vb over;
//   * the triangular solves run on wave 0 only; wave 1 takes each pass's dU from LDS.
// Wave 0 alone writes the outputs.
template <int T, int NX, int NU, int NB, bool LS = false, bool DS = false, bool L5 = false, bool W2 = false>
__global__ __launch_bounds__(W2 ? 128 : 64, 1) void mpc_ipm3_kernel(const MpcConst c, const MpcPtrs P) {
    constexpr int MC = 4 + NB, NS = 3, NT = T * (T + 1) / 2, NP = 16 * T, NXP = (NX + 3) & ~3;
    constexpr int NI = 2 * NU, RX = MC > NI ? MC : NI;
    constexpr int CW = ls_cw<NB>();  // LS: row coefficients per stage
    static_assert(!LS || (NX == 9 && NU == 2), "LS: the reference's agent model");
    static_assert(!DS || (NX == 4 && NU == 2 && !LS), "DS: the 2-D double integrator");
    static_assert(!L5 || LS, "L5: a variant of LS");
    constexpr int CWD = ds_cw<NB>();  // DS: plane coefficients per stage
    extern __shared__ __attribute__((aligned(16))) double sm[];
    static_assert(!W2 || DS, "W2: the fused double-integrator instantiation");
    const int l0 = threadIdx.x & 63, b = blockIdx.x, N = c.N, n = N * NU, ms = N * MC;
    const int l = l0;
    // the wave index as a scalar (wave-uniform: the branches on it are scalar, never exec-masked)
    const int wvi = W2 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    const Lds3 L = lds3_layout<T, NX, NU, NB, LS, DS, W2>(N);
    const int po = wvi * L.psz;  // this wave's private images
    double* Q2 = sm + L.cst;          // 2Q
    double* R2 = Q2 + NX * NX;        // 2R
    double* dR2 = R2 + NU * NU;       // 2dR
    double* Qs2 = dR2 + NU * NU;      // 2Qs
    double* ub = Qs2 + 3;
    double* lb = ub + NU;
    double* sA = sm + L.A;
    double* sB = sm + L.B;
    double* sC = sm + L.C;
    double* sH = sm + L.H;
    double* sP = sm + L.Pq;
    double* sx0 = sm + L.x0;
    double* sup = sm + L.up;
    double* sW = sm + po + L.W;
    double* X = sm + po + L.X;
    double* dX = sm + po + L.dX;
    double* yb = sm + po + L.yb;
    double* U = sm + po + L.U;
    double* dU = sm + po + L.dU;
    double* rd = sm + po + L.rd;
    double* vb = sm + po + L.vb;
    double* thin = sm + po + L.thin;
    double* bU = sm + po + L.bU;
    double* Ld = sm + po + L.Ld;
    double* red = sm + po + L.red;
    double* SP = sW;  // Cholesky panel scratch (aliases W | Gb after the K build)
    const bool stamp = P.stamps != nullptr;
    // diagnostic per-section clock sums live in LDS (registers stay with the solver)
    unsigned long long* tsum = reinterpret_cast<unsigned long long*>(sm + po + L.stamps);
    if (l < kStampSlots) tsum[l] = 0;
    unsigned long long t_a = stamp ? clock64_() : 0, t_b = 0;
#define STAMP(slot)                                \
    if (stamp) {                                   \
        t_b = clock64_();                          \
        if (l == 0) tsum[slot] += t_b - t_a;       \
        t_a = t_b;                                 \
    }

    // ---------------- stage the agent's data and the shared weights into LDS ----------------
    // (W2: the shared images by wave 0 alone — the fused row build accumulates into the linear cost, so two
    // writers would race — then a barrier before their first use below)
    if (wvi == 0) {
        const double* gA = P.A + (size_t)b * N * NX * NX;
        const double* gB = P.B + (size_t)b * N * NX * NU;
        const double* gC = P.C + (size_t)b * N * MC * NX;
        const double* gP = P.p + (size_t)b * (N + 1) * NX;
        if constexpr (LS) {
            // D_k = A_k - I on columns 0..2 (the builder's A_k = I + dt A_c, LPV_Planner.py:583); B_k rows
            // 0..2; the rows' coefficients [vx of rows 0, 1 | ey of rows 2, 3 | (X, Y) of each plane]
            for (int i = l; i < N * 27; i += 64) {
                const int kk = i / 27, q = i - kk * 27, r = q / 3, t = q - r * 3;
                sA[i] = gA[kk * 81 + r * 9 + t] - (r == t ? 1.0 : 0.0);
            }
            for (int i = l; i < N * 6; i += 64) sB[i] = gB[(i / 6) * 18 + (i % 6)];
            for (int i = l; i < N * CW; i += 64) {
                const int kk = i / CW, q = i - kk * CW;
                const int r = q < 4 ? q : 4 + ((q - 4) >> 1), col = q < 2 ? 0 : (q < 4 ? 3 : 7 + ((q - 4) & 1));
                sC[i] = gC[(kk * MC + r) * NX + col];
            }
        } else {
            for (int i = l; i < N * NX * NX; i += 64) sA[i] = gA[i];
            for (int i = l; i < N * NX * NU; i += 64) sB[i] = gB[i];
        }
        if (LS) {
            for (int i = l; i < ms; i += 64) sH[i] = P.h[(size_t)b * ms + i];
            for (int i = l; i < (N + 1) * NX; i += 64) sP[i] = gP[i];
        } else if (P.fuse.on) {
            // fused round: this agent's rows and linear cost built from the exchanged
            // trajectories straight into LDS (bit-identical to di_build_kernel's)
            const DiFuse& F = P.fuse;
            const double* own = F.traj_all + (size_t)(F.c.self_offset + b) * (N + 1) * 2;
            const int* nbr = F.nbr + (size_t)b * NB;
            const double ln = F.lane[b];
            for (int kk = l; kk <= N; kk += 64) {
                const int h1 = kk > 0 ? kk - 1 : 0;
                if constexpr (DS)
                    di_stage_rows<true>(F.c, nbr, ln, F.traj_all, own, kk, sP + kk * NX, sC + h1 * CWD, sH + h1 * MC);
                else
                    di_stage_rows(F.c, nbr, ln, F.traj_all, own, kk, sP + kk * NX, sC + h1 * MC * NX, sH + h1 * MC);
            }
        } else {
            for (int i = l; i < N * MC * NX; i += 64) sC[i] = gC[i];
            for (int i = l; i < ms; i += 64) sH[i] = P.h[(size_t)b * ms + i];
            for (int i = l; i < (N + 1) * NX; i += 64) sP[i] = gP[i];
        }
        if (l < NX) sx0[l] = P.x0[(size_t)b * NX + l];
        if (l < NU) sup[l] = P.up[(size_t)b * NU + l];
        for (int i = l; i < NX * NX; i += 64) Q2[i] = 2.0 * c.Q[i];
        if (l < NU * NU) {
            R2[l] = 2.0 * c.R[l];
            dR2[l] = 2.0 * c.dR[l];
        }
        if (l < 3) Qs2[l] = 2.0 * c.Qs[l];
        if (l < NU) {
            ub[l] = c.u_ub[l];
            lb[l] = c.u_lb[l];
        }
    }
    {
        for (int i = l; i < NP; i += 64) {
            U[i] = 0.0;
            dU[i] = 0.0;
            vb[i] = 0.0;
            thin[i] = 0.0;
            bU[i] = 0.0;
        }
    }
    // ---- rows owned by this lane: stage k+1 rows (lanes 0..31) or input rows of u_k (32..63) ----
    const bool lo = l < 32;
    const int k = l & 31;
    const bool own = k < N;
    double t[RX], lam[RX], th[RX], rp[RX], rho[RX], gdu[RX];
    unsigned actm = 0;  // bit r: row r of this lane exists and has a finite bound
    // rows are evaluated branch-free: every LDS read is unconditional (indices of lanes that
    // own no such row stay inside the LDS allocation and are masked afterwards); a read inside a
    // select arm cannot be speculated, and each became a divergent branch with its own wait
    auto wv = [&](int r) -> double {
        const double h = sH[k * MC + r];
        const double bl = lb[r >> 1], bu = ub[r >> 1];
        const double wi = (r & 1) ? -bl : bu;
        return lo ? h : wi;
    };
    double sg[NS] = {0.0, 0.0, 0.0};
    // the rescue image (hand_doubles, internal.h): [flag, -, U, sigma, t, lambda] in the oracle's row order
    auto write_image = [&]() __attribute__((always_inline)) {
        double* hd = P.ws + (size_t)b * c.ws_stride;
        const int m = c.m, ht = (int)hand_t(c);
        for (int i = l; i < n; i += 64) hd[2 + i] = U[i];
        if (own) {
            if (lo) {
#pragma unroll
                for (int j = 0; j < NS; ++j) hd[2 + n + k * NS + j] = sg[j];
#pragma unroll
                for (int r = 0; r < MC; ++r) {
                    hd[ht + k * MC + r] = t[r];
                    hd[ht + m + k * MC + r] = lam[r];
                }
            } else {
#pragma unroll
                for (int r = 0; r < NI; ++r) {  // input rows of u_k: ms + (k nu + i) 2 + (lb ? 1 : 0)
                    hd[ht + ms + k * NI + r] = t[r];
                    hd[ht + m + ms + k * NI + r] = lam[r];
                }
            }
        }
    };
    wsync();
    if constexpr (W2) __syncthreads();  // wave 0's shared images
    if (own) {
#pragma unroll
        for (int r = 0; r < RX; ++r)
            if ((lo ? r < MC : r < NI) && isfinite(wv(r))) actm |= 1u << r;
    }
#define ACT(r) ((actm >> (r)) & 1u)
    constexpr bool kSeg = seg_on<T, NX, NU, LS>();
    double* sPhi = sm + L.Phi;
    // x_{k+1} = A_k x_k + B_k u_k, by segments where the instantiation has them.  The lane index is
    // an argument: inside the iteration loop it is the loop's own (opaque) copy, so the segment
    // bounds derived from it are recomputed there instead of hoisted and held across the loop
    auto fwd = [&](int lv, const double* x0v, const double* Uv, double* Xv) __attribute__((always_inline)) {
        if constexpr (kSeg) fwd3seg<NX, NU>(lv, N, sA, sB, x0v, Uv, Xv, sPhi);
        else fwd3<NX, NU, LS>(lv, N, sA, sB, x0v, Uv, Xv);
    };
    double* sPst = sm + L.Pst;
    if constexpr (kSeg) {
        if (wvi == 0) {
            phi_build<NX>(l, N, sA, sPhi);
            psi_build<NX>(l, N, sA, sPst);
        }
        wsync();
    }
    if constexpr (W2) __syncthreads();  // wave 0's transitions
    fwd(l, sx0, U, X);
    wsync();

    // value of row r at (Xv, Uv[, sig]) for this lane's rows
    auto rowval = [&](int r, const double* Xv, const double* Uv, bool with_sig) -> double {
        const double* xk = Xv + (k + 1) * NX;
        double v = 0.0;
        if constexpr (LS) {  // the rows' nonzeros only (the dense form adds exact zeros: same bits)
            const double* cr = sC + k * CW;
            if (r < 2) v = cr[r] * xk[0];
            else if (r < 4) v = cr[r] * xk[3];
            else v = fma(cr[4 + 2 * (r - 4) + 1], xk[8], cr[4 + 2 * (r - 4)] * xk[7]);
        } else if constexpr (DS) {  // the dense chain's nonzero terms, from the same +0 start
            if (r < 2) v = fma(r == 0 ? -1.0 : 1.0, xk[2], 0.0);
            else if (r < 4) v = fma(r == 2 ? 1.0 : -1.0, xk[1], 0.0);
            else {
                const double* cr = sC + k * CWD + 2 * (r - 4);
                v = fma(cr[1], xk[1], fma(cr[0], xk[0], 0.0));
            }
        } else {
            const double* cr = sC + (k * MC + r) * NX;
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                const double cs = cr[s], xs = xk[s];
                v = fma(cs, xs, v);
            }
        }
        if (with_sig && slk(r) >= 0) v += sgn(r) * sg[slk(r)];
        const double u = Uv[k * NU + (r >> 1)];
        const double uu = (r & 1) ? -u : u;
        return lo ? v : uu;
    };

    double mact_l = 0.0, sp_l = 1.0;
#pragma unroll
    for (int r = 0; r < RX; ++r) {
        if (ACT(r)) {
            const double w = wv(r);
            t[r] = fmax(w - rowval(r, X, U, true), kT0FloorCond);
            lam[r] = 1.0;
            mact_l += 1.0;
            sp_l = fmax(sp_l, fabs(w));
        } else {
            t[r] = 1.0;
            lam[r] = 0.0;
        }
        th[r] = rp[r] = rho[r] = gdu[r] = 0.0;
    }
    const double mact = fmax(wave_sum(mact_l), 1.0);
    const double scale_p = wave_max(sp_l);
    STAMP(14);

    // best iterate by merit max(res, 1e4 mu) (< tol <=> converged), returned when the method
    // stops short of convergence (iteration cap, factorisation breakdown, stagnation)
    double best_m = INFINITY, best_kkt = INFINITY, bsg[NS] = {0.0, 0.0, 0.0};
    int best_it = 0, stop = kStopMaxIter, it;
    double kkt = INFINITY;
    // iDs: 1 / D_sigma of the stage's slack groups (one division each per iteration; the W build, rho~
    // and the slack directions multiply by it)
    double iDs[NS] = {1.0, 1.0, 1.0}, rsig[NS] = {0.0, 0.0, 0.0}, dsg[NS] = {0.0, 0.0, 0.0};
    v4d acc[NT];
    double alpha_prev = 1;  // step of the previous iteration (kShortStep guard)
    for (it = 1; it <= c.max_iter; ++it) {
        // Opaque zero: the lane-index arithmetic and lane masks below are recomputed inside the
        // iteration instead of being hoisted out of it by LICM (hoisted, they held hundreds of
        // registers for the whole solve and spilled to scratch).
        int oz_;
        asm volatile("v_mov_b32 %0, 0" : "=v"(oz_));
        const int l = l0 + oz_;
        const bool lo = l < 32;
        const int k = l & 31;
        const bool own = k < N;
        // ================= residuals =================
        for (int i = l; i < (N + 1) * NX; i += 64) {
            const int kk = i / NX, s = i - kk * NX;
            double v = 2.0 * sP[i];
#pragma unroll
            for (int u = 0; u < NX; ++u) v = fma(Q2[s * NX + u], X[kk * NX + u], v);
            yb[i] = v;
        }
        wsync();
        // second adjoint input (in dX) = yb + C' lambda on stages 1..N
        if (lo && own) {
            if constexpr (LS) {
                const double* cr = sC + k * CW;
                static_for<0, NX>([&](auto s_c) __attribute__((always_inline)) {
                    constexpr int s2 = decltype(s_c)::value;
                    double v = yb[(k + 1) * NX + s2];
                    if constexpr (s2 == 0) v = fma(lam[1], cr[1], fma(lam[0], cr[0], v));
                    if constexpr (s2 == 3) v = fma(lam[3], cr[3], fma(lam[2], cr[2], v));
                    if constexpr (s2 == 7 || s2 == 8) {
#pragma unroll
                        for (int q = 0; q < NB; ++q) v = fma(lam[4 + q], cr[4 + 2 * q + (s2 - 7)], v);
                    }
                    dX[(k + 1) * NX + s2] = v;
                });
            } else if constexpr (DS) {
                const double* cr = sC + k * CWD;
                const double* y = yb + (k + 1) * NX;
                double v0 = y[0], v1 = y[1], v2 = y[2];
                v1 = fma(lam[3], -1.0, fma(lam[2], 1.0, v1));
                v2 = fma(lam[1], 1.0, fma(lam[0], -1.0, v2));
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    v0 = fma(lam[4 + q], cr[2 * q], v0);
                    v1 = fma(lam[4 + q], cr[2 * q + 1], v1);
                }
                double* d = dX + (k + 1) * NX;
                d[0] = v0;
                d[1] = v1;
                d[2] = v2;
                d[3] = y[3];
            } else {
#pragma unroll
                for (int s = 0; s < NX; ++s) {
                    double v = yb[(k + 1) * NX + s];
#pragma unroll
                    for (int r = 0; r < MC; ++r) v = fma(lam[r], sC[(k * MC + r) * NX + s], v);
                    dX[(k + 1) * NX + s] = v;
                }
            }
        }
        if (l < NX) dX[l] = yb[l];
        wsync();
        STAMP(0);
        // psi over yb (-> gradient) and over dX (-> rd): two 30-stage chains side by side on the rows of
        // the wave (segmenting both on the quads of the rows measured slower: 3.7k -> 3.9k clk)
        psi3<NX, LS>(l, N, sA, yb, dX);
        wsync();
        STAMP(1);
        double gs_l = 1.0, nrd_l = 0.0, nrs_l = 0.0, nrp_l = 0.0, mu_l = 0.0;
        if (own) {
            if (lo) {
#pragma unroll
                for (int j = 0; j < NS; ++j) {
                    double v = Qs2[j] * sg[j];
#pragma unroll
                    for (int r = 0; r < MC; ++r)
                        if (slk(r) == j) v += sgn(r) * lam[r];
                    rsig[j] = v;
                    nrs_l = nmax(nrs_l, fabs(v));
                }
            } else {
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    const int ci = k * NU + i;
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j < NU; ++j) {
                        const double uk = U[k * NU + j];
                        const double duk = uk - (k ? U[(k - 1) * NU + j] : sup[j]);
                        const double dun = (k + 1 < N) ? U[(k + 1) * NU + j] - uk : 0.0;
                        v += R2[i * NU + j] * uk + dR2[i * NU + j] * (duk - dun);
                    }
                    const double g = bpsi3<NX, NU, LS>(sB, yb, k, i) + v;
                    const double rdv = bpsi3<NX, NU, LS>(sB, dX, k, i) + v + lam[2 * i] - lam[2 * i + 1];
                    rd[ci] = rdv;
                    gs_l = nmax(gs_l, fabs(g));
                    nrd_l = nmax(nrd_l, fabs(rdv));
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RX; ++r) {
            const double rvr = rowval(r, X, U, true), wr = wv(r);
            if (ACT(r)) {
                rp[r] = rvr + t[r] - wr;
                nrp_l = nmax(nrp_l, fabs(rp[r]));
                mu_l += t[r] * lam[r];
            } else {
                rp[r] = 0.0;
            }
        }
        const double mu = wave_sum(mu_l) / mact;
        const double res = nmax(nmax(wave_max(nrd_l) / wave_max(gs_l), wave_max(nrs_l) / c.qs_max),
                                wave_max(nrp_l) / scale_p);
        kkt = nmax(res, mu);
        STAMP(2);
        const double merit = nmax(res, 1e4 * mu);
#ifdef CMPC_DBG_MERIT  // lab: the merit of iterations 1..15 (instead of the section clocks)
        if (l == 0 && wvi == 0 && P.stamps && it < kStampSlots)
            P.stamps[(size_t)b * kStampSlots + it] = (unsigned long long)__double_as_longlong(merit);
#endif
        if constexpr (W2) {
            // wave 0 decides for the pair: the waves hold identical values, and taking wave 0's verdict at a
            // barrier keeps any divergence from leaving one wave waiting at a barrier the other never reaches
            int dec = 0;
            if (!isfinite(merit)) {
                dec = kStopNonFinite;
            } else {
                if (merit < best_m) {
                    best_m = merit;
                    best_kkt = kkt;
                    best_it = it;
                    for (int i = l; i < NP; i += 64) bU[i] = U[i];
#pragma unroll
                    for (int j = 0; j < NS; ++j) bsg[j] = sg[j];
                }
                if (merit < c.tol) dec = kStopConverged;
                else if (best_m < 1e3 * c.tol && it - best_it >= kStallIters) dec = kStopStalled;
            }
            if (wvi == 0 && l == 0) sm[L.xf + 1] = (double)dec;
            __syncthreads();
            dec = (int)sm[L.xf + 1];
            if (dec) {
                stop = dec;
                break;
            }
        } else {
        if (!isfinite(merit)) {
            stop = kStopNonFinite;
            break;
        }
        if (merit < best_m) {
            best_m = merit;
            best_kkt = kkt;
            best_it = it;
            for (int i = l; i < NP; i += 64) bU[i] = U[i];
#pragma unroll
            for (int j = 0; j < NS; ++j) bsg[j] = sg[j];
        }
        if (merit < c.tol) {
            stop = kStopConverged;
            break;
        }
        if (best_m < 1e3 * c.tol && it - best_it >= kStallIters) {
            stop = kStopStalled;
            break;
        }
        }

        // ================= Newton matrix K = Gamma' W Gamma + Hc + diag =================
        // theta = lam / t through 1 / t_r, and 1 / D_sigma.  The passes need 1 / t_r, theta and 1 / D_sigma
        // again: they recompute them after the factorisation, bit for bit, rather than hold 15 doubles
        // in registers across the K build and the Cholesky (held, they made the T = 4 instantiation
        // spill to scratch).  `oz` is an opaque zero that keeps the compiler from merging the two.
        double tin[RX];
        auto theta = [&](double oz) __attribute__((always_inline)) {
#pragma unroll
            for (int r = 0; r < RX; ++r) tin[r] = ACT(r) ? 1.0 / (t[r] + oz) : 0.0;
#pragma unroll
            for (int r = 0; r < RX; ++r) th[r] = lam[r] * tin[r];
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                double v = Qs2[j];
#pragma unroll
                for (int r = 0; r < MC; ++r)
                    if (slk(r) == j) v += th[r];
                iDs[j] = 1.0 / v;
            }
        };
        theta(0.0);
        if (own) {
            if (lo) {
                // W_{k+1} = 2Q + sum_r th'_r c_r c_r' + sum_{pairs in a slack group} phi (a_r - a_r')(a_r - a_r')'
                double thp[MC];
#pragma unroll
                for (int r = 0; r < MC; ++r) thp[r] = slk(r) < 0 ? th[r] : Qs2[slk(r)] * th[r] * iDs[slk(r)];
                if constexpr (LS) {
                    // block diagonal (Q diagonal, rows on vx / ey / (X, Y)): the five entries that are
                    // not 2Q's, accumulated in the dense build's order
                    const double* cr = sC + k * CW;
                    double wvx = fma(thp[1] * cr[1], cr[1], fma(thp[0] * cr[0], cr[0], Q2[0]));
                    double wey = fma(thp[3] * cr[3], cr[3], fma(thp[2] * cr[2], cr[2], Q2[3 * NX + 3]));
                    const double phi23 = th[2] * th[3] * iDs[1], d23 = cr[2] - cr[3];
                    wey = fma(phi23 * d23, d23, wey);
                    double wxx = Q2[7 * NX + 7], wxy = Q2[7 * NX + 8], wyy = Q2[8 * NX + 8];
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        const double ax = cr[4 + 2 * q], ay = cr[5 + 2 * q];
                        wxx = fma(thp[4 + q] * ax, ax, wxx);
                        wxy = fma(thp[4 + q] * ax, ay, wxy);
                        wyy = fma(thp[4 + q] * ay, ay, wyy);
                    }
#pragma unroll
                    for (int q = 0; q < NB; ++q)
#pragma unroll
                        for (int q2 = q + 1; q2 < NB; ++q2) {  // plane rows share slack 2, sign -1
                            const double phi = th[4 + q] * th[4 + q2] * iDs[2];
                            const double dx = cr[4 + 2 * q2] - cr[4 + 2 * q], dy = cr[5 + 2 * q2] - cr[5 + 2 * q];
                            wxx = fma(phi * dx, dx, wxx);
                            wxy = fma(phi * dx, dy, wxy);
                            wyy = fma(phi * dy, dy, wyy);
                        }
                    double* wk = sW + k * kLsW;
                    wk[0] = wvx;
                    wk[1] = wey;
                    wk[2] = wxx;
                    wk[3] = wxy;
                    wk[4] = wyy;
                } else if constexpr (DS) {
                    // the dense build's entries that are not exact zeros, term by term in its order
                    // (rows r, then the slack pairs: (2, 3) in group 1, the plane pairs in group 2)
                    const double* cr = sC + k * CWD;
                    double wxx = Q2[0], wxy = Q2[1], wyx = Q2[NX], wyy = Q2[NX + 1];
                    double wvx = Q2[2 * NX + 2];
                    wvx = fma(thp[0] * -1.0, -1.0, wvx);
                    wvx = fma(thp[1] * 1.0, 1.0, wvx);
                    wyy = fma(thp[2] * 1.0, 1.0, wyy);
                    wyy = fma(thp[3] * -1.0, -1.0, wyy);
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        const double ax = cr[2 * q], ay = cr[2 * q + 1], tq = thp[4 + q];
                        wxx = fma(tq * ax, ax, wxx);
                        wxy = fma(tq * ax, ay, wxy);
                        wyx = fma(tq * ay, ax, wyx);
                        wyy = fma(tq * ay, ay, wyy);
                    }
                    {  // rows 2, 3 (slack 1, signs +1): a_2 - a_3 = 2 on p_y
                        const double phi = th[2] * th[3] * iDs[1], ds = 1.0 * 1.0 - 1.0 * -1.0;
                        wyy = fma(phi * ds, ds, wyy);
                    }
#pragma unroll
                    for (int q = 0; q < NB; ++q)
#pragma unroll
                        for (int q2 = q + 1; q2 < NB; ++q2) {  // plane rows: slack 2, signs -1
                            const double phi = th[4 + q] * th[4 + q2] * iDs[2];
                            const double dx = -1.0 * cr[2 * q] - -1.0 * cr[2 * q2];
                            const double dy = -1.0 * cr[2 * q + 1] - -1.0 * cr[2 * q2 + 1];
                            wxx = fma(phi * dx, dx, wxx);
                            wxy = fma(phi * dx, dy, wxy);
                            wyx = fma(phi * dy, dx, wyx);
                            wyy = fma(phi * dy, dy, wyy);
                        }
                    double* wk = sW + k * kDsW;
                    wk[0] = wxx;
                    wk[1] = wxy;
                    wk[2] = wyx;
                    wk[3] = wyy;
                    wk[4] = wvx;
                    wk[5] = Q2[3 * NX + 3];
                } else {
                // the stage's rows and 2Q into registers in one batch of LDS reads (read inside the
                // loops below they were issued one dependent wait at a time)
                // (small NX only: larger ones would not fit the VGPR file and read in place)
                constexpr bool kWr = NX * (MC + NX) <= 48;
                constexpr int PC = kWr ? MC * NX : 1, PQ = kWr ? NX * NX : 1;
                double ckr[PC], q2r[PQ];
                if constexpr (kWr) {
#pragma unroll
                    for (int i = 0; i < PC; ++i) ckr[i] = sC[k * MC * NX + i];
#pragma unroll
                    for (int i = 0; i < PQ; ++i) q2r[i] = Q2[i];
                }
                const double* Ckp = sC + k * MC * NX;
                auto Ck_ = [&](int i) __attribute__((always_inline)) {
                    if constexpr (kWr) return ckr[i];
                    else return Ckp[i];
                };
                auto q2_ = [&](int i) __attribute__((always_inline)) {
                    if constexpr (kWr) return q2r[i];
                    else return Q2[i];
                };
#pragma unroll
                for (int s = 0; s < NX; ++s)
#pragma unroll
                    for (int u = 0; u < NX; ++u) {
                        double v = q2_(s * NX + u);
#pragma unroll
                        for (int r = 0; r < MC; ++r) v = fma(thp[r] * Ck_(r * NX + s), Ck_(r * NX + u), v);
#pragma unroll
                        for (int r = 0; r < MC; ++r) {
                            if (slk(r) < 0) continue;
#pragma unroll
                            for (int r2 = r + 1; r2 < MC; ++r2) {
                                if (slk(r2) != slk(r)) continue;
                                const double phi = th[r] * th[r2] * iDs[slk(r)];
                                const double ds = sgn(r) * Ck_(r * NX + s) - sgn(r2) * Ck_(r2 * NX + s);
                                const double du = sgn(r) * Ck_(r * NX + u) - sgn(r2) * Ck_(r2 * NX + u);
                                v = fma(phi * ds, du, v);
                            }
                        }
                        sW[(k * NX + s) * NX + u] = v;
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < NU; ++i) thin[k * NU + i] = th[2 * i] + th[2 * i + 1];
            }
        }
        wsync();
        STAMP(3);
        // zero the accumulators with an MFMA so they are defined in the accumulator registers:
        // a VALU zero made the tiles first touched in a late horizon segment live in VGPRs and
        // cost a VGPR<->AGPR copy (and an MFMA-result stall) per stage
        {
            const v4d z4 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < NT; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(0.0, 0.0, z4, 0, 0, 0);
        }
        if constexpr (LS) {
            // the same contraction on the reference model's structure: Gamma_{k+1} = Gamma_k +
            // D_k Gamma_k[0..2] (+ B_k's column at its stage), and W_k Gamma_k from the block-diagonal
            // W_k (2Q's diagonal, the vx / ey entries, the (X, Y) block): 27 + 11 multiply-adds per
            // stage and lane instead of 81 + 81, 32 LDS reads instead of 162
            double g[NX], q2d[NX], bcol[NX];
            const int col = l;
            const int kc = col / NU, ic = col - kc * NU, kcl = kc < N ? kc : N - 1;
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2) {
                g[s2] = 0.0;
                q2d[s2] = Q2[s2 * NX + s2];
                const double bv = sB[(kcl * 3 + (s2 < 3 ? s2 : 0)) * NU + ic];
                bcol[s2] = s2 < 3 ? bv : 0.0;
            }
            auto stage = [&](auto tau_c, int kk) __attribute__((always_inline)) {
                constexpr int tau = decltype(tau_c)::value;
                const double* Dk = sA + kk * 27;
                const double* wk = sW + kk * kLsW;
                double dv[27], w5[kLsW];
#pragma unroll
                for (int i = 0; i < 27; ++i) dv[i] = Dk[i];
#pragma unroll
                for (int i = 0; i < kLsW; ++i) w5[i] = wk[i];
                const bool inj = kk == kc;
                double gn[NX];
#pragma unroll
                for (int s2 = 0; s2 < NX; ++s2) {
                    double v = 0.0;
#pragma unroll
                    for (int t2 = 0; t2 < 3; ++t2) v = fma(dv[s2 * 3 + t2], g[t2], v);
                    gn[s2] = inj ? bcol[s2] : v + g[s2];
                }
#pragma unroll
                for (int s2 = 0; s2 < NX; ++s2) g[s2] = gn[s2];
                // contraction slot j -> state s2 (L5: the five states W_k weights, zero padding after)
                constexpr int KP = L5 ? 8 : NXP;
                double gf[KP], yf[KP];
                static_for<0, KP>([&](auto j_c) __attribute__((always_inline)) {
                    constexpr int j = decltype(j_c)::value;
                    constexpr int s2 = L5 ? (j == 0 ? 0 : j == 1 ? 3 : j == 2 ? 4 : j == 3 ? 7 : j == 4 ? 8 : NX) : j;
                    if constexpr (s2 < NX) {
                        gf[j] = g[s2];
                        if constexpr (s2 == 0) yf[j] = w5[0] * g[0];
                        else if constexpr (s2 == 3) yf[j] = w5[1] * g[3];
                        else if constexpr (s2 == 7) yf[j] = fma(w5[3], g[8], w5[2] * g[7]);
                        else if constexpr (s2 == 8) yf[j] = fma(w5[4], g[8], w5[3] * g[7]);
                        else yf[j] = q2d[s2] * g[s2];
                    } else {
                        gf[j] = 0.0;
                        yf[j] = 0.0;
                    }
                });
#pragma unroll
                for (int q = 0; q < KP; q += 4) {
                    transpose_rows4(gf[q], gf[q + 1], gf[q + 2], gf[q + 3]);
                    transpose_rows4(yf[q], yf[q + 1], yf[q + 2], yf[q + 3]);
#pragma unroll
                    for (int ti = 0; ti <= tau; ++ti)
#pragma unroll
                        for (int tj = 0; tj <= ti; ++tj)
                            acc[ti * (ti + 1) / 2 + tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                                gf[q + ti], yf[q + tj], acc[ti * (ti + 1) / 2 + tj], 0, 0, 0);
                }
            };
            static_for<0, T>([&](auto tau_c) __attribute__((always_inline)) {
                constexpr int tau = decltype(tau_c)::value;
                const int kb = (16 * tau + NU) / NU - 1;
                const int ke0 = (16 * (tau + 1) + NU) / NU - 1;
                const int ke = ke0 < N ? ke0 : N;
                for (int kk = kb; kk < ke; ++kk) stage(tau_c, kk);
            });
        } else {
            // lane l carries column l of Gamma_k (Gamma_0 = 0) and of W_k Gamma_k; both reach the
            // MFMA fragment layout by an in-register row transpose (no LDS round trip).
            //  * column l = kc NU + ic is zero up to stage kc, where it becomes B_kc[:, ic]: the lane
            //    loads that column once and selects it at its stage (A_k Gamma_k is exactly 0 there);
            //  * for small NX, A_k is fetched one stage ahead into ping-pong registers (the stage
            //    loop is unrolled by two: no copies); larger NX read A_k in place.
            constexpr bool kPf = NX * NX <= 16;
            constexpr int PA = kPf ? NX * NX : 1;
            double g[NX];
#pragma unroll
            for (int s = 0; s < NX; ++s) g[s] = 0.0;
            const int col = l;
            const int kc = col / NU, ic = col - kc * NU, kcl = kc < N ? kc : N - 1;
            double bcol[NX];
#pragma unroll
            for (int s = 0; s < NX; ++s) bcol[s] = sB[(kcl * NX + s) * NU + ic];
            double a0[PA], a1[PA];
            auto fetchA = [&](int kk, double* av) __attribute__((always_inline)) {
                if constexpr (kPf) {
#pragma unroll
                    for (int i = 0; i < PA; ++i) av[i] = sA[kk * NX * NX + i];
                }
            };
            fetchA(0, a0);
            // W_k is loaded first, then the next stage's A (pf): LDS returns in order, so W_k's wait
            // (after the Gamma chain) does not include the prefetch
            // role: 2 every tile (one wave per agent); W2: 0 / 1 the tiles of wave 0 / 1 (w2_own0), each
            // wave's K build a copy of its own with a static MFMA set (no branch between accumulations)
            auto stage = [&](auto tau_c, auto role_c, int kk, const double* av, auto pf) __attribute__((always_inline)) {
                constexpr int tau = decltype(tau_c)::value;
                constexpr int role = decltype(role_c)::value;
                const double* Ak = sA + kk * NX * NX;
                const double* Wk = sW + kk * (DS ? kDsW : NX * NX);
                constexpr int PW = DS ? kDsW : PA;
                double wk[PW];
                if constexpr (kPf || DS) {
#pragma unroll
                    for (int i = 0; i < PW; ++i) wk[i] = Wk[i];
                }
                pf();
                __builtin_amdgcn_sched_barrier(0);
                auto A_ = [&](int i) __attribute__((always_inline)) {
                    if constexpr (kPf) return av[i];
                    else return Ak[i];
                };
                auto W_ = [&](int i) __attribute__((always_inline)) {
                    if constexpr (kPf) return wk[i];
                    else return Wk[i];
                };
                const bool inj = kk == kc;
                double gn[NX];
#pragma unroll
                for (int s = 0; s < NX; ++s) {
                    double v = 0.0;
#pragma unroll
                    for (int u = 0; u < NX; ++u) v = fma(A_(s * NX + u), g[u], v);
                    gn[s] = inj ? bcol[s] : v;
                }
#pragma unroll
                for (int s = 0; s < NX; ++s) g[s] = gn[s];
                double gf[NXP], yf[NXP];
                static_for<0, NXP>([&](auto s_c) __attribute__((always_inline)) {
                    constexpr int s = decltype(s_c)::value;
                    double y = 0.0;
                    if constexpr (DS && s < NX) {  // W_k's nonzero entries (kDsW order), the dense chain's terms
                        if constexpr (s == 0) y = fma(wk[1], g[1], fma(wk[0], g[0], 0.0));
                        else if constexpr (s == 1) y = fma(wk[3], g[1], fma(wk[2], g[0], 0.0));
                        else y = fma(wk[s + 2], g[s], 0.0);
                        gf[s] = g[s];
                    } else if constexpr (s < NX) {
#pragma unroll
                        for (int u = 0; u < NX; ++u) y = fma(W_(s * NX + u), g[u], y);
                        gf[s] = g[s];
                    } else {
                        gf[s] = 0.0;
                    }
                    yf[s] = y;
                });
#pragma unroll
                for (int q = 0; q < NXP; q += 4) {
                    transpose_rows4(gf[q], gf[q + 1], gf[q + 2], gf[q + 3]);
                    transpose_rows4(yf[q], yf[q + 1], yf[q + 2], yf[q + 3]);
                    static_for<0, tau + 1>([&](auto ti_c) __attribute__((always_inline)) {
                        constexpr int ti = decltype(ti_c)::value;
                        static_for<0, ti + 1>([&](auto tj_c) __attribute__((always_inline)) {
                            constexpr int tj = decltype(tj_c)::value;
                            if constexpr (role == 2 || w2_own0(T, ti, tj) == (role == 0))
                                acc[ti * (ti + 1) / 2 + tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                                    gf[q + ti], yf[q + tj], acc[ti * (ti + 1) / 2 + tj], 0, 0, 0);
                        });
                    });
                }
            };
            auto kbuild = [&](auto role_c) __attribute__((always_inline)) {
            static_for<0, T>([&](auto tau_c) __attribute__((always_inline)) {
                constexpr int tau = decltype(tau_c)::value;
                // stages whose Gamma_{k+1} has tiles 0..tau nonzero (last column (k+1)NU-1 in tile tau)
                const int kb = (16 * tau + NU) / NU - 1;
                const int ke0 = (16 * (tau + 1) + NU) / NU - 1;
                const int ke = ke0 < N ? ke0 : N;
                int kk = kb;
                for (; kk + 1 < ke; kk += 2) {
                    stage(tau_c, role_c, kk, a0, [&]() __attribute__((always_inline)) { fetchA(kk + 1, a1); });
                    stage(tau_c, role_c, kk + 1, a1,
                          [&]() __attribute__((always_inline)) { fetchA(kk + 2 < N ? kk + 2 : N - 1, a0); });
                }
                if (kk < ke) {
                    stage(tau_c, role_c, kk, a0,
                          [&]() __attribute__((always_inline)) { fetchA(kk + 1 < N ? kk + 1 : N - 1, a1); });
#pragma unroll
                    for (int i = 0; i < PA; ++i) a0[i] = a1[i];
                }
            });
            };
            if constexpr (!W2) {
                kbuild(std::integral_constant<int, 2>{});
            } else if (wvi == 0) {
                kbuild(std::integral_constant<int, 0>{});
            } else {
                kbuild(std::integral_constant<int, 1>{});
            }
        }
        STAMP(4);
        if constexpr (W2) {  // wave 1's tiles to wave 0 (slot-major, [register][lane]: conflict-free)
            double* xk = sm + L.xk;
            if (wvi != 0) {
                static_for<0, T>([&](auto ti_c) __attribute__((always_inline)) {
                    constexpr int ti = decltype(ti_c)::value;
                    static_for<0, ti + 1>([&](auto tj_c) __attribute__((always_inline)) {
                        constexpr int tj = decltype(tj_c)::value;
                        if constexpr (!w2_own0(T, ti, tj)) {
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                xk[(w2_slot1(T, ti, tj) * 4 + r) * 64 + l] = acc[ti * (ti + 1) / 2 + tj][r];
                        }
                    });
                });
            }
            __syncthreads();
            if (wvi == 0) {
                static_for<0, T>([&](auto ti_c) __attribute__((always_inline)) {
                    constexpr int ti = decltype(ti_c)::value;
                    static_for<0, ti + 1>([&](auto tj_c) __attribute__((always_inline)) {
                        constexpr int tj = decltype(tj_c)::value;
                        if constexpr (!w2_own0(T, ti, tj)) {
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                acc[ti * (ti + 1) / 2 + tj][r] = xk[(w2_slot1(T, ti, tj) * 4 + r) * 64 + l];
                        }
                    });
                });
            }
        }
        // + 2R + 2D'dR D (block tridiagonal) + input-row curvature; identity on the padding.
        // The band half-width 2NU - 1 < 16 touches only the diagonal and first sub-diagonal tiles;
        // branch-free: unconditional (clamped) LDS reads and selects.
#pragma unroll
        for (int ti = 0; ti < T; ++ti)
#pragma unroll
            for (int tj = (ti > 0 ? ti - 1 : 0); tj <= ti; ++tj)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = ti * 16 + (l >> 4) + 4 * r, col = tj * 16 + (l & 15);
                    const int kr = row / NU, a = row - kr * NU, kc = col / NU, bq = col - kc * NU;
                    const double r2 = R2[a * NU + bq], d2 = dR2[a * NU + bq], thr = thin[row];
                    const bool in = row < n && col < n;
                    // 0/1 masks instead of selects around the loaded values (the compiler turns those
                    // into divergent branches with the loads inside); thin of a padding row may be
                    // garbage: the final select drops it
                    const double md = (kr == kc) ? 1.0 : 0.0, mo = (kr == kc + 1 || kc == kr + 1) ? 1.0 : 0.0;
                    const double me = (row == col) ? 1.0 : 0.0, f = (kr + 1 < N) ? 2.0 : 1.0;
                    double add = fma(md, fma(d2, f, r2), fma(md * me, thr, -mo * d2));
                    add = in ? add : me;
                    acc[ti * (ti + 1) / 2 + tj][r] += add;
                }
        STAMP(5);

        // ================= blocked Cholesky in the accumulator registers =================
        bool chol_ok = true;
        // diagonal blocks L_JJ -> L_JJ^{-1} in place (LDS, lower triangle; zeros above): row q of the
        // wave inverts block q, lane (q, j) forms column j by forward substitution.  Done once per
        // factorisation, it turns every in-block substitution of the four triangular solves per
        // iteration (16 dependent broadcast -> multiply -> fma steps) into a 16-term mat-vec
        auto invert_diag = [&]() __attribute__((always_inline)) {
            const int q = l >> 4, j = l & 15;
            double* Lq = Ld + (q < T ? q : 0) * 272;
            double x[16];
            static_for<0, 16>([&](auto i_c) __attribute__((always_inline)) {
                constexpr int i = decltype(i_c)::value;
                double s0 = (j == i) ? 1.0 : 0.0, s1 = 0.0;
#pragma unroll
                for (int c = 0; c < i; ++c) {
                    if (c & 1) s1 = fma(-Lq[i * 17 + c], x[c], s1);
                    else s0 = fma(-Lq[i * 17 + c], x[c], s0);
                }
                x[i] = (s0 + s1) * rcp_d(Lq[i * 17 + i]);
            });
            wsync();
            if (q < T) {
#pragma unroll
                for (int i = 0; i < 16; ++i) Lq[i * 17 + j] = x[i];
            }
            wsync();
        };
        if (!W2 || wvi == 0) {
#pragma unroll
        for (int J = 0; J < T; ++J) {
            const int JJ = J * (J + 1) / 2 + J;
            double* S0 = Ld + J * 272;
#pragma unroll
            for (int r = 0; r < 4; ++r) S0[((l >> 4) + 4 * r) * 17 + (l & 15)] = acc[JJ][r];
            wsync();
            // 16x16 diagonal factor: every row of 16 lanes holds the block (lane i: row i), pivots and
            // L columns move by DPP row_newbcast; 1/sqrt by rsq + Newton
            double rw[16];
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) rw[cc] = S0[(l & 15) * 17 + cc];
            {
                // pivot chain: lane j+1's next diagonal entry is its own update fma(-l, l, d) (the
                // broadcast of its own l is l itself: same bits), so the chain between pivots is
                // rsq + Newton -> l -> fma -> one broadcast.  l = rw[j] y on every lane: on lane j,
                // rw[j] is the pivot itself (= djj), above the diagonal the values are never read
                // (the store below writes zeros there)
                double dn = 0.0;
                static_for<0, 16>([&](auto jc) __attribute__((always_inline)) {
                    constexpr int j = decltype(jc)::value;
                    const double djj = bcast16<j>(j == 0 ? rw[0] : dn);
                    if (!(djj > 0.0)) chol_ok = false;
                    const double y = rsqrt_d(djj);
                    const double lj = rw[j] * y;
                    rw[j] = lj;
                    if constexpr (j + 1 < 16) dn = fma(-lj, lj, rw[j + 1]);
                    static_for<j + 1, 16>([&](auto cc) __attribute__((always_inline)) {
                        constexpr int c2 = decltype(cc)::value;
                        rw[c2] = fma(-lj, bcast16<c2>(lj), rw[c2]);
                    });
                    // (no scheduling barrier: the next pivot overlaps this one's trailing updates)
                });
            }
            if (l < 16) {
#pragma unroll
                for (int cc = 0; cc < 16; ++cc) S0[l * 17 + cc] = (cc <= l) ? rw[cc] : 0.0;
            }
            wsync();
            STAMP(6);
            if (J + 1 < T) {
                // panel TRSM in the accumulator layout: L_IJ = K_IJ L_JJ^{-T} column by column; lane l
                // holds column (l & 15) of every panel tile, its own row of L_JJ in rw (lane = row), so
                // L[l & 15][cc] = rw[cc] and Y[:, cc] reaches the row of 16 lanes by DPP row_newbcast.
                // Unscaled form: with y_c = x_c L_cc the update is k_i -= y_c (L_ic / L_cc) for i > c
                // (a zero multiplier elsewhere), so each step is one broadcast and one fma per value;
                // x = y / L_ii once at the end
                {
                    const int i16 = l & 15;
                    const double inv_own = 1.0 / S0[i16 * 17 + i16];
                    static_for<0, 16>([&](auto jc) __attribute__((always_inline)) {
                        constexpr int cc = decltype(jc)::value;
                        // the broadcast stays outside the select: under a divergent EXEC mask the
                        // source lane cc would be inactive (DPP then reads 0)
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
                }
                // stacked panel rows to LDS for the transposed MFMA operands of the SYRK
#pragma unroll
                for (int I = J + 1; I < T; ++I)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        SP[((I - J - 1) * 16 + (l >> 4) + 4 * r) * 17 + (l & 15)] = acc[I * (I + 1) / 2 + J][r];
                wsync();
                // trailing SYRK: K_IK -= L_IJ L_KJ'  (I >= K > J) on MFMA
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
            STAMP(7);
        }
        }
        // ================= predictor / corrector =================
        double sig_c = 0.0, alpha = 0.0;
        // the right-hand side of a pass: rho (pass 1: Mehrotra's second-order term from the predictor still
        // in (rho, gdu, dsg)), C' rho~ into yb, the adjoint recursion, vb
        auto pass_rhs = [&](int pass) __attribute__((always_inline)) {
            // pass 1: Mehrotra's second-order term dt_aff * dl_aff from the predictor still in (rho, gdu, dsg)
#pragma unroll
            for (int r = 0; r < RX; ++r) {
                if (!ACT(r)) {
                    rho[r] = 0.0;
                    continue;
                }
                double rc = -t[r] * lam[r];
                if (pass) {
                    const double sd = (lo && slk(r) >= 0) ? sgn(r) * dsg[slk(r)] : 0.0;
                    const double dta = -rp[r] - gdu[r] - sd;
                    const double dla = rho[r] + th[r] * (gdu[r] + sd);
                    rc += sig_c * mu - dta * dla;
                }
                rho[r] = (rc + lam[r] * rp[r]) * tin[r];
            }
            // rho~ (stable slack-group form) of the stage rows enters only through C' rho~
            if (lo && own) {
                double ybv[NX];
#pragma unroll
                for (int s = 0; s < NX; ++s) ybv[s] = 0.0;
#pragma unroll
                for (int r = 0; r < MC; ++r) {
                    double v = rho[r];
                    if (slk(r) >= 0) {
                        const int j = slk(r);
                        v = Qs2[j] * rho[r] - th[r] * sgn(r) * rsig[j];
#pragma unroll
                        for (int r2 = 0; r2 < MC; ++r2) {
                            if (r2 == r || slk(r2) != j) continue;
                            v += th[r2] * rho[r] - th[r] * sgn(r) * sgn(r2) * rho[r2];
                        }
                        v *= iDs[j];
                    }
                    if constexpr (LS) {  // the row's nonzeros (same accumulation order)
                        const double* cr = sC + k * CW;
                        if (r < 2) ybv[0] = fma(v, cr[r], ybv[0]);
                        else if (r < 4) ybv[3] = fma(v, cr[r], ybv[3]);
                        else {
                            ybv[7] = fma(v, cr[4 + 2 * (r - 4)], ybv[7]);
                            ybv[8] = fma(v, cr[5 + 2 * (r - 4)], ybv[8]);
                        }
                    } else if constexpr (DS) {  // -v_x, v_x, p_y, -p_y, planes on (p_x, p_y)
                        if (r < 2) ybv[2] = fma(v, r == 0 ? -1.0 : 1.0, ybv[2]);
                        else if (r < 4) ybv[1] = fma(v, r == 2 ? 1.0 : -1.0, ybv[1]);
                        else {
                            const double* cr = sC + k * CWD + 2 * (r - 4);
                            ybv[0] = fma(v, cr[0], ybv[0]);
                            ybv[1] = fma(v, cr[1], ybv[1]);
                        }
                    } else {
#pragma unroll
                        for (int s = 0; s < NX; ++s) ybv[s] = fma(v, sC[(k * MC + r) * NX + s], ybv[s]);
                    }
                }
#pragma unroll
                for (int s = 0; s < NX; ++s) yb[(k + 1) * NX + s] = ybv[s];
            }
            if (l < NX) yb[l] = 0.0;
            wsync();
            STAMP(8);
            if constexpr (kSeg) psi3seg<NX>(l, N, sA, yb, sPst);
            else psi3<NX, LS>(l, N, sA, yb, yb);
            wsync();
            STAMP(9);
            if (!lo && own) {
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    const int ci = k * NU + i;
                    vb[ci] = -rd[ci] - (bpsi3<NX, NU, LS>(sB, yb, k, i) + rho[2 * i] - rho[2 * i + 1]);
                }
            }
            wsync();
        };
        if constexpr (W2) {
            // wave 1 forms the predictor's right-hand side while wave 0 factors; then rho (per lane) and vb
            // change hands, with wave 0's factorisation verdict
            if (kW2Rhs && wvi != 0) {
                int ozi;
                asm volatile("v_mov_b32 %0, 0" : "=v"(ozi));
                theta((double)ozi);
                pass_rhs(0);
#pragma unroll
                for (int r = 0; r < RX; ++r) sm[L.xr + r * 64 + l] = rho[r];
                for (int i = l; i < NP; i += 64) sm[L.xv + i] = vb[i];
            } else if (l == 0) {
                sm[L.xf] = chol_ok ? 1.0 : 0.0;
            }
            __syncthreads();
            chol_ok = sm[L.xf] != 0.0;
        }
        if (!chol_ok) {
            stop = kStopBreakdown;
            if (wvi == 0 && c.rescue && P.ws) {  // hand the iterate to the Riccati rescue (hand_doubles, internal.h)
                write_image();
                if (l == 0) P.ws[(size_t)b * c.ws_stride + 1] = it - 1;
            }
            break;
        }
        if (wvi == 0) invert_diag();  // (W2: after the hand-over; before it, its registers spilled)
        // this lane's diagonal block (J = lane >> 4) of L^{-1}: row / column (l & 15)
        const double* Lme = Ld + ((l >> 4) < T ? (l >> 4) : 0) * 272;
        if (wvi == 0) {
            int ozi;
            asm volatile("v_mov_b32 %0, 0" : "=v"(ozi));
            theta((double)ozi);
        }
        for (int pass = 0; pass < 2; ++pass) {
            if (!W2 || !kW2Rhs || pass) {
                pass_rhs(pass);
            } else if (wvi == 0) {  // W2, pass 0: wave 1's rho and vb
#pragma unroll
                for (int r = 0; r < RX; ++r) rho[r] = sm[L.xr + r * 64 + l];
                for (int i = l; i < NP; i += 64) vb[i] = sm[L.xv + i];
                wsync();
            }
            if (wvi == 0) {  // (W2: the triangular solves on wave 0, which holds L)
            // ---- forward solve L y = vb (block rows; L_JI tiles in acc, L_JJ in LDS) ----
            // this lane's row of its row group's inverted diagonal block: the same for every J
            // (only row group J's result is kept), so it is loaded once, not per block row
            double Lr[16];
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) Lr[cc] = Lme[(l & 15) * 17 + cc];
#pragma unroll
            for (int J = 0; J < T; ++J) {
                double pr4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int I = 0; I < J; ++I) {
                    const double yv = vb[I * 16 + (l & 15)];
#pragma unroll
                    for (int r = 0; r < 4; ++r) pr4[r] = fma(acc[J * (J + 1) / 2 + I][r], yv, pr4[r]);
                }
                if (J > 0) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) pr4[r] = sum16(pr4[r]);
                    if ((l & 15) == 0) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) red[(l >> 4) + 4 * r] = pr4[r];
                    }
                    wsync();
                }
                double rv = 0.0;
                if ((l >> 4) == J) rv = vb[J * 16 + (l & 15)] - (J > 0 ? red[l & 15] : 0.0);
                {  // y_J = L_JJ^{-1} r_J: row J broadcasts its lanes, four independent fma chains
                    double y4[4] = {0.0, 0.0, 0.0, 0.0};
                    static_for<0, 16>([&](auto jc) __attribute__((always_inline)) {
                        constexpr int cc = decltype(jc)::value;
                        y4[cc & 3] = fma(Lr[cc], bcast16<cc>(rv), y4[cc & 3]);
                    });
                    rv = (y4[0] + y4[1]) + (y4[2] + y4[3]);
                }
                if ((l >> 4) == J) vb[J * 16 + (l & 15)] = rv;
                wsync();
            }
            // ---- backward solve L' x = y ----
            double Lc[16];  // column of the inverted diagonal block, loaded once (as Lr)
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) Lc[cc] = Lme[cc * 17 + (l & 15)];
#pragma unroll
            for (int J = T - 1; J >= 0; --J) {
                double p = 0.0;
#pragma unroll
                for (int I = J + 1; I < T; ++I)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        p = fma(acc[I * (I + 1) / 2 + J][r], vb[I * 16 + (l >> 4) + 4 * r], p);
                if (J + 1 < T) p = sum_groups(p);
                double rv = ((l >> 4) == J) ? vb[J * 16 + (l & 15)] - p : 0.0;
                {  // x_J = L_JJ^{-T} r_J
                    double x4[4] = {0.0, 0.0, 0.0, 0.0};
                    static_for<0, 16>([&](auto jc) __attribute__((always_inline)) {
                        constexpr int cc = decltype(jc)::value;
                        x4[cc & 3] = fma(Lc[cc], bcast16<cc>(rv), x4[cc & 3]);
                    });
                    rv = (x4[0] + x4[1]) + (x4[2] + x4[3]);
                }
                if ((l >> 4) == J) vb[J * 16 + (l & 15)] = rv;
                wsync();
            }
            for (int i = l; i < NP; i += 64) dU[i] = (i < n) ? vb[i] : 0.0;
            }
            if constexpr (W2) {  // each pass's dU to wave 1 (one slot per pass)
                double* xu = sm + (pass ? L.xu1 : L.xu0);
                if (wvi == 0)
                    for (int i = l; i < NP; i += 64) xu[i] = dU[i];
                __syncthreads();
                if (wvi != 0)
                    for (int i = l; i < NP; i += 64) dU[i] = xu[i];
            }
            wsync();
            STAMP(10);
            fwd(l, nullptr, dU, dX);
            wsync();
            STAMP(11);
#pragma unroll
            for (int r = 0; r < RX; ++r) {
                const double rvr = rowval(r, dX, dU, false);
                gdu[r] = ACT(r) ? rvr : 0.0;
            }
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                double v = rsig[j];
#pragma unroll
                for (int r = 0; r < MC; ++r)
                    if (slk(r) == j) v += sgn(r) * (rho[r] + th[r] * gdu[r]);
                dsg[j] = (lo && own) ? -v * iDs[j] : 0.0;
            }
            // dt_r = -rp - G dU - s dsig ;  dl_r = rho + th (G dU + s dsig)
            auto sdr = [&](int r) -> double { return (lo && slk(r) >= 0) ? sgn(r) * dsg[slk(r)] : 0.0; };
            double amax_l = 1.0e300;
#pragma unroll
            for (int r = 0; r < RX; ++r) {
                if (!ACT(r)) continue;
                const double sd = sdr(r);
                const double dtv = -rp[r] - gdu[r] - sd;
                const double dlv = rho[r] + th[r] * (gdu[r] + sd);
                // ratio tests by the hardware reciprocal: the step is cut to 0.995 of it anyway
                if (dtv < 0.0) amax_l = fmin(amax_l, -t[r] * __builtin_amdgcn_rcp(dtv));
                if (dlv < 0.0) amax_l = fmin(amax_l, -lam[r] * __builtin_amdgcn_rcp(dlv));
            }
            const double amax = wave_min(amax_l);
            if (!pass) {
                const double a = fmin(amax, 1.0);
                double mua_l = 0.0;
#pragma unroll
                for (int r = 0; r < RX; ++r) {
                    if (!ACT(r)) continue;
                    const double sd = sdr(r);
                    mua_l += (t[r] + a * (-rp[r] - gdu[r] - sd)) * (lam[r] + a * (rho[r] + th[r] * (gdu[r] + sd)));
                }
                const double mu_aff = wave_sum(mua_l) / mact;
                const double ratio = mu > 0.0 ? mu_aff / mu : 0.0;
                sig_c = ratio * ratio;  // (the condensed kernels: e = 2, internal.h)
                if (alpha_prev < kShortStep) sig_c = fmax(sig_c, kSigmaMin);
                STAMP(12);
            } else {
                alpha = fmin(1.0, 0.995 * amax);
                // stay in the wide neighbourhood t_r lam_r >= gamma mu(alpha) (see kNbhdGamma)
                for (int bt = 0; bt < kMaxBacktrack; ++bt) {
                    double mn_l = 0.0, pm_l = INFINITY;
#pragma unroll
                    for (int r = 0; r < RX; ++r)
                        if (ACT(r)) {
                            const double sd = sdr(r);
                            const double pr = (t[r] + alpha * (-rp[r] - gdu[r] - sd)) *
                                              (lam[r] + alpha * (rho[r] + th[r] * (gdu[r] + sd)));
                            mn_l += pr;
                            pm_l = fmin(pm_l, pr);
                        }
                    if (wave_min(pm_l) >= kNbhdGamma * (wave_sum(mn_l) / mact)) break;
                    alpha *= 0.8;
                }
#pragma unroll
                for (int r = 0; r < RX; ++r)
                    if (ACT(r)) {
                        const double sd = sdr(r);
                        t[r] = fma(alpha, -rp[r] - gdu[r] - sd, t[r]);
                        lam[r] = fma(alpha, rho[r] + th[r] * (gdu[r] + sd), lam[r]);
                    }
#pragma unroll
                for (int j = 0; j < NS; ++j) sg[j] = fma(alpha, dsg[j], sg[j]);
                STAMP(12);
            }
        }
        alpha_prev = alpha;
        for (int i = l; i < n; i += 64) U[i] = fma(alpha, dU[i], U[i]);
        for (int i = l; i < (N + 1) * NX; i += 64) X[i] = fma(alpha, dX[i], X[i]);
        wsync();
        STAMP(13);
    }
    if (it > c.max_iter) it = c.max_iter;
    if constexpr (W2) {  // wave 0 holds everything wave 1 has (bit-identical) and writes the outputs
        if (wvi != 0) return;
    }
    wsync();
    int status = CMPC_SOLVED;
    // a converged endpoint with a weakly active row (kPolishDegenerate) is polished as well
    bool degen = false;
    if (c.polish && P.ws && stop == kStopConverged) {
        double dg_l = 0.0;
#pragma unroll
        for (int r = 0; r < RX; ++r)
            if (ACT(r)) dg_l = fmax(dg_l, fmin(t[r], lam[r]));
        degen = wave_max(dg_l) > kPolishDegenerate;
    }
    // polish (CMPC_FLAG_POLISH): a stall or max-iteration exit at the rounding floor leaves its last iterate
    // too (a breakdown wrote it above)
    if (c.polish && P.ws &&
        ((stop != kStopConverged && stop != kStopBreakdown && stop != kStopNonFinite &&
          (best_m < 1e3 * c.tol || stop == kStopMaxIter)) ||
         degen))
        write_image();
    if (stop != kStopConverged) {
        if (best_it > 0) {  // restore the best iterate
            for (int i = l; i < NP; i += 64) U[i] = bU[i];
#pragma unroll
            for (int j = 0; j < NS; ++j) sg[j] = bsg[j];
            kkt = best_kkt;
        }
        status = stop_status(stop, best_m, c.tol);
    }
    wsync();

    // ---- output in the reference layout ----
    fwd(l, sx0, U, X);
    wsync();
    constexpr int NXE = NX + NS;
    const size_t nz = (size_t)NXE * (N + 1) + 2 * (size_t)n;
    double* z = P.z + (size_t)b * nz;
    for (int i = l; i < (N + 1) * NX; i += 64) {
        const int kk = i / NX, s = i - kk * NX;
        z[kk * NXE + s] = X[i];
    }
    if (l < NS) z[NX + l] = 0.0;
    if (lo && own) {
#pragma unroll
        for (int j = 0; j < NS; ++j) z[(k + 1) * NXE + NX + j] = sg[j];
    }
    for (int i = l; i < n; i += 64) {
        const int kk = i / NU, j = i - kk * NU;
        z[(size_t)(N + 1) * NXE + i] = U[i];
        z[(size_t)(N + 1) * NXE + n + i] = U[i] - (kk ? U[(kk - 1) * NU + j] : sup[j]);
    }
    if (l == 0) {
        if (P.kkt) P.kkt[b] = kkt;
        if (P.iters) P.iters[b] = it;
        if (P.status) P.status[b] = status;
        if (c.rescue && P.ws) {  // rescue image flag: 1 handed over (a breakdown), 2 polish (a
            // breakdown at the rounding floor with CMPC_FLAG_POLISH; slot 1 then holds its best merit)
            double* hd = P.ws + (size_t)b * c.ws_stride;
            const bool ho = hand_over(stop, best_m, c);
            // polished: a final exit short of tol (status 2 or -2; CMPC_UNSOLVED goes on to the Riccati rescue)
            const bool pol = !ho && c.polish &&
                             ((stop != kStopConverged && stop != kStopNonFinite &&
                               (best_m < 1e3 * c.tol || stop == kStopMaxIter)) ||
                              degen);
            hd[0] = ho ? 1.0 : (pol ? 2.0 : 0.0);
            if (pol) hd[1] = best_m;
        }
#ifndef CMPC_DBG_MERIT
        if (stamp) {
            unsigned long long* st = P.stamps + (size_t)b * kStampSlots;
            for (int i = 0; i < kStampSlots - 1; ++i) st[i] = tsum[i];
            st[kStampSlots - 1] = it;
        }
#endif
    }
#undef STAMP
#undef ACT
}

template <int T, int NX, int NU, int NB, bool LS, bool DS, bool L5, bool W2 = false>
static hipError_t launch3(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s) {
    const size_t lds = sizeof(double) * (size_t)lds3_layout<T, NX, NU, NB, LS, DS, W2>(c.N).total;
    hipError_t e = hipFuncSetAttribute((const void*)mpc_ipm3_kernel<T, NX, NU, NB, LS, DS, L5, W2>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((mpc_ipm3_kernel<T, NX, NU, NB, LS, DS, L5, W2>), dim3(batch), dim3(W2 ? 128 : 64), lds, s,
                       c, p);
    return hipGetLastError();
}

template <int NX, int NU, int NB, bool LS = false, bool DS = false, bool L5 = false, bool W2 = false>
static hipError_t launch3_t(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s) {
    switch (c.npad / 16) {
        case 1: return launch3<1, NX, NU, NB, LS, DS, L5, W2>(c, p, batch, s);
        case 2: return launch3<2, NX, NU, NB, LS, DS, L5, W2>(c, p, batch, s);
        case 3: return launch3<3, NX, NU, NB, LS, DS, L5, W2>(c, p, batch, s);
        default: return launch3<4, NX, NU, NB, LS, DS, L5, W2>(c, p, batch, s);
    }
}

// Q diagonal (the DS images keep only W_k's diagonal outside the (p_x, p_y) block)
static bool q_diagonal(const MpcConst& c) {
    for (int s = 0; s < c.nx; ++s)
        for (int u = 0; u < c.nx; ++u)
            if (s != u && c.Q[s * c.nx + u] != 0.0) return false;
    return true;
}

// This file is compiled once per instantiation set (CMPC_V3_SET = 1 .. 5; see the Makefile) so
// the instantiations build in parallel.  Set 1 also holds the dispatcher.
#ifndef CMPC_V3_SET
#define CMPC_V3_SET 1
#endif
#define CASE(NX_, NU_, NB_)                                 \
    if (c.nx == NX_ && c.nu == NU_ && nb == NB_) {          \
        *err = launch3_t<NX_, NU_, NB_>(c, p, batch, s);    \
        return true;                                        \
    }
// the reference's agent as built by lpv_build.hip (MpcConst::lpv; the fused DI rows never apply)
#define CASE_LS(NB_)                                                                              \
    if (c.lpv && c.nx == 9 && c.nu == 2 && nb == NB_ && !p.fuse.on) {                             \
        *err = c.lpv == 2 ? launch3_t<9, 2, NB_, true, false, true>(c, p, batch, s)               \
                          : launch3_t<9, 2, NB_, true>(c, p, batch, s);                           \
        return true;                                                                              \
    }
// the fused double-integrator round with a diagonal Q (DS images; the dense form gives the same bits);
// two wavefronts per agent where one per agent would leave SIMDs idle (mpc3_two_waves)
#define CASE_DS(NB_)                                                                   \
    if (p.fuse.on && c.nx == 4 && c.nu == 2 && nb == NB_ && q_diagonal(c)) {           \
        *err = mpc3_two_waves(c, batch) ? launch3_t<4, 2, NB_, false, true, false, true>(c, p, batch, s) \
                                        : launch3_t<4, 2, NB_, false, true>(c, p, batch, s); \
        return true;                                                                   \
    }
#if CMPC_V3_SET == 1
// Two-wave mode: opt-in (CMPC_FLAG_TWO_WAVES).  Measured at 512 agents on one MI355X (tools/w2_ab.py, 20 cfg3
// rounds, bit-identical results): 0.646 ms per launch against 0.640 ms with one wave.  Wave 0's K build
// shrinks 19.9k -> 15.8k clk per iteration and the predictor's right-hand side leaves its path, but the five
// barriers per iteration, the second wave's LDS traffic on the same CU and a few spilled registers take
// the gain back (tools/stamps.py --two-waves).
bool mpc3_two_waves(const MpcConst& c, int batch) {
    (void)batch;
    return c.waves == 2;
}

// host: the LDS image of the instantiation mpc3_try_launch picks (the same coverage rules)
size_t mpc3_lds_bytes(const MpcConst& c) {
    if (c.ns != 3 || c.N > 32 || c.mc < 4 || c.n > 64) return 0;
    for (int r = 0; r < c.mc; ++r)
        if (c.row_slack[r] != slk(r) || c.row_sign[r] != (int)sgn(r)) return 0;
    const int nb = c.mc - 4, T = c.npad / 16;
    auto lay = [&](auto nx_c, auto nu_c, auto nb_c, auto ls_c) -> size_t {
        constexpr int NX_ = decltype(nx_c)::value, NU_ = decltype(nu_c)::value, NB_ = decltype(nb_c)::value;
        constexpr bool LS_ = decltype(ls_c)::value;
        int o;
        switch (T) {
            case 1: o = lds3_layout<1, NX_, NU_, NB_, LS_>(c.N).total; break;
            case 2: o = lds3_layout<2, NX_, NU_, NB_, LS_>(c.N).total; break;
            case 3: o = lds3_layout<3, NX_, NU_, NB_, LS_>(c.N).total; break;
            default: o = lds3_layout<4, NX_, NU_, NB_, LS_>(c.N).total; break;
        }
        return sizeof(double) * (size_t)o;
    };
    using std::integral_constant;
#define LAY(NX_, NU_, NB_, LS_) \
    lay(integral_constant<int, NX_>{}, integral_constant<int, NU_>{}, integral_constant<int, NB_>{}, \
        integral_constant<bool, LS_>{})
    if (c.nx == 4 && c.nu == 2 && nb <= 2)
        return nb == 2 ? LAY(4, 2, 2, false) : (nb == 1 ? LAY(4, 2, 1, false) : LAY(4, 2, 0, false));
    if (c.nx == 9 && c.nu == 2 && nb <= 3) {
        if (c.lpv)
            return nb == 3 ? LAY(9, 2, 3, true)
                           : (nb == 2 ? LAY(9, 2, 2, true) : (nb == 1 ? LAY(9, 2, 1, true) : LAY(9, 2, 0, true)));
        return nb == 3 ? LAY(9, 2, 3, false)
                       : (nb == 2 ? LAY(9, 2, 2, false) : (nb == 1 ? LAY(9, 2, 1, false) : LAY(9, 2, 0, false)));
    }
    if (c.nx == 6 && c.nu == 3 && nb == 2) return LAY(6, 3, 2, false);
#undef LAY
    return 0;
}

bool mpc3_try_set2(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err, int nb);
bool mpc3_try_set5(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err, int nb);
bool mpc3_try_set3(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err, int nb);
bool mpc3_try_set4(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err, int nb);

// Returns true (and launches) when a v3 instantiation covers the problem: PlannerLPV row
// pattern with nb <= 2 neighbour rows (nb = 3 at nx = 9: the reference's 4-agent case),
// N <= 32, N*nu <= 64; (nx, nu) in {(4,2), (9,2), (6,3)}.
bool mpc3_try_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err) {
    if (c.ns != 3 || c.N > 32 || c.mc < 4 || c.n > 64) return false;
    for (int r = 0; r < c.mc; ++r)
        if (c.row_slack[r] != slk(r) || c.row_sign[r] != (int)sgn(r)) return false;
    const int nb = c.mc - 4;
    if (mpc3_try_set5(c, p, batch, s, err, nb)) return true;
    CASE(4, 2, 2)
    CASE(4, 2, 1)
    CASE(4, 2, 0)
    return mpc3_try_set2(c, p, batch, s, err, nb) || mpc3_try_set3(c, p, batch, s, err, nb) ||
           mpc3_try_set4(c, p, batch, s, err, nb);
}
#elif CMPC_V3_SET == 2
bool mpc3_try_set2(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err, int nb) {
    CASE_LS(2)
    CASE_LS(1)
    CASE_LS(0)
    CASE(9, 2, 2)
    CASE(9, 2, 1)
    CASE(9, 2, 0)
    return false;
}
#elif CMPC_V3_SET == 3
bool mpc3_try_set3(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err, int nb) {
    CASE(6, 3, 2)
    return false;
}
#elif CMPC_V3_SET == 5
bool mpc3_try_set5(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err, int nb) {
    CASE_DS(2)
    CASE_DS(1)
    CASE_DS(0)
    return false;
}
#else
bool mpc3_try_set4(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err, int nb) {
    CASE_LS(3)
    CASE(9, 2, 3)
    return false;
}
#endif
#undef CASE
#undef CASE_LS
#undef CASE_DS

}  // namespace cmpc
