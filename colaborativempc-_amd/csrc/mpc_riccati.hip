// Stage-wise (Riccati) interior-point solver for the structured LTV agent-QP: long horizons.
//
// The QP is the one PlannerLPV assembles (reference: planner/lib/plan_lib/distributedPlanner/
// LPV_Planner.py:279-475) and the reference ships it at N = 125 (planner/scripts/config_files/
// config_LPV.py:13-24): N*nu = 250 condensed inputs, whose dense Newton matrix (500 KB fp64)
// cannot live in LDS.  This kernel runs the SAME Mehrotra method as the condensed kernels
// (mpc_ipm.hip: same residuals, scaling, step control, safeguards and termination, internal.h),
// and only replaces the Newton solve K dU = rhs, K = sum_k Gamma_k' W_k Gamma_k + 2R + 2D'dR D
// + diag(input rows), by the equivalent linear-quadratic problem over the horizon
//
//   min  sum_{k=1..N} 1/2 dX_k' W_k dX_k + sum_k [1/2 dU_k'(2R + th_k) dU_k + 1/2 (dU_k - dU_{k-1})' 2dR (.)]
//        - rhs' dU     s.t.  dX_{k+1} = A_k dX_k + B_k dU_k,  dX_0 = 0,  dU_{-1} = 0,
//
// solved by a Riccati recursion on the augmented state y_k = [dX_k; dU_{k-1}] (na = nx + nu):
// O(N (nx+nu)^3) work and O(N nu (nx+nu)) storage instead of O((N nu)^3) and O((N nu)^2).
//
// One 64-lane wavefront (= one workgroup) per agent.  Everything the row loops touch lives in
// LDS; the per-stage operands of the recursions (A_k, B_k and the Riccati gains) stream from
// global memory through a double-buffered LDS stage image, fetched one stage ahead into
// registers so the load latency overlaps the current stage.  The Riccati gains, the stage
// weights W_k, the predictor direction and the best-iterate copy live in a per-agent global
// scratch (MpcPtrs::ws).
//
// Precision.  fp64, except near the solution of hard agents: once max th = lam/t exceeds
// kDdTh (rows pinned at t ~ 1e-13 with multipliers ~ 1e5, th -> 1e18..1e21 on the reference's
// N = 125 case) the double recursion loses the small directions of the cost-to-go to
// cancellation, and its Newton direction is off by O(1) where the condensed Cholesky is
// still usable.  Those iterations factor in double-double (dd.h) and refine the direction
// against the Newton residual evaluated in double-double (up to kRefineMax steps), which
// restores the exact direction (tools/ipm_lab.py, oracle/cmpc_oracle.c newton = 3).
#include <cmath>

#include "dd.h"
#include "internal.h"
#include "wave_ops.h"

namespace cmpc {

namespace {

constexpr int kMaxNa = CMPC_MAX_NX + CMPC_MAX_NU;
constexpr int kStageMax = CMPC_MAX_NX * CMPC_MAX_NX + CMPC_MAX_NX * CMPC_MAX_NU + CMPC_MAX_NU * kMaxNa +
                          CMPC_MAX_NU * CMPC_MAX_NU;
constexpr int kPerMax = (kStageMax + kWave - 1) / kWave;  // stage-image values per lane (largest dims)
constexpr int kPerSmall = 2;                               // ... when the stage image fits 128 values
constexpr int kDepth = 6;  // stage images in flight: a sweep step waits for a load issued 5 steps earlier
// Row loops over r = l, l + 64, ... < m run in chunks of kRowChunk rows per lane, every load of a chunk
// issued before any of its arithmetic (rows past m read row l, a valid index, and are not used): the GR
// instantiations keep the row vectors in global scratch, and a per-row loop with the loads behind its
// branches waited one memory latency per row.  The same operations in the same order per row.
constexpr int kRowChunk = 4;
constexpr double kDdTh = 1e10;   // max th above which an iteration runs in double-double ...
// ... once the solve has made no new best iterate for kDdStall iterations (or the fp64 factorisation
// broke down): on 2048 BASELINE cfg5 agents the double-double iterations drop 3136 -> 181 (25 % ->
// 1.5 % of all) with the same statuses to 3 agents and z to 8e-10, and every captured reference QP
// (N = 10 .. 125) takes the same iterations to the same statuses (oracle newton 3, tools/f32_lab.py)
constexpr int kDdStall = 2;
// Cfg::F32: an agent leaves fp32 for good after this many iterations without a new best iterate
// (or at an fp32 factorisation breakdown) — the lane kernel's kF32Stall (lane_body.h)
constexpr int kRicF32Stall = 2;
// rescue 3 (the fp32 path's last pass, mpc_launch): th capped here — on the one BASELINE cfg5 QP where every
// fp64 variant broke down at ~27 iterations with th ~ 1e25 (tools/f32_capture.py, round 6), the capped
// solve reaches KKT 6.9e-9 in 40 iterations without a breakdown (oracle RIC_F32 lab: 1e16 4.5e-8, 1e15
// 4.3e-7) — and it stops at the KKT bar (kkt < the requested tol: status 2 when the merit is not below it)
constexpr double kThCapLast = 1e17;
#ifndef RIC_P1
#define RIC_P1 1
#endif
#ifndef RIC_P4
#define RIC_P4 1
#endif
constexpr bool kP1 = RIC_P1, kP4 = RIC_P4;
constexpr int kRefineMax = 6;    // refinement steps of a double-double iteration's direction
// ... in a continued (rescue hand-over) solve: 2 — over the 22 lpv_lab rounds the continued
// agents end with the same statuses as with 6 (278 vs 279 at the rounding floor; oracle
// RIC_REFINE_WARM), and a step costs ~0.3 M clocks at N = 30
constexpr int kRefineMaxWarm = 2;
constexpr double kRefineTol = 1e-13;  // ... until |correction| <= kRefineTol |dU|: 1e-16 -> 1e-13 cut
                                      // the steps on the captured LPV QPs by 39% (752 -> 456) with the
                                      // same iterates to 1e-13 (tools/ipm_lab.py, oracle REF_TOL)

// The lane of this thread in its wavefront: the sweep helpers below are wave-level code, run by the one
// wave of mpc_riccati_kernel or by one of the waves of the latency mode (mpc_riccati_mw_kernel)
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (kWave - 1)); }

struct RLds {
    int t, lam, th, rp, rho, rt, w, GdU;  // per row
    int X, dX, yb, yb2, psi;              // per stage state (yb | yb2: the dd states of kres_dd)
    int U, dU, rd, gU, rh, cr;            // per condensed input
    int sig, dsig, Dsig, rsig;            // per stage slack
    int P, pv, sb, T, G, Hy, Kk, gv, xpp; // Riccati working set
    int Pd, PAd, PBd, Hd, Hyd, Kd, psid;  // double-double working set
    int stamps;                           // diagnostic clock sums (kStampSlots u64)
    int cst;                              // copy of MpcConst (weights read from LDS)
    int sb2, red, ring;                   // latency mode only: wave 1's stage slots, block reductions, gains ring
    int total;
};

struct Dims {
    int nx, nu, na, nc, sA, sB, sF, sAB, S;
    int SW;  // factor / residual stage image [A_k | B_k | W_{k-1}]
    int Sl;  // LDS slot stride max(S, SW)
};

// Compile-time problem configuration of a kernel instantiation: stage-image values per lane
// (KP) and, when nonzero, the state / input / rows-per-stage counts.  With the dimensions
// fixed the stage loops unroll and their independent loads issue together — the sweeps are
// serial chains of short steps on one wavefront, so latency is all that counts.
// GR: the six lane-owned row vectors (t, lam, w, rp, rho, GdU) live in the global scratch
// instead of LDS (r_rows_global): fewer LDS bytes per wave, more waves per CU.
template <int KP_, int NX_, int NU_, int MC_, bool GR_ = false, bool F32_ = false>
struct Cfg {
    static constexpr int KP = KP_, NX = NX_, NU = NU_, MC = MC_;
    static constexpr bool GR = GR_;
    // F32: BASELINE cfg5's fp32 path (CMPC_FLAG_FP32, MpcConst::f32): the factorisation, its gains
    // and both Newton recursions in fp32, iterates / residuals / rows / the direction's state
    // recursion in fp64; an agent continues in fp64 after an fp32 breakdown or kF32Stall
    // iterations without a new best iterate (the lane kernel's scheme, tools/f32_lab.py)
    static constexpr bool F32 = F32_;
    // values per lane of the [A | B | W] images of the factor and residual sweeps
    static constexpr int KPW = NX_ ? (2 * NX_ * NX_ + NX_ * NU_ + kWave - 1) / kWave
                                   : (2 * CMPC_MAX_NX * CMPC_MAX_NX + CMPC_MAX_NX * CMPC_MAX_NU + kWave - 1) / kWave;
};

__host__ __device__ inline Dims dims_of(const MpcConst& c) {
    Dims d;
    d.nx = c.nx;
    d.nu = c.nu;
    d.na = c.nx + c.nu;
    d.nc = c.nx + c.nu;
    d.sA = c.nx * c.nx;
    d.sB = c.nx * c.nu;
    d.sF = c.nu * d.na + c.nu * c.nu;  // gains K_k (nu x na) | Hinv_k (nu x nu)
    d.sAB = d.sA + d.sB;
    d.S = d.sAB + d.sF;
    d.SW = d.sAB + d.sA;
    d.Sl = d.S > d.SW ? d.S : d.SW;
    return d;
}

template <class G>
__device__ __forceinline__ Dims dims_t(const MpcConst& c) {
    Dims d;
    d.nx = G::NX ? G::NX : c.nx;
    d.nu = G::NU ? G::NU : c.nu;
    d.na = d.nx + d.nu;
    d.nc = d.na;
    d.sA = d.nx * d.nx;
    d.sB = d.nx * d.nu;
    d.sF = d.nu * d.na + d.nu * d.nu;
    d.sAB = d.sA + d.sB;
    d.S = d.sAB + d.sF;
    d.SW = d.sAB + d.sA;
    d.Sl = d.S > d.SW ? d.S : d.SW;
    return d;
}
template <class G>
__device__ __forceinline__ int mc_t(const MpcConst& c) { return G::MC ? G::MC : c.mc; }

__host__ __device__ inline RLds r_layout_ex(const MpcConst& c, bool gr) {
    const Dims d = dims_of(c);
    RLds L;
    int o = 0;
    auto take = [&](int cnt) {
        const int r = o;
        o += (cnt + 1) & ~1;
        return r;
    };
    const int m = c.m, n = c.n, N = c.N, nx = c.nx, ns = c.ns;
    const int mr = gr ? 0 : m;  // lane-owned rows: LDS, or (gr) the global scratch (r_glb)
    L.t = take(mr);
    L.lam = take(mr);
    L.th = take(m);
    L.rp = take(mr);
    L.rho = take(mr);
    L.rt = take(m);
    L.w = take(mr);
    L.GdU = take(mr);
    L.X = take((N + 1) * nx);
    L.dX = take((N + 1) * nx);
    L.yb = take((N + 1) * nx);
    L.yb2 = take((N + 1) * nx);  // must follow yb: [yb, yb2) holds (N+1)*nx dd values
    L.psi = take(2 * nx);
    L.U = take(n);
    L.dU = take(n);
    L.rd = take(n);
    L.gU = take(n);
    L.rh = take(n);
    L.cr = take(n);
    L.sig = take(N * ns);
    L.dsig = take(N * ns);
    L.Dsig = take(N * ns);
    L.rsig = take(N * ns);
    L.P = take(d.na * d.na);
    L.pv = take(2 * d.na);
    L.sb = take(2 * d.Sl);
    L.T = take(d.na * d.nc);
    L.G = take(d.nc * d.nc);
    L.Hy = take(c.nu * d.na);
    L.Kk = take(c.nu * d.na);
    L.gv = take(c.nu + nx);
    L.xpp = take(2 * nx);
    L.Pd = take(2 * d.na * d.na);
    L.PAd = take(2 * d.na * nx);
    L.PBd = take(2 * d.na * c.nu);
    L.Hd = take(2 * c.nu * c.nu);
    L.Hyd = take(2 * c.nu * d.na);
    L.Kd = take(2 * c.nu * d.na);
    L.psid = take(4 * nx);
    L.stamps = take(kStampSlots);
    // the weights' LDS copy, up to the last Q entry in use: at BASELINE cfg5 the whole struct made the
    // image 41.3 KB, over the 40 KB that lets four waves share a CU (three did: a quarter of the
    // SIMDs idle); without Q's unused tail it is 40.4 KB
    L.cst = take(mpc_const_used_doubles(c));
    L.sb2 = L.red = L.ring = 0;
    L.total = o;
    return L;
}

// Row vectors in the global scratch when that lifts the waves per CU (LDS-bound; the VGPR
// budget of these kernels, > 256 per lane, caps it at one wave per SIMD = 4 per CU) and the
// dimensions have a GR instantiation (BASELINE cfg5: nx 6, nu 3, 6 rows per stage; 67 KB ->
// 39 KB of LDS at N = 50, 2 -> 4 waves per CU).
__host__ __device__ inline bool r_rows_global(const MpcConst& c) {
    if (!(c.nx == 6 && c.nu == 3 && c.mc == 6)) return false;
    auto waves = [](int dbl) {
        const int w = (int)(kMaxLdsBytes / (sizeof(double) * (size_t)dbl));
        return w < 4 ? w : 4;
    };
    return waves(r_layout_ex(c, true).total) > waves(r_layout_ex(c, false).total);
}

__host__ __device__ inline RLds r_layout(const MpcConst& c) { return r_layout_ex(c, r_rows_global(c)); }

// per-agent global scratch (doubles): predictor direction (dt, dl), Riccati factors, stage
// weights W_k = 2Q + M_k of the state X_{k+1}, best iterate
struct RGlb {
    size_t hand, dta, dla, F, Wk, bU, bsig, t, lam, w, rp, rho, GdU, total;
};

__host__ __device__ inline RGlb r_glb(const MpcConst& c) {
    const Dims d = dims_of(c);
    RGlb g;
    size_t o = 0;
    auto take = [&](size_t cnt) {
        const size_t r = o;
        o += (cnt + 31) & ~size_t(31);  // 256-byte aligned regions
        return r;
    };
    g.hand = take(hand_doubles(c));  // first: the condensed kernels address it at ws + b * ws_stride
    g.dta = take(c.m);
    g.dla = take(c.m);
    g.F = take((size_t)c.N * d.sF);
    g.Wk = take((size_t)c.N * c.nx * c.nx);
    g.bU = take(c.n);
    g.bsig = take((size_t)c.N * c.ns);
    const size_t mr = r_rows_global(c) ? c.m : 0;  // see RLds / r_rows_global
    g.t = take(mr);
    g.lam = take(mr);
    g.w = take(mr);
    g.rp = take(mr);
    g.rho = take(mr);
    g.GdU = take(mr);
    g.total = o;
    return g;
}

// Stage image of stage k: [A_k (nx x nx) | B_k (nx x nu) | third segment] (the first `cnt`
// values; lane l holds values l, l + 64, ...).  The third segment is the gains K_k | Hinv_k of
// the solve sweeps (lag 0) or the weight W_{k-1} of the factor's P_k update (lag 1).
struct StageSrc {
    const double* A;
    const double* B;
    const double* F;
    int sA, sB, sF;
    int lag;
};

// Exactly KP loads per lane from clamped addresses, no branches: the compiler's wait counting
// then keeps the prefetched stages in flight (a data-dependent number of loads makes it drain
// the counter before every use)
template <int KP>
__device__ __forceinline__ void stage_fetch(const StageSrc& s, int k, int cnt, double (&r)[KP]) {
    const int l = lane_id();
    const int kf = k - s.lag > 0 ? k - s.lag : 0;
#pragma unroll
    for (int q = 0; q < KP; ++q) {
        int e = l + q * kWave;
        e = e < cnt ? e : cnt - 1;
        const double* p = (e < s.sA) ? s.A + (size_t)k * s.sA + e
                                     : ((e < s.sA + s.sB) ? s.B + (size_t)k * s.sB + (e - s.sA)
                                                          : s.F + (size_t)kf * s.sF + (e - s.sA - s.sB));
        r[q] = *p;
    }
}

template <int KP>
__device__ __forceinline__ void stage_put(double* buf, int cnt, const double (&r)[KP]) {
    const int l = lane_id();
#pragma unroll
    for (int q = 0; q < KP; ++q) {
        const int e = l + q * kWave;
        if (e < cnt) buf[e] = r[q];
    }
}

// Stage images of a sweep (forward: k = 0..N-1, backward: k = N-1..0) streamed through the
// 2-slot LDS buffer sb (stage k in slot k & 1), each fetched into registers kDepth steps
// before it is stored: the sweep is a serial chain of short steps, so one step cannot hide
// a global load.  Register sets are indexed statically (sweep() unrolls by kDepth).
template <int KP>
struct Pipe {
    double r[kDepth][KP];
    const StageSrc src;
    const int cnt, N, S;
    const bool back;
    double* const sb;
    // per lane and load q: the element's address at stage 0, its per-stage stride and whether it
    // is in the lagged third segment — fixed for the sweep, so a fetch is one multiply-add per
    // load (stage_fetch re-derived the segment and the 64-bit offsets at every step)
    const double* pb[KP];
    int ps[KP];
    bool pf[KP];
    __device__ Pipe(const StageSrc& s_, int cnt_, int N_, int S_, bool back_, double* sb_)
        : src(s_), cnt(cnt_), N(N_), S(S_), back(back_), sb(sb_) {
#pragma unroll
        for (int q = 0; q < KP; ++q) {
            int e = lane_id() + q * kWave;
            e = e < cnt ? e : cnt - 1;
            const bool ia = e < src.sA, ib = !ia && e < src.sA + src.sB;
            pb[q] = ia ? src.A + e : (ib ? src.B + (e - src.sA) : src.F + (e - src.sA - src.sB));
            ps[q] = ia ? src.sA : (ib ? src.sB : src.sF);
            pf[q] = !ia && !ib;
        }
    }
    // the loads of stage_fetch (same addresses)
    __device__ void fetch(int k, double (&r_)[KP]) const {
        const int kf = k - src.lag > 0 ? k - src.lag : 0;
#pragma unroll
        for (int q = 0; q < KP; ++q) r_[q] = pb[q][(pf[q] ? kf : k) * ps[q]];
    }
    __device__ int stg(int j) const { return back ? N - 1 - j : j; }
    // stage of step j, clamped into the horizon (steps past the end fetch a real stage, unused)
    __device__ int stc(int j) const { return stg(j < N ? j : N - 1); }
    // fetch the first kDepth stages, store the first; follow with wsync()
    __device__ void prime() {
        static_for<0, kDepth>([&](auto i) { fetch(stc(i), r[i]); });
        stage_put<KP>(sb + (stg(0) & 1) * S, cnt, r[0]);
        fetch(stc(kDepth), r[0]);
    }
    // after step j: store stage j+1 (register set I = (j+1) % kDepth) into the other slot and
    // refill the set with stage j+1+kDepth — unconditionally (see stage_fetch)
    template <int I>
    __device__ void advance(int j) {
        stage_put<KP>(sb + ((stg(j) + 1) & 1) * S, cnt, r[I]);
        fetch(stc(j + 1 + kDepth), r[I]);
    }
};

// body(k, img) for every stage of the sweep (img: the stage image of k), then bar()
// (the step count is padded to a multiple of kDepth; padding steps run no body, only the
// pipe's unconditional advance, so every path issues the same loads)
template <int KP, class Body>
__device__ __forceinline__ void sweep(Pipe<KP>& p, Body&& body) {
    for (int j0 = 0; j0 < p.N; j0 += kDepth)
        static_for<0, kDepth>([&](auto ii) {
            const int j = j0 + ii;
            const int k = p.stg(j);
            if (j < p.N) body(k, (const double*)(p.sb + (k & 1) * p.S));
            p.template advance<(ii + 1) % kDepth>(j);
            wsync();
        });
}

// 2R u_k + 2dR (du_k - du_{k+1}) for condensed variable index cidx (k*nu + i)
template <class G>
__device__ __forceinline__ double rdr_grad(const MpcConst& c, const double* U, const double* up, int cidx) {
    const int nu = G::NU ? G::NU : c.nu, k = cidx / nu, i = cidx - k * nu;
    double v = 0.0;
    for (int j = 0; j < nu; ++j) {
        const double uk = U[k * nu + j];
        const double duk = uk - (k ? U[(k - 1) * nu + j] : up[j]);
        const double dun = (k + 1 < c.N) ? U[(k + 1) * nu + j] - uk : 0.0;
        v += 2.0 * c.R[i * nu + j] * uk + 2.0 * c.dR[i * nu + j] * (duk - dun);
    }
    return v;
}

// Value of row r at (X, U, sig): state rows C_{k,r} . X_{k+1} (+ sign * sig), input rows +-U
template <class G>
__device__ __forceinline__ double row_value(const MpcConst& c, const double* __restrict__ C, int r, const double* X,
                                            const double* U, const double* sig) {
    const int nx = G::NX ? G::NX : c.nx, mc = mc_t<G>(c);
    if (r < c.ms) {
        const int k = r / mc, rr = r - k * mc;
        const double* cr = C + (size_t)r * nx;
        const double* xk = X + (k + 1) * nx;
        double v = 0.0;
        for (int s = 0; s < nx; ++s) v = fma(cr[s], xk[s], v);
        const int j = c.row_slack[rr];
        if (sig && j >= 0) v += c.row_sign[rr] * sig[k * c.ns + j];
        return v;
    }
    const int q = r - c.ms;
    const double u = U[q >> 1];
    return (q & 1) ? -u : u;
}

// Entry (s,u) of the per-stage constraint curvature M (stable group Schur form; see
// mpc_ipm.hip m_entry): no-slack rows th c c'; slack group j
// [q sum_r th_r c_r c_r' + sum_{r<r'} th_r th_r' (a_r - a_r')(a_r - a_r')'] / (q + sum th)
template <class G>
__device__ __forceinline__ double m_entry(const MpcConst& c, const double* __restrict__ Ck, const double* th_k,
                                          const double* Dsig_k, int s, int u) {
    const int nx = G::NX ? G::NX : c.nx, mc = mc_t<G>(c);
    double v = 0.0;
    for (int r = 0; r < mc; ++r) {
        const double* c1 = Ck + r * nx;
        const double t1 = th_k[r];
        const int j = c.row_slack[r];
        if (j < 0) {
            v = fma(t1 * c1[s], c1[u], v);
            continue;
        }
        const double inv = 1.0 / Dsig_k[j];
        const double q = 2.0 * c.Qs[j];
        double g = q * t1 * c1[s] * c1[u];
        const double s1 = c.row_sign[r];
        for (int r2 = r + 1; r2 < mc; ++r2) {
            if (c.row_slack[r2] != j) continue;
            const double* c2 = Ck + r2 * nx;
            const double s2 = c.row_sign[r2];
            g += t1 * th_k[r2] * (s1 * c1[s] - s2 * c2[s]) * (s1 * c1[u] - s2 * c2[u]);
        }
        v = fma(g, inv, v);
    }
    return v;
}

// X_0 = x0 (or 0), X_{k+1} = A_k X_k + B_k U_k  (stage images through sb)
template <class G>
__device__ __forceinline__ void fwd_sim(const MpcConst& c, const Dims& d, const StageSrc& src, double* sb,
                        const double* __restrict__ x0, const double* U, double* X) {
    const int l = lane_id(), nx = d.nx, nu = d.nu, N = c.N;
    Pipe<G::KP> pp(src, d.sAB, N, d.Sl, false, sb);
    pp.prime();
    if (l < nx) X[l] = x0 ? x0[l] : 0.0;
    wsync();
    sweep(pp, [&](int k, const double* Ak) {
        const double* Bk = Ak + d.sA;
        if constexpr (G::NX != 0) {  // fixed dimensions: every read issued before the chain (same sums)
            constexpr int NX = G::NX, NU = G::NU;
            const int r = l < NX ? l : NX - 1;
            double a[NX], x[NX], bb[NU], u[NU];
#pragma unroll
            for (int t = 0; t < NX; ++t) {
                a[t] = Ak[r * NX + t];
                x[t] = X[k * NX + t];
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                bb[i] = Bk[r * NU + i];
                u[i] = U[k * NU + i];
            }
            __builtin_amdgcn_sched_barrier(0);
            double v = 0.0;
#pragma unroll
            for (int t = 0; t < NX; ++t) v = fma(a[t], x[t], v);
#pragma unroll
            for (int i = 0; i < NU; ++i) v = fma(bb[i], u[i], v);
            if (l < NX) X[(k + 1) * NX + l] = v;
        } else if (l < nx) {
            double v = 0.0;
            for (int t = 0; t < nx; ++t) v = fma(Ak[l * nx + t], X[k * nx + t], v);
            for (int i = 0; i < nu; ++i) v = fma(Bk[l * nu + i], U[k * nu + i], v);
            X[(k + 1) * nx + l] = v;
        }
    });
}

// out_k = B_k' psi_{k+1}, psi_N = yb_N, psi_k = yb_k + A_k' psi_{k+1}   (out: n values)
template <class G>
__device__ __forceinline__ void adjoint(const MpcConst& c, const Dims& d, const StageSrc& src, double* sb, const double* yb,
                        double* out, double* psi2) {
    const int l = lane_id(), nx = d.nx, nu = d.nu, N = c.N;
    Pipe<G::KP> pp(src, d.sAB, N, d.Sl, true, sb);
    pp.prime();
    if (l < nx) psi2[l] = yb[N * nx + l];
    wsync();
    sweep(pp, [&](int k, const double* Ak) {
        const double* Bk = Ak + d.sA;
        const double* pa = psi2 + ((N - 1 - k) & 1) * nx;
        double* pb = psi2 + ((N - k) & 1) * nx;
        if constexpr (G::NX != 0) {
            // fixed dimensions: lanes < nu (B' psi) and 32..32+nx (psi) run one chain shape,
            // every read issued before it (same sums as below)
            constexpr int NX = G::NX, NU = G::NU;
            const bool bl = l < 32;
            const int t = bl ? (l < NU ? l : NU - 1) : (l - 32 < NX ? l - 32 : NX - 1);
            const double* col = bl ? Bk + t : Ak + t;
            const int ld = bl ? NU : NX;
            double cv[NX], pv[NX];
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2) {
                cv[s2] = col[s2 * ld];
                pv[s2] = pa[s2];
            }
            const double y0 = yb[k * NX + (bl ? 0 : t)];
            __builtin_amdgcn_sched_barrier(0);
            double v = bl ? 0.0 : y0;
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2) v = fma(cv[s2], pv[s2], v);
            if (l < NU) out[k * NU + l] = v;
            else if (k > 0 && l >= 32 && l < 32 + NX) pb[l - 32] = v;
        } else if (l < nu) {
            double v = 0.0;
            for (int s = 0; s < nx; ++s) v = fma(Bk[s * nu + l], pa[s], v);
            out[k * nu + l] = v;
        } else if (k > 0 && l >= 32 && l < 32 + nx) {
            const int t = l - 32;
            double v = yb[k * nx + t];
            for (int s = 0; s < nx; ++s) v = fma(Ak[s * nx + t], pa[s], v);
            pb[t] = v;
        }
    });
}

// Two independent adjoint recursions in one backward sweep (fixed dimensions): out1 / out2 from
// yb1 / yb2, the arithmetic of two adjoint() calls (bit-identical), one stage advance per stage
// and two chains in flight.  Lanes: 0..nu-1 B'psi1, 16..16+nu-1 B'psi2, 32..32+nx-1 psi1,
// 48..48+nx-1 psi2.  psi4: 4 nx doubles (two ping-pong pairs).
template <class G>
__device__ __forceinline__ void adjoint2(const MpcConst& c, const Dims& d, const StageSrc& src, double* sb,
                                         const double* yb1, double* out1, const double* yb2, double* out2,
                                         double* psi4, volatile double* prog = nullptr) {
    // prog (latency mode): stages done, after the stage's outputs
    constexpr int NX = G::NX, NU = G::NU;
    static_assert(NX != 0 && NX <= 16 && NU <= 16, "fixed dimensions");
    const int l = lane_id(), N = c.N;
    Pipe<G::KP> pp(src, d.sAB, N, d.Sl, true, sb);
    pp.prime();
    const bool second = (l & 16) != 0;  // lanes 16..31, 48..63
    const double* yb = second ? yb2 : yb1;
    double* psi = psi4 + (second ? 2 * NX : 0);
    if ((l & 15) < NX && l >= 32) psi[l & 15] = yb[N * NX + (l & 15)];
    wsync();
    const bool bl = l < 32;
    const int t = bl ? ((l & 15) < NU ? (l & 15) : NU - 1) : ((l & 15) < NX ? (l & 15) : NX - 1);
    double* out = second ? out2 : out1;
    sweep(pp, [&](int k, const double* Ak) {
        const double* Bk = Ak + NX * NX;
        const double* pa = psi + ((N - 1 - k) & 1) * NX;
        double* pb = psi + ((N - k) & 1) * NX;
        const double* col = bl ? Bk + t : Ak + t;
        const int ld = bl ? NU : NX;
        double cv[NX], pv[NX];
#pragma unroll
        for (int s2 = 0; s2 < NX; ++s2) {
            cv[s2] = col[s2 * ld];
            pv[s2] = pa[s2];
        }
        const double y0 = yb[k * NX + (bl ? 0 : t)];
        __builtin_amdgcn_sched_barrier(0);
        double v = bl ? 0.0 : y0;
#pragma unroll
        for (int s2 = 0; s2 < NX; ++s2) v = fma(cv[s2], pv[s2], v);
        if (bl && (l & 15) < NU) out[k * NU + (l & 15)] = v;
        else if (!bl && k > 0 && (l & 15) < NX) pb[l & 15] = v;
        if (prog) {
            wsync();
            if (l == 0) *prog = (double)(N - k);
        }
    });
}

// W_k = 2Q + M_k of the state X_{k+1} for every block k (global scratch, one pass of all lanes)
template <class G>
__device__ __forceinline__ void stage_weights(const MpcConst& c, const RLds& L, const double* sm,
                                              const double* __restrict__ C, double* __restrict__ Wg,
                                              int e0 = -1, int stride = kWave) {
    if (e0 < 0) e0 = lane_id();  // (the latency mode spreads the items over its four waves)
    const int nx = G::NX ? G::NX : c.nx, nx2 = nx * nx, mc = mc_t<G>(c), ns = c.ns;
    const double* th = sm + L.th;
    const double* Dsig = sm + L.Dsig;
    if constexpr (G::NX != 0 && G::MC != 0) {
        // one lane per row (k, i) of W_k: the stage's constraint rows are read once per row
        // and every load of an item issues together (same grouping as m_entry)
        constexpr int NX = G::NX, MC = G::MC;
        for (int e = e0; e < c.N * NX; e += stride) {
            const int k = e / NX, i = e - k * NX;
            const double* Ck = C + (size_t)k * MC * NX;
            const double* thk = th + k * MC;
            double w[NX];
#pragma unroll
            for (int u = 0; u < NX; ++u) w[u] = 0.0;
            // rows streamed one (or one pair) at a time: few registers live across the loop;
            // the sums round exactly like m_entry's (2Q added last)
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                const double* c1 = Ck + r * NX;
                const double t1 = thk[r], ci1 = c1[i];
                const int j = c.row_slack[r];
                if (j < 0) {
#pragma unroll
                    for (int u = 0; u < NX; ++u) w[u] = fma(t1 * ci1, c1[u], w[u]);
                    continue;
                }
                const double inv = 1.0 / Dsig[k * ns + j];
                const double q = 2.0 * c.Qs[j];
                const double s1 = c.row_sign[r];
                double g[NX];
#pragma unroll
                for (int u = 0; u < NX; ++u) g[u] = q * t1 * ci1 * c1[u];
#pragma unroll
                for (int r2 = r + 1; r2 < MC; ++r2) {
                    if (c.row_slack[r2] != j) continue;
                    const double* c2 = Ck + r2 * NX;
                    const double s2 = c.row_sign[r2];
                    const double a2 = t1 * thk[r2] * (s1 * ci1 - s2 * c2[i]);
#pragma unroll
                    for (int u = 0; u < NX; ++u) g[u] += a2 * (s1 * c1[u] - s2 * c2[u]);
                }
#pragma unroll
                for (int u = 0; u < NX; ++u) w[u] = fma(g[u], inv, w[u]);
            }
#pragma unroll
            for (int u = 0; u < NX; ++u) Wg[(size_t)k * NX * NX + i * NX + u] = 2.0 * c.Q[i * NX + u] + w[u];
        }
    } else {
        for (int e = e0; e < c.N * nx2; e += stride) {
            const int k = e / nx2, q = e - k * nx2, i = q / nx, j = q - i * nx;
            Wg[e] = 2.0 * c.Q[q] + m_entry<G>(c, C + (size_t)k * mc * nx, th + k * mc, Dsig + k * ns, i, j);
        }
    }
}

// Lower-triangle entry t of an n x n matrix -> (i, j), j <= i (row-major over the triangle).
__device__ __forceinline__ void tri_ij(int t, int n, int& i, int& j) {
    i = 0;
    for (int r = 1; r < n; ++r) i += (r * (r + 1) / 2 <= t) ? 1 : 0;
    j = t - i * (i + 1) / 2;
}

// 1/sqrt and 1/x in the factor's precision (hardware estimate + Newton steps to full precision)
__device__ __forceinline__ double rsqrt_r(double x) { return rsqrt_d(x); }
__device__ __forceinline__ double rcp_r(double x) { return rcp_d(x); }
__device__ __forceinline__ float rsqrt_r(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    return y * fmaf(-0.5f * x, y * y, 1.5f);
}
__device__ __forceinline__ float rcp_r(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    return fmaf(r, fmaf(-x, r, 1.0f), r);
}

// One stage of the fp64 factor sweep for compile-time dimensions (G::NX != 0): the arithmetic of
// the generic stage below, every sum in the same order (the gains and P are bit-identical), in
// three phases instead of four, each issuing all of its LDS reads before its first FMA.
//   1. T = P[:, :nx] [A_k | B_k]          (the old P_uu block is read here too)
//   2. G = [A_k | B_k]' T[:nx, :]         (lower triangle)
//   3. every lane: Hvv, its Cholesky factor and inverse; the lane's gain entries (into F);
//      its entries of P_k = blkdiag(W_k + A'Pxx A, 2dR) + Hvy' K_k, the Hvy / K columns they
//      need formed from G and T in registers — no hand-off through LDS between K and P_k.
// The generic stage let the compiler interleave its reads with the FMA chains that consume
// them (one LDS latency per two products) and ran the A / B column cases of T as divergent
// branches: ~2 k clocks per phase (tools/ric_stamps.py, lab build CMPC_RIC_SUBSTAMP).
// R = float: the same stage in fp32 (Cfg::F32; operands rounded to float on load, results
// stored widened).
template <class G, class R = double>
__device__ __forceinline__ bool factor_stage_fixed(const MpcConst& c, int k, const double* Ak, double* P, double* T,
                                                   double* Gm, const double* th, double* __restrict__ Fk, int ms,
                                                   unsigned long long* sub, double* Fr = nullptr) {
    constexpr int NX = G::NX, NU = G::NU, NA = NX + NU, NC = NA;
    constexpr int NE = NA * NC, RT = (NE + kWave - 1) / kWave;           // T entries, rounds
    constexpr int NT = NC * (NC + 1) / 2, RG = (NT + kWave - 1) / kWave; // G lower entries
    constexpr int NP = NA * (NA + 1) / 2, RP = (NP + kWave - 1) / kWave; // P lower entries
    const int l = lane_id();
    const double* Bk = Ak + NX * NX;
    const double* Wk = Ak + NX * NX + NX * NU;
#ifdef CMPC_RIC_SUBSTAMP
    unsigned long long s_a = sub ? clock64_() : 0;
#define FSTAMP(slot)                                    \
    if (sub) {                                          \
        const unsigned long long s_b = clock64_();      \
        if (l == 0) sub[slot] += s_b - s_a;             \
        s_a = s_b;                                      \
    }
#else
#define FSTAMP(slot)
#endif
    // ---- phase 1: T ----
    {
        R pr[RT][NX], cv[RT][NX];
        R pu[NU][NU];
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            int e = l + q * kWave;
            e = e < NE ? e : NE - 1;
            const int i = e / NC, j = e - i * NC;
            const double* col = (j < NX) ? Ak + j : Bk + (j - NX);
            const int ld = (j < NX) ? NX : NU;
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                pr[q][s] = (R)P[i * NA + s];
                cv[q][s] = (R)col[s * ld];
            }
        }
#pragma unroll
        for (int a = 0; a < NU; ++a)
#pragma unroll
            for (int b = 0; b <= a; ++b) pu[a][b] = (R)P[(NX + a) * NA + NX + b];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            R v = R(0);
#pragma unroll
            for (int s = 0; s < NX; ++s) v = fma(pr[q][s], cv[q][s], v);
            if (l + q * kWave < NE) T[l + q * kWave] = v;
        }
        wsync();  // (pu: P_uu of P_{k+1}, held in registers; phase 3 overwrites P)
        FSTAMP(9)
        // ---- phase 2: G (lower triangle) ----
        R tr[RG][NX], cg[RG][NX];
        int ge[RG];
#pragma unroll
        for (int q = 0; q < RG; ++q) {
            int t = l + q * kWave;
            t = t < NT ? t : NT - 1;
            int i, j;
            tri_ij(t, NC, i, j);
            ge[q] = i * NC + j;
            const double* ci = (i < NX) ? Ak + i : Bk + (i - NX);
            const int ldi = (i < NX) ? NX : NU;
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                cg[q][s] = (R)ci[s * ldi];
                tr[q][s] = (R)T[s * NC + j];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < RG; ++q) {
            R v = R(0);
#pragma unroll
            for (int s = 0; s < NX; ++s) v = fma(cg[q][s], tr[q][s], v);
            if (l + q * kWave < NT) Gm[ge[q]] = v;
        }
        wsync();
        FSTAMP(10)
        // ---- phase 3 ----
        // reads: Hvv's G / T entries, the lane's gain column, its P entries' columns
        // (the weights live in LDS too (c): their reads belong before the barrier as well)
        R hg[NU][NU], ht1[NU][NU], ht2[NU][NU], thu[NU][2], r2[NU][NU], dr2[NU][NU];
#pragma unroll
        for (int a = 0; a < NU; ++a) {
#pragma unroll
            for (int b = 0; b <= a; ++b) {
                hg[a][b] = (R)Gm[(NX + a) * NC + NX + b];
                ht1[a][b] = (R)T[(NX + a) * NC + NX + b];
                ht2[a][b] = (R)T[(NX + b) * NC + NX + a];
                r2[a][b] = (R)c.R[a * NU + b];
                dr2[a][b] = (R)c.dR[a * NU + b];
            }
            const int rr = ms + 2 * (k * NU + a);
            thu[a][0] = (R)th[rr];
            thu[a][1] = (R)th[rr + 1];
        }
        // gain entry e = l (a = e / NA, column j): hv(b, j) = G[nx+b][j] + T[nx+b][j] (j < nx)
        constexpr int NK = NU * NA;
        const int ek = l < NK ? l : NK - 1;
        const int ka = ek / NA, kj = ek - ka * NA;
        R kg[NU], kt[NU], kd[NU];
#pragma unroll
        for (int b = 0; b < NU; ++b) {
            const int jj = kj < NX ? kj : 0;
            kg[b] = (R)Gm[(NX + b) * NC + jj];
            kt[b] = (R)T[(NX + b) * NC + jj];
            kd[b] = (R)c.dR[b * NU + (kj < NX ? 0 : kj - NX)];
        }
        // P entries (i, j), j <= i: W + G[i][j] and the columns i, j of Hvy
        R pw[RP], pg[RP], pd[RP], ci_g[RP][NU], ci_t[RP][NU], cj_g[RP][NU], cj_t[RP][NU], ci_d[RP][NU],
            cj_d[RP][NU];
        int pi_[RP], pj_[RP];
#pragma unroll
        for (int q = 0; q < RP; ++q) {
            int t = l + q * kWave;
            t = t < NP ? t : NP - 1;
            int i, j;
            tri_ij(t, NA, i, j);
            pi_[q] = i;
            pj_[q] = j;
            const int ix = i < NX ? i : 0, jx = j < NX ? j : 0;
            const int iu = i < NX ? 0 : i - NX, ju = j < NX ? 0 : j - NX;
            pw[q] = (R)Wk[ix * NX + jx];
            pg[q] = (R)Gm[ix * NC + jx];
            pd[q] = (R)c.dR[iu * NU + ju];
#pragma unroll
            for (int b = 0; b < NU; ++b) {
                ci_g[q][b] = (R)Gm[(NX + b) * NC + ix];
                ci_t[q][b] = (R)T[(NX + b) * NC + ix];
                cj_g[q][b] = (R)Gm[(NX + b) * NC + jx];
                cj_t[q][b] = (R)T[(NX + b) * NC + jx];
                ci_d[q][b] = (R)c.dR[b * NU + iu];
                cj_d[q][b] = (R)c.dR[b * NU + ju];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // Hvv and its Cholesky factor / inverse (as the generic stage)
        R Lf[CMPC_MAX_NU][CMPC_MAX_NU], Hi[CMPC_MAX_NU][CMPC_MAX_NU];
        bool ok = true;
#pragma unroll
        for (int a = 0; a < CMPC_MAX_NU; ++a)
#pragma unroll
            for (int b = 0; b < CMPC_MAX_NU; ++b) {
                R v = R(0);
                if (a < NU && b <= a) {
                    v = R(2.0) * r2[a][b] + R(2.0) * dr2[a][b] + hg[a][b] + ht1[a][b] + ht2[a][b] + pu[a][b];
                    if (a == b) v += thu[a][0] + thu[a][1];
                }
                Lf[a][b] = v;
            }
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            R dj = Lf[j][j];
#pragma unroll
            for (int p = 0; p < j; ++p) dj = fma(-Lf[j][p], Lf[j][p], dj);
            ok = ok && (dj > R(0));
            const R rs = rsqrt_r(dj > R(0) ? dj : R(1));
            Lf[j][j] = dj * rs;
#pragma unroll
            for (int i = j + 1; i < NU; ++i) {
                R v = Lf[i][j];
#pragma unroll
                for (int p = 0; p < j; ++p) v = fma(-Lf[i][p], Lf[j][p], v);
                Lf[i][j] = v * rs;
            }
        }
        R Li[CMPC_MAX_NU][CMPC_MAX_NU];
#pragma unroll
        for (int i = 0; i < CMPC_MAX_NU; ++i)
#pragma unroll
            for (int j = 0; j < CMPC_MAX_NU; ++j) Li[i][j] = R(0);
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const R di = rcp_r(Lf[i][i]);
            Li[i][i] = di;
#pragma unroll
            for (int j = 0; j < i; ++j) {
                R v = R(0);
#pragma unroll
                for (int p = j; p < i; ++p) v = fma(Lf[i][p], Li[p][j], v);
                Li[i][j] = -v * di;
            }
        }
#pragma unroll
        for (int a = 0; a < CMPC_MAX_NU; ++a)
#pragma unroll
            for (int b = 0; b < CMPC_MAX_NU; ++b) {
                R v = R(0);
#pragma unroll
                for (int p = 0; p < CMPC_MAX_NU; ++p) v = fma(Li[p][a], Li[p][b], v);
                Hi[a][b] = v;
            }
        // hv(b, col) and K(a, col) = sum_b -Hinv[a][b] hv(b, col), in the generic stage's order
        auto hv = [&](int col, R g, R t, R dr) { return (col < NX) ? g + t : R(-2.0) * dr; };
        // the lane's gain entry and Hinv entry
        {
            R kv = R(0);
#pragma unroll
            for (int b = 0; b < NU; ++b) {
                R hab = R(0);
#pragma unroll
                for (int a2 = 0; a2 < NU; ++a2)
                    if (a2 == ka) hab = Hi[a2][b];
                kv = fma(-hab, hv(kj, kg[b], kt[b], kd[b]), kv);
            }
            if (l < NK) {
                Fk[l] = kv;
                if (Fr) Fr[l] = kv;  // (latency mode: the gains to wave 2 through an LDS ring)
            }
            if (l < NU * NU) {
                const int a = l / NU, b = l - a * NU;
                R v = R(0);
#pragma unroll
                for (int a2 = 0; a2 < NU; ++a2)
#pragma unroll
                    for (int b2 = 0; b2 < NU; ++b2)
                        if (a2 == a && b2 == b) v = Hi[a2][b2];
                Fk[NK + l] = v;
                if (Fr) Fr[NK + l] = v;
            }
        }
        // P_k entries (k > 0)
        if (k > 0) {
#pragma unroll
            for (int q = 0; q < RP; ++q) {
                const int i = pi_[q], j = pj_[q];
                R v = (i < NX) ? pw[q] + pg[q] : ((j >= NX) ? R(2.0) * pd[q] : R(0));
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    R kv = R(0);
#pragma unroll
                    for (int b = 0; b < NU; ++b) kv = fma(-Hi[a][b], hv(j, cj_g[q][b], cj_t[q][b], cj_d[q][b]), kv);
                    v = fma(hv(i, ci_g[q][a], ci_t[q][a], ci_d[q][a]), kv, v);
                }
                if (l + q * kWave < NP) {
                    P[i * NA + j] = v;
                    P[j * NA + i] = v;
                }
            }
        }
        FSTAMP(11)
#undef FSTAMP
        return ok;
    }
}

// Riccati factorisation of the Newton system at the current (th, Dsig), with the stage weights
// Wg of stage_weights: writes the gains K_k = -Hvv^-1 Hvy and Hinv_k = Hvv^-1 of every stage
// into F.  Returns false on a non-positive pivot (wave-uniform).  R = float: the fp32 stages of
// Cfg::F32 (fixed dimensions only).
// Latency mode: wait (bounded) until *v >= want; false on a timeout (the caller marks the agent unsolved
// rather than hang the workgroup)
// (LDS: a wave's LDS operations execute in order and the waiting wave's later reads issue after the flag's,
// so the compiler fence of wsync() on both sides is the whole protocol)
__device__ __forceinline__ bool spin_until(const volatile double* v, double want) {
    bool ok = false;
    for (int i = 0; i < (1 << 18) && !ok; ++i) {
        ok = *v >= want;
        if (!ok) __builtin_amdgcn_s_sleep(1);
    }
    wsync();
    return ok;
}
constexpr int kRing = 4;  // latency mode: stages of gains in flight between waves 1 and 2

template <class G, class R = double>
__device__ __forceinline__ bool riccati_factor(const MpcConst& c, const Dims& d, const RLds& L, double* sm,
                               const double* __restrict__ A, const double* __restrict__ B,
                               const double* __restrict__ Wg, double* __restrict__ F,
                               unsigned long long* sub = nullptr, double* ring = nullptr,
                               volatile double* prog = nullptr, const volatile double* cons = nullptr,
                               volatile double* err = nullptr) {
    // ring / prog / cons (latency mode, fixed dimensions): stage k's gains also go to LDS ring slot k % kRing,
    // the slot written only once the consumer (wave 2) has passed stage k + kRing; prog = stages done
    const int l = lane_id(), nx = d.nx, nu = d.nu, na = d.na, nc = d.nc, N = c.N;
    const int ms = c.ms;  // (a register: see riccati_solve)
#ifdef CMPC_RIC_SUBSTAMP  // lab build (tools/ric_stamps.py --sub): per-phase clocks of the fp64 factor sweep
    unsigned long long s_a = sub ? clock64_() : 0;
#define SUBSTAMP(slot)                                  \
    if (sub) {                                          \
        const unsigned long long s_b = clock64_();      \
        if (slot >= 0 && l == 0) sub[slot] += s_b - s_a; \
        s_a = s_b;                                      \
    }
#else
#define SUBSTAMP(slot)
#endif
    double* P = sm + L.P;
    double* T = sm + L.T;
    double* Gm = sm + L.G;
    double* Hy = sm + L.Hy;
    double* Kk = sm + L.Kk;
    double* sb = sm + L.sb;
    const double* th = sm + L.th;
    const StageSrc src{A, B, Wg, d.sA, d.sB, d.sA, 1};  // [A_k | B_k | W_{k-1}]
    Pipe<G::KPW> pp(src, d.SW, N, d.Sl, true, sb);
    pp.prime();
    // P_N = blkdiag(W_N, 0),  W_N = 2Q + M_N (stage rows of X_N)
    for (int e = l; e < na * na; e += kWave) {
        const int i = e / na, j = e - i * na;
        P[e] = (i < nx && j < nx) ? Wg[(size_t)(N - 1) * nx * nx + i * nx + j] : 0.0;
    }
    wsync();
    bool ok = true;
    sweep(pp, [&](int k, const double* Ak) {
      if constexpr (G::NX != 0) {
        double* Fr = nullptr;
        if (ring) {
            if (!spin_until(cons, (double)(N - k - kRing)) && l == 0) *err = 1.0;
            Fr = ring + (k % kRing) * d.sF;
        }
        ok = factor_stage_fixed<G, R>(c, k, Ak, P, T, Gm, th, F + (size_t)k * d.sF, ms, sub, Fr) && ok;
        if (prog) {
            wsync();
            if (l == 0) *prog = (double)(N - k);
        }
      } else {
        const double* Bk = Ak + d.sA;
        SUBSTAMP(-1)  // slots 9-11: T, G, Hvv..K; the rest of the factor (P update, stage advance) is slot 2 minus them
        // T = P[:, :nx] [A_k | B_k]   (na x nc)
        for (int e = l; e < na * nc; e += kWave) {
            const int i = e / nc, j = e - i * nc;
            double v = 0.0;
            if (j < nx)
                for (int s = 0; s < nx; ++s) v = fma(P[i * na + s], Ak[s * nx + j], v);
            else
                for (int s = 0; s < nx; ++s) v = fma(P[i * na + s], Bk[s * nu + (j - nx)], v);
            T[e] = v;
        }
        wsync();
        SUBSTAMP(9)
        // G = [A_k | B_k]' T[:nx, :]   (nc x nc, lower triangle)
        for (int e = l; e < nc * nc; e += kWave) {
            const int i = e / nc, j = e - i * nc;
            if (j > i) continue;
            const double* ci = (i < nx) ? Ak + i : Bk + (i - nx);
            const int ldi = (i < nx) ? nx : nu;
            double v = 0.0;
            for (int s = 0; s < nx; ++s) v = fma(ci[s * ldi], T[s * nc + j], v);
            Gm[e] = v;
        }
        wsync();
        SUBSTAMP(10)
        // Hvv = 2R + 2dR + diag(th_u) + B'Pxx B + Pux B + B'Pxu + Puu  (every lane, nu <= 4),
        // its Cholesky factor and inverse in registers
        double Lf[CMPC_MAX_NU][CMPC_MAX_NU], Hi[CMPC_MAX_NU][CMPC_MAX_NU];
#pragma unroll
        for (int a = 0; a < CMPC_MAX_NU; ++a)
#pragma unroll
            for (int b = 0; b < CMPC_MAX_NU; ++b) {
                double v = 0.0;
                if (a < nu && b <= a) {
                    v = 2.0 * c.R[a * nu + b] + 2.0 * c.dR[a * nu + b] + Gm[(nx + a) * nc + nx + b] +
                        T[(nx + a) * nc + nx + b] + T[(nx + b) * nc + nx + a] + P[(nx + a) * na + nx + b];
                    if (a == b) {
                        const int rr = c.ms + 2 * (k * nu + a);
                        v += th[rr] + th[rr + 1];
                    }
                }
                Lf[a][b] = v;
            }
#pragma unroll
        for (int j = 0; j < CMPC_MAX_NU; ++j) {
            if (j < nu) {
                double dj = Lf[j][j];
#pragma unroll
                for (int p = 0; p < j; ++p) dj = fma(-Lf[j][p], Lf[j][p], dj);
                ok = ok && (dj > 0.0);
                const double rs = rsqrt_d(dj > 0.0 ? dj : 1.0);
                Lf[j][j] = dj * rs;
#pragma unroll
                for (int i = j + 1; i < CMPC_MAX_NU; ++i) {
                    if (i < nu) {
                        double v = Lf[i][j];
#pragma unroll
                        for (int p = 0; p < j; ++p) v = fma(-Lf[i][p], Lf[j][p], v);
                        Lf[i][j] = v * rs;
                    }
                }
            }
        }
        // Li = L^-1 (lower), Hinv = Li' Li
        double Li[CMPC_MAX_NU][CMPC_MAX_NU];
#pragma unroll
        for (int i = 0; i < CMPC_MAX_NU; ++i)
#pragma unroll
            for (int j = 0; j < CMPC_MAX_NU; ++j) Li[i][j] = 0.0;
#pragma unroll
        for (int i = 0; i < CMPC_MAX_NU; ++i) {
            if (i < nu) {
                const double di = rcp_d(Lf[i][i]);
                Li[i][i] = di;
#pragma unroll
                for (int j = 0; j < i; ++j) {
                    double v = 0.0;
#pragma unroll
                    for (int p = j; p < i; ++p) v = fma(Lf[i][p], Li[p][j], v);
                    Li[i][j] = -v * di;
                }
            }
        }
#pragma unroll
        for (int a = 0; a < CMPC_MAX_NU; ++a)
#pragma unroll
            for (int b = 0; b < CMPC_MAX_NU; ++b) {
                double v = 0.0;
#pragma unroll
                for (int p = 0; p < CMPC_MAX_NU; ++p) v = fma(Li[p][a], Li[p][b], v);
                Hi[a][b] = v;
            }
        // Hvy = [B'Pxx A + Pux A | -2dR] (nu x na);  K_k = -Hinv Hvy
        double* Fk = F + (size_t)k * d.sF;
        for (int e = l; e < nu * na; e += kWave) {
            const int a = e / na, j = e - a * na;
            double kv = 0.0, ha = 0.0;
#pragma unroll
            for (int b = 0; b < CMPC_MAX_NU; ++b) {
                if (b < nu) {
                    const double hv = (j < nx) ? Gm[(nx + b) * nc + j] + T[(nx + b) * nc + j] : -2.0 * c.dR[b * nu + (j - nx)];
                    double hab = 0.0;
#pragma unroll
                    for (int a2 = 0; a2 < CMPC_MAX_NU; ++a2)
                        if (a2 == a) hab = Hi[a2][b];
                    kv = fma(-hab, hv, kv);
                    if (b == a) ha = hv;
                }
            }
            Kk[e] = kv;
            Hy[e] = ha;
            Fk[e] = kv;
        }
        if (l < nu * nu) {
            const int a = l / nu, b = l - a * nu;
            double v = 0.0;
#pragma unroll
            for (int a2 = 0; a2 < CMPC_MAX_NU; ++a2)
#pragma unroll
                for (int b2 = 0; b2 < CMPC_MAX_NU; ++b2)
                    if (a2 == a && b2 == b) v = Hi[a2][b2];
            Fk[nu * na + l] = v;
        }
        wsync();
        SUBSTAMP(11)
        // P_k = blkdiag(W_k + A'Pxx A, 2dR) + Hvy' K_k   (symmetric: lower triangle mirrored)
        for (int e = l; e < na * na && k > 0; e += kWave) {
            const int i = e / na, j = e - i * na;
            if (j > i) continue;
            double v = (i < nx) ? Ak[d.sAB + i * nx + j] + Gm[i * nc + j]
                                : ((j >= nx) ? 2.0 * c.dR[(i - nx) * nu + (j - nx)] : 0.0);
            for (int a = 0; a < nu; ++a) v = fma(Hy[a * na + i], Kk[a * na + j], v);
            P[i * na + j] = v;
            P[j * na + i] = v;
        }
      }
    });
#undef SUBSTAMP
    return ok;
}

// riccati_factor in double-double (standard form: P_k = blkdiag(W_k + A'Pxx A, 2dR) + Hvy'K_k),
// for the iterations whose th span defeats fp64 (kDdTh).  The gains are rounded to double
// into F; the refinement against the double-double residual (kres_dd) absorbs that rounding.
template <class G>
__device__ __forceinline__ bool riccati_factor_dd(const MpcConst& c, const Dims& d, const RLds& L, double* sm,
                                  const double* __restrict__ A, const double* __restrict__ B,
                                  const double* __restrict__ Wg, double* __restrict__ F) {
    const int l = lane_id(), nx = d.nx, nu = d.nu, na = d.na, N = c.N;
    double* P = sm + L.Pd;
    double* PA = sm + L.PAd;
    double* PB = sm + L.PBd;
    double* H = sm + L.Hd;
    double* Hy = sm + L.Hyd;
    double* Kk = sm + L.Kd;
    double* sb = sm + L.sb;
    const double* th = sm + L.th;
    const StageSrc src{A, B, Wg, d.sA, d.sB, d.sA, 1};  // [A_k | B_k | W_{k-1}]
    Pipe<G::KPW> pp(src, d.SW, N, d.Sl, true, sb);
    pp.prime();
    for (int e = l; e < na * na; e += kWave) {
        const int i = e / na, j = e - i * na;
        st_dd(P, e, dd_of((i < nx && j < nx) ? Wg[(size_t)(N - 1) * nx * nx + i * nx + j] : 0.0));
    }
    wsync();
    bool ok = true;
    sweep(pp, [&](int k, const double* Ak) {
        const double* Bk = Ak + d.sA;
        // PA = P[:, :nx] A_k (na x nx);  PB = P [B_k; I] (na x nu)
        if constexpr (kP1 && G::NX != 0) {
            // fixed dimensions: a lane's entries (l, l + 64) with every read issued before the two
            // chains, which then run interleaved (same sums; clamped entries are computed, not stored)
            constexpr int NX = G::NX, NU = G::NU, NA = NX + NU, E1 = NA * (NX + NU);
            constexpr int QN = (E1 + kWave - 1) / kWave;
            dd v[QN], pr[QN][NX];
            double cf[QN][NX];
#pragma unroll
            for (int q = 0; q < QN; ++q) {
                int e = l + q * kWave;
                e = e < E1 ? e : E1 - 1;
                const bool isA = e < NA * NX;
                const int e2 = e - NA * NX;
                const int i = isA ? e / NX : e2 / NU, j = isA ? e - (e / NX) * NX : e2 - (e2 / NU) * NU;
                const double* cp = isA ? Ak + j : Bk + j;
                const int cs = isA ? NX : NU;
                v[q] = isA ? dd_of(0.0) : ld_dd(P, i * NA + NX + j);
#pragma unroll
                for (int s2 = 0; s2 < NX; ++s2) {
                    pr[q][s2] = ld_dd(P, i * NA + s2);
                    cf[q][s2] = cp[s2 * cs];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2)
#pragma unroll
                for (int q = 0; q < QN; ++q) v[q] = dd_fmad(v[q], pr[q][s2], cf[q][s2]);
#pragma unroll
            for (int q = 0; q < QN; ++q) {
                const int e = l + q * kWave;
                if (e < NA * NX) st_dd(PA, e, v[q]);
                else if (e < E1) st_dd(PB, e - NA * NX, v[q]);
            }
        } else
        for (int e = l; e < na * (nx + nu); e += kWave) {
            if (e < na * nx) {
                const int i = e / nx, j = e - i * nx;
                dd v = dd_of(0.0);
                for (int s2 = 0; s2 < nx; ++s2) v = dd_fmad(v, ld_dd(P, i * na + s2), Ak[s2 * nx + j]);
                st_dd(PA, e, v);
            } else {
                const int e2 = e - na * nx, i = e2 / nu, cc = e2 - i * nu;
                dd v = ld_dd(P, i * na + nx + cc);
                for (int s2 = 0; s2 < nx; ++s2) v = dd_fmad(v, ld_dd(P, i * na + s2), Bk[s2 * nu + cc]);
                st_dd(PB, e2, v);
            }
        }
        wsync();
        // Hvy = [B'PA + PA_u | -2dR] (nu x na);  Hvv = 2R + 2dR + diag(th_u) + B'PB + PB_u (nu x nu)
        if constexpr (kP1 && G::NX != 0) {
            // fixed dimensions (nu na + nu nu <= 64: one entry per lane), every read issued before
            // the chain (same sums; the Hvy columns j >= nx take their -2dR value at the end)
            constexpr int NX = G::NX, NU = G::NU, NA = NX + NU, EY = NU * NA, E2 = EY + NU * NU;
            static_assert(E2 <= kWave, "one Hvy / Hvv entry per lane");
            const int e = l < E2 ? l : E2 - 1;
            const bool isY = e < EY;
            const int cc = isY ? e / NA : (e - EY) / NU;
            const int j = isY ? e - cc * NA : 0, ee = isY ? 0 : (e - EY) - cc * NU;
            const int jc = j < NX ? j : 0;
            const double* ob = isY ? PA + 2 * jc : PB + 2 * ee;   // operand column (dd)
            const int os = isY ? NX : NU;
            dd v = isY ? (j < NX ? ld_dd(PA, (NX + cc) * NX + jc) : dd_of(0.0))
                       : dd_add(dd_ts(2.0 * c.R[cc * NU + ee], 2.0 * c.dR[cc * NU + ee]), ld_dd(PB, (NX + cc) * NU + ee));
            dd pr[NX];
            double cf[NX];
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2) {
                pr[s2] = ld_dd(ob, s2 * os);
                cf[s2] = Bk[s2 * NU + cc];
            }
            const int rr = c.ms + 2 * (k * NU + cc);
            const double th0 = th[rr], th1 = th[rr + 1];
            const double dry = -2.0 * c.dR[cc * NU + (j >= NX ? j - NX : 0)];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2) v = dd_fmad(v, pr[s2], cf[s2]);
            if (!isY && cc == ee) v = dd_add(v, dd_ts(th0, th1));
            if (isY && j >= NX) v = dd_of(dry);
            if (l < EY) st_dd(Hy, l, v);
            else if (l < E2) st_dd(H, l - EY, v);
        } else
        for (int e = l; e < nu * na + nu * nu; e += kWave) {
            if (e < nu * na) {
                const int cc = e / na, j = e - cc * na;
                dd v;
                if (j < nx) {
                    v = ld_dd(PA, (nx + cc) * nx + j);
                    for (int s2 = 0; s2 < nx; ++s2) v = dd_fmad(v, ld_dd(PA, s2 * nx + j), Bk[s2 * nu + cc]);
                } else {
                    v = dd_of(-2.0 * c.dR[cc * nu + (j - nx)]);
                }
                st_dd(Hy, e, v);
            } else {
                const int e2 = e - nu * na, cc = e2 / nu, ee = e2 - cc * nu;
                dd v = dd_add(dd_ts(2.0 * c.R[cc * nu + ee], 2.0 * c.dR[cc * nu + ee]), ld_dd(PB, (nx + cc) * nu + ee));
                for (int s2 = 0; s2 < nx; ++s2) v = dd_fmad(v, ld_dd(PB, s2 * nu + ee), Bk[s2 * nu + cc]);
                if (cc == ee) {
                    const int rr = c.ms + 2 * (k * nu + cc);
                    v = dd_add(v, dd_ts(th[rr], th[rr + 1]));
                }
                st_dd(H, e2, v);
            }
        }
        wsync();
        // Cholesky of Hvv and its inverse, in registers (every lane; nu <= 4)
        dd Lf[CMPC_MAX_NU][CMPC_MAX_NU], Hi[CMPC_MAX_NU][CMPC_MAX_NU];
#pragma unroll
        for (int a = 0; a < CMPC_MAX_NU; ++a)
#pragma unroll
            for (int b = 0; b < CMPC_MAX_NU; ++b) Lf[a][b] = (a < nu && b <= a) ? ld_dd(H, a * nu + b) : dd_of(0.0);
#pragma unroll
        for (int j = 0; j < CMPC_MAX_NU; ++j) {
            if (j < nu) {
                dd dj = Lf[j][j];
#pragma unroll
                for (int p = 0; p < j; ++p) dj = dd_sub(dj, dd_mul(Lf[j][p], Lf[j][p]));
                ok = ok && (dj.hi > 0.0);
                if (!(dj.hi > 0.0)) dj = dd_of(1.0);
                dj = dd_sqrt(dj);
                Lf[j][j] = dj;
#pragma unroll
                for (int i = j + 1; i < CMPC_MAX_NU; ++i) {
                    if (i < nu) {
                        dd v = Lf[i][j];
#pragma unroll
                        for (int p = 0; p < j; ++p) v = dd_sub(v, dd_mul(Lf[i][p], Lf[j][p]));
                        Lf[i][j] = dd_div(v, dj);
                    }
                }
            }
        }
#pragma unroll
        for (int col = 0; col < CMPC_MAX_NU; ++col) {
            dd e[CMPC_MAX_NU];
#pragma unroll
            for (int i = 0; i < CMPC_MAX_NU; ++i) e[i] = dd_of(i == col ? 1.0 : 0.0);
#pragma unroll
            for (int i = 0; i < CMPC_MAX_NU; ++i) {
                if (i < nu) {
                    dd v = e[i];
#pragma unroll
                    for (int p = 0; p < i; ++p) v = dd_sub(v, dd_mul(Lf[i][p], e[p]));
                    e[i] = dd_div(v, Lf[i][i]);
                }
            }
#pragma unroll
            for (int i = CMPC_MAX_NU - 1; i >= 0; --i) {
                if (i < nu) {
                    dd v = e[i];
#pragma unroll
                    for (int p = i + 1; p < CMPC_MAX_NU; ++p)
                        if (p < nu) v = dd_sub(v, dd_mul(Lf[p][i], e[p]));
                    e[i] = dd_div(v, Lf[i][i]);
                }
            }
#pragma unroll
            for (int i = 0; i < CMPC_MAX_NU; ++i) Hi[i][col] = e[i];
        }
        // K_k = -Hinv Hvy (nu x na) into LDS (dd) and F (double);  Hinv into F
        double* Fk = F + (size_t)k * d.sF;
        for (int e = l; e < nu * na; e += kWave) {
            const int a = e / na, j = e - a * na;
            dd v = dd_of(0.0);
#pragma unroll
            for (int b = 0; b < CMPC_MAX_NU; ++b) {
                if (b < nu) {
                    dd hab = dd_of(0.0);
#pragma unroll
                    for (int a2 = 0; a2 < CMPC_MAX_NU; ++a2)
                        if (a2 == a) hab = Hi[a2][b];
                    v = dd_sub(v, dd_mul(hab, ld_dd(Hy, b * na + j)));
                }
            }
            st_dd(Kk, e, v);
            Fk[e] = v.hi;
        }
        if (l < nu * nu) {
            const int a = l / nu, b = l - a * nu;
            double v = 0.0;
#pragma unroll
            for (int a2 = 0; a2 < CMPC_MAX_NU; ++a2)
#pragma unroll
                for (int b2 = 0; b2 < CMPC_MAX_NU; ++b2)
                    if (a2 == a && b2 == b) v = Hi[a2][b2].hi;
            Fk[nu * na + l] = v;
        }
        wsync();
        // P_k = blkdiag(W_k + A'Pxx A, 2dR) + Hvy'K_k
        if constexpr (kP4 && G::NX != 0) {
            // fixed dimensions: a lane's two entries (l, l + 64) as two interleaved chains, their
            // reads left to the compiler's schedule (hoisting both entries' operands spilled); the
            // A'Pxx A chain runs on every lane and is kept by the rows i < nx only (same sums)
            constexpr int NX = G::NX, NU = G::NU, NA = NX + NU, E4 = NA * NA;
            constexpr int QN = (E4 + kWave - 1) / kWave;
            int iq[QN], jq[QN], icq[QN], jcq[QN];
            dd v0[QN], t[QN];
#pragma unroll
            for (int q = 0; q < QN; ++q) {
                int e = l + q * kWave;
                e = e < E4 ? e : E4 - 1;
                iq[q] = e / NA;
                jq[q] = e - iq[q] * NA;
                icq[q] = iq[q] < NX ? iq[q] : NX - 1;
                jcq[q] = jq[q] < NX ? jq[q] : 0;
                v0[q] = iq[q] < NX ? dd_of(Ak[d.sAB + icq[q] * NX + jcq[q]])
                                   : dd_of((jq[q] >= NX) ? 2.0 * c.dR[(iq[q] - NX) * NU + (jq[q] >= NX ? jq[q] - NX : 0)] : 0.0);
                t[q] = v0[q];
            }
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2)
#pragma unroll
                for (int q = 0; q < QN; ++q) t[q] = dd_fmad(t[q], ld_dd(PA, s2 * NX + jcq[q]), Ak[s2 * NX + icq[q]]);
#pragma unroll
            for (int q = 0; q < QN; ++q) {
                dd v = iq[q] < NX ? t[q] : v0[q];
#pragma unroll
                for (int a = 0; a < NU; ++a) v = dd_fma(v, ld_dd(Hy, a * NA + iq[q]), ld_dd(Kk, a * NA + jq[q]));
                if (l + q * kWave < E4 && k > 0 && jq[q] <= iq[q]) {
                    st_dd(P, iq[q] * NA + jq[q], v);
                    st_dd(P, jq[q] * NA + iq[q], v);
                }
            }
        } else
        for (int e = l; e < na * na && k > 0; e += kWave) {
            const int i = e / na, j = e - i * na;
            if (j > i) continue;
            dd v;
            if (i < nx) {
                v = dd_of(Ak[d.sAB + i * nx + j]);
                for (int s2 = 0; s2 < nx; ++s2) v = dd_fmad(v, ld_dd(PA, s2 * nx + j), Ak[s2 * nx + i]);
            } else {
                v = dd_of((j >= nx) ? 2.0 * c.dR[(i - nx) * nu + (j - nx)] : 0.0);
            }
            for (int a = 0; a < nu; ++a) v = dd_fma(v, ld_dd(Hy, a * na + i), ld_dd(Kk, a * na + j));
            st_dd(P, i * na + j, v);
            st_dd(P, j * na + i, v);
        }
    });
    return ok;
}

// Solve the Newton system for the right-hand side rh (n values): dU (n) and, when dX is not
// null, dX ((N+1) nx, dX_0 = 0), with the gains of riccati_factor.
//
// Fused form (yb != null, rh unused): the right-hand side rh = -rd - (B'psi + rt_u) of a pass,
// whose psi is the adjoint recursion psi_k = yb_k + A_k' psi_{k+1} of the stage rows' C'rt,
// is formed inside the backward sweep: with s = psi + p_x (p the Riccati costate) both
// recursions become one, s_k = yb_k + A_k' s_{k+1} + (K_k'g)_x, g = p_u + rd_k + rt_u + B_k' s_{k+1}
// — one sweep fewer per pass.
// R = float (Cfg::F32): the backward recursion (g, p) and the forward feedback v_k in fp32 with the
// fp32 gains; the right-hand side, dU and the direction's state recursion dX in fp64.
template <class G, class R = double>
__device__ __forceinline__ void riccati_solve(const MpcConst& c, const Dims& d, const RLds& L, double* sm,
                              const double* __restrict__ A, const double* __restrict__ B,
                              const double* __restrict__ F, const double* rh, double* dU, double* dX,
                              const double* yb = nullptr, const double* rd = nullptr, const double* rt = nullptr,
                              int part = 3) {  // part: 1 the backward pass, 2 the forward pass, 3 both
    const int l = lane_id(), nx = d.nx, nu = d.nu, na = d.na, N = c.N;
    const int ms = c.ms;  // in a register: a read of c (LDS) inside a step waits on every read before it
    double* sb = sm + L.sb;
    double* pv = sm + L.pv;
    double* xb = sm + L.xpp;  // dX_k, ping-pong
    const StageSrc src{A, B, F, d.sA, d.sB, d.sF, 0};
    // backward: p_N = 0;  g = -rh_k + B'p_x + p_u;  kk_k = -Hinv g (into dU);  p_k = [A'p_x; 0] + K'g.
    // Every lane forms the nu values of g itself (nu <= 4), so a stage needs one barrier.
    if (part & 1) {
        Pipe<G::KP> pp(src, d.S, N, d.Sl, true, sb);
        pp.prime();
        if (l < na) pv[l] = (yb && l < nx) ? yb[N * nx + l] : 0.0;
        wsync();
        sweep(pp, [&](int k, const double* Ak) {
            const double* Bk = Ak + d.sA;
            const double* Kg = Bk + d.sB;
            const double* Hg = Kg + nu * na;
            const double* pc = pv + ((N - 1 - k) & 1) * na;
            double* pn = pv + ((N - k) & 1) * na;
            if constexpr (G::NX != 0) {
                // fixed dimensions: every read of the step issued before its chains (same sums)
                constexpr int NX = G::NX, NU = G::NU, NA = NX + NU;
                const int lx = l < NX ? l : NX - 1, la = l < NA ? l : NA - 1, lu = l < NU ? l : NU - 1;
                R p[NA], bm[NX][NU], ac[NX], kg[NU], hg[NU], r0[NU];
#pragma unroll
                for (int s2 = 0; s2 < NX; ++s2) {
#pragma unroll
                    for (int a = 0; a < NU; ++a) bm[s2][a] = (R)Bk[s2 * NU + a];
                    ac[s2] = (R)Ak[s2 * NX + lx];
                }
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    const int ci = k * NU + a;
                    r0[a] = (R)(yb ? rd[ci] + (rt[ms + 2 * ci] - rt[ms + 2 * ci + 1]) : -rh[ci]);
                    kg[a] = (R)Kg[a * NA + la];
                    hg[a] = (R)Hg[lu * NU + a];
                }
                const R y0 = (R)((yb && l < NX) ? yb[k * NX + l] : 0.0);
#pragma unroll
                for (int s2 = 0; s2 < NA; ++s2) p[s2] = (R)pc[s2];
                __builtin_amdgcn_sched_barrier(0);
                R g[NU];
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    R v = p[NX + a] + r0[a];
#pragma unroll
                    for (int s2 = 0; s2 < NX; ++s2) v = fma(bm[s2][a], p[s2], v);
                    g[a] = v;
                }
                R v = y0;
                if (l < NX) {
#pragma unroll
                    for (int s2 = 0; s2 < NX; ++s2) v = fma(ac[s2], p[s2], v);
                }
#pragma unroll
                for (int a = 0; a < NU; ++a) v = fma(kg[a], g[a], v);
                if (l < NA) pn[l] = v;
                if (l < NU) {
                    R u = R(0);
#pragma unroll
                    for (int b = 0; b < NU; ++b) u = fma(-hg[b], g[b], u);
                    dU[k * NU + l] = u;
                }
            } else if (l < na) {
                double g[CMPC_MAX_NU];
#pragma unroll
                for (int a = 0; a < CMPC_MAX_NU; ++a) {
                    double v = 0.0;
                    if (a < nu) {
                        const int ci = k * nu + a;
                        v = pc[nx + a] + (yb ? rd[ci] + (rt[c.ms + 2 * ci] - rt[c.ms + 2 * ci + 1]) : -rh[ci]);
                        for (int s2 = 0; s2 < nx; ++s2) v = fma(Bk[s2 * nu + a], pc[s2], v);
                    }
                    g[a] = v;
                }
                double v = (yb && l < nx) ? yb[k * nx + l] : 0.0;
                if (l < nx)
                    for (int s2 = 0; s2 < nx; ++s2) v = fma(Ak[s2 * nx + l], pc[s2], v);
#pragma unroll
                for (int a = 0; a < CMPC_MAX_NU; ++a)
                    if (a < nu) v = fma(Kg[a * na + l], g[a], v);
                pn[l] = v;
                if (l < nu) {
                    double u = 0.0;
#pragma unroll
                    for (int b = 0; b < CMPC_MAX_NU; ++b)
                        if (b < nu) u = fma(-Hg[l * nu + b], g[b], u);
                    dU[k * nu + l] = u;
                }
            }
        });
    }
    // forward: y_0 = 0;  v_k = kk_k + K_k y_k;  dX_{k+1} = A_k dX_k + B_k v_k (every lane < nx forms v_k)
    if (part & 2) {
        Pipe<G::KP> pp(src, d.S, N, d.Sl, false, sb);
        pp.prime();
        if (l < nx) {
            xb[l] = 0.0;
            if (dX) dX[l] = 0.0;
        }
        wsync();
        sweep(pp, [&](int k, const double* Ak) {
            const double* Bk = Ak + d.sA;
            const double* Kg = Bk + d.sB;
            const double* xc = xb + (k & 1) * nx;
            if constexpr (G::NX != 0) {
                // fixed dimensions: every read of the step issued before its chains (same sums)
                constexpr int NX = G::NX, NU = G::NU, NA = NX + NU;
                const int lx = l < NX ? l : NX - 1;
                double x[NX], ar[NX], br[NU];
                R kg[NU][NA], d0[NU], dp[NU];
#pragma unroll
                for (int a = 0; a < NU; ++a) {
#pragma unroll
                    for (int j = 0; j < NA; ++j) kg[a][j] = (R)Kg[a * NA + j];
                    d0[a] = (R)dU[k * NU + a];
                    dp[a] = (R)dU[(k > 0 ? k - 1 : 0) * NU + a];
                    br[a] = Bk[lx * NU + a];
                }
#pragma unroll
                for (int t = 0; t < NX; ++t) ar[t] = Ak[lx * NX + t];
#pragma unroll
                for (int t = 0; t < NX; ++t) x[t] = xc[t];
                __builtin_amdgcn_sched_barrier(0);
                R vk[NU];
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    R v = d0[a];
#pragma unroll
                    for (int j = 0; j < NX; ++j) v = fma(kg[a][j], (R)x[j], v);
                    if (k > 0)
#pragma unroll
                        for (int b = 0; b < NU; ++b) v = fma(kg[a][NX + b], dp[b], v);
                    vk[a] = v;
                }
                double v = 0.0;
#pragma unroll
                for (int t = 0; t < NX; ++t) v = fma(ar[t], x[t], v);
#pragma unroll
                for (int a = 0; a < NU; ++a) v = fma(br[a], (double)vk[a], v);
                if (l < NX) {
                    xb[((k + 1) & 1) * NX + l] = v;
                    if (dX) dX[(k + 1) * NX + l] = v;
                }
#pragma unroll
                for (int a = 0; a < NU; ++a)
                    if (l == a) dU[k * NU + a] = vk[a];
            } else if (l < nx || l < nu) {
                double vk[CMPC_MAX_NU];
#pragma unroll
                for (int a = 0; a < CMPC_MAX_NU; ++a) {
                    double v = 0.0;
                    if (a < nu) {
                        v = dU[k * nu + a];
                        for (int j = 0; j < nx; ++j) v = fma(Kg[a * na + j], xc[j], v);
                        if (k > 0)
                            for (int b = 0; b < nu; ++b) v = fma(Kg[a * na + nx + b], dU[(k - 1) * nu + b], v);
                    }
                    vk[a] = v;
                }
                if (l < nx) {
                    double v = 0.0;
                    for (int t = 0; t < nx; ++t) v = fma(Ak[l * nx + t], xc[t], v);
#pragma unroll
                    for (int a = 0; a < CMPC_MAX_NU; ++a)
                        if (a < nu) v = fma(Bk[l * nu + a], vk[a], v);
                    xb[((k + 1) & 1) * nx + l] = v;
                    if (dX) dX[(k + 1) * nx + l] = v;
                }
                // one wavefront: every lane's reads of dU_k above precede this write-back
#pragma unroll
                for (int a = 0; a < CMPC_MAX_NU; ++a)
                    if (a < nu && l == a) dU[k * nu + a] = vk[a];
            }
        });
    }
}

// Latency mode, wave 2: the predictor's backward Riccati pass (riccati_solve part 1 with the pass-0
// right-hand side, the same arithmetic) run stage by stage behind wave 1's factorisation and wave 0's
// residual adjoint sweep: stage k's gains from the LDS ring once prog_f says the factorisation has passed
// k, the adjoint's rd of stage k (finished here as the residual phase finishes it: + the 2R / 2dR gradient
// and the input rows' multipliers) once prog_a says the adjoint sweep has.  cons: stages done (the
// factorisation's ring back-pressure).  ybC: C'rt of the pass-0 rows.  Returns false on a wait timeout.
template <class G>
__device__ __forceinline__ bool riccati_back_piped(const MpcConst& c, const double* __restrict__ A,
                                                   const double* __restrict__ B, const double* ring, int sF,
                                                   const volatile double* prog_f, const volatile double* prog_a,
                                                   volatile double* cons, const double* ybC, const double* rdA,
                                                   const double* rt, const double* lam, const double* U,
                                                   const double* up, double* pv, double* dU, int ms) {
    constexpr int NX = G::NX, NU = G::NU, NA = NX + NU;
    static_assert(NX != 0, "fixed dimensions");
    const int l = lane_id(), N = c.N;
    const int lx = l < NX ? l : NX - 1, la = l < NA ? l : NA - 1, lu = l < NU ? l : NU - 1;
    if (l < NA) pv[l] = (l < NX) ? ybC[N * NX + l] : 0.0;
    wsync();
    bool okw = true;
    // A_k, B_k (kernel inputs, never written) prefetched one stage ahead into two register sets (a stage
    // that waited on its own loads ran at ~3 k clk, slower than the factorisation it follows)
    auto load = [&](int k, double (&bm)[NX][NU], double (&ac)[NX]) __attribute__((always_inline)) {
        const double* Ak = A + (size_t)k * NX * NX;
        const double* Bk = B + (size_t)k * NX * NU;
#pragma unroll
        for (int s2 = 0; s2 < NX; ++s2) {
#pragma unroll
            for (int a = 0; a < NU; ++a) bm[s2][a] = Bk[s2 * NU + a];
            ac[s2] = Ak[s2 * NX + lx];
        }
    };
    auto stage = [&](int k, const double (&bm)[NX][NU], const double (&ac)[NX]) __attribute__((always_inline)) {
        okw = spin_until(prog_a, (double)(N - k)) && okw;
        okw = spin_until(prog_f, (double)(N - k)) && okw;
        const double* Kg = ring + (k % kRing) * sF;
        const double* Hg = Kg + NU * NA;
        const double* pc = pv + ((N - 1 - k) & 1) * NA;
        double* pn = pv + ((N - k) & 1) * NA;
        double p[NA], kg[NU], hg[NU], r0[NU];
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            const int ci = k * NU + a, r = ms + 2 * ci;
            const double rdf = rdA[ci] + (rdr_grad<G>(c, U, up, ci) + lam[r] - lam[r + 1]);  // (the residual phase's rd)
            r0[a] = rdf + (rt[ms + 2 * ci] - rt[ms + 2 * ci + 1]);
            kg[a] = Kg[a * NA + la];
            hg[a] = Hg[lu * NU + a];
        }
        const double y0 = (l < NX) ? ybC[k * NX + l] : 0.0;
#pragma unroll
        for (int s2 = 0; s2 < NA; ++s2) p[s2] = pc[s2];
        __builtin_amdgcn_sched_barrier(0);
        double g[NU];
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            double v = p[NX + a] + r0[a];
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2) v = fma(bm[s2][a], p[s2], v);
            g[a] = v;
        }
        double v = y0;
        if (l < NX) {
#pragma unroll
            for (int s2 = 0; s2 < NX; ++s2) v = fma(ac[s2], p[s2], v);
        }
#pragma unroll
        for (int a = 0; a < NU; ++a) v = fma(kg[a], g[a], v);
        if (l < NA) pn[l] = v;
        if (l < NU) {
            double u = 0.0;
#pragma unroll
            for (int b = 0; b < NU; ++b) u = fma(-hg[b], g[b], u);
            dU[k * NU + l] = u;
        }
        wsync();
        if (l == 0) *cons = (double)(N - k);
    };
    double bm0[NX][NU], ac0[NX], bm1[NX][NU], ac1[NX];
    load(N - 1, bm0, ac0);
    for (int k = N - 1; k >= 0; k -= 2) {
        if (k >= 1) load(k - 1, bm1, ac1);
        stage(k, bm0, ac0);
        if (k < 1) break;
        if (k >= 2) load(k - 2, bm0, ac0);
        stage(k - 1, bm1, ac1);
    }
    return okw;
}

// out = rhs - K v with the product evaluated in double-double (the refinement residual of a
// double-double iteration):  K v = sum_k Gamma_k' W_k Gamma_k v + (2R + 2D'dR D + diag(th_u)) v,
// through the stage recursions (dd states in [yb, yb2), dd adjoint in psid).
template <class G>
__device__ __forceinline__ void kres_dd(const MpcConst& c, const Dims& d, const RLds& L, double* sm,
                                        const double* __restrict__ A, const double* __restrict__ B,
                                        const double* __restrict__ Wg, const double* v, const double* rhs,
                                        double* out) {
    const int l = lane_id(), nx = d.nx, nu = d.nu, N = c.N, nx2 = nx * nx;
    double* Xd = sm + L.yb;
    double* sb = sm + L.sb;
    const double* th = sm + L.th;
    double* psid = sm + L.psid;  // two dd vectors of nx, ping-pong
    const StageSrc src{A, B, B, d.sA, d.sB, d.sF, 0};  // third segment unused (cnt = sAB); never null
    // forward: X_0 = 0, X_{k+1} = A_k X_k + B_k v_k
    {
        Pipe<G::KP> pp(src, d.sAB, N, d.Sl, false, sb);
        pp.prime();
        if (l < nx) st_dd(Xd, l, dd_of(0.0));
        wsync();
        sweep(pp, [&](int k, const double* Ak) {
            const double* Bk = Ak + d.sA;
            if constexpr (G::NX != 0) {
                // fixed dimensions: every read of the step issued before its chain (same sums)
                constexpr int NX = G::NX, NU = G::NU;
                const int lx = l < NX ? l : NX - 1;
                dd x[NX];
                double ar[NX], br[NU], vk[NU];
#pragma unroll
                for (int t = 0; t < NX; ++t) {
                    ar[t] = Ak[lx * NX + t];
                    x[t] = ld_dd(Xd, k * NX + t);
                }
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    br[i] = Bk[lx * NU + i];
                    vk[i] = v[k * NU + i];
                }
                __builtin_amdgcn_sched_barrier(0);
                dd acc = dd_of(0.0);
#pragma unroll
                for (int t = 0; t < NX; ++t) acc = dd_fmad(acc, x[t], ar[t]);
#pragma unroll
                for (int i = 0; i < NU; ++i) acc = dd_fmadd(acc, br[i], vk[i]);
                if (l < NX) st_dd(Xd, (k + 1) * NX + l, acc);
            } else if (l < nx) {
                dd acc = dd_of(0.0);
                for (int t = 0; t < nx; ++t) acc = dd_fmad(acc, ld_dd(Xd, k * nx + t), Ak[l * nx + t]);
                for (int i = 0; i < nu; ++i) acc = dd_fmadd(acc, Bk[l * nu + i], v[k * nu + i]);
                st_dd(Xd, (k + 1) * nx + l, acc);
            }
        });
    }
    // adjoint: psi_N = W X_N, psi_k = W X_k + A_k' psi_{k+1};  out_k = rhs_k - B_k' psi_{k+1} - (...)
    {
        const StageSrc srw{A, B, Wg, d.sA, d.sB, d.sA, 1};  // [A_k | B_k | W_{k-1}]
        Pipe<G::KPW> pp(srw, d.SW, N, d.Sl, true, sb);
        pp.prime();
        if (l < nx) {
            dd acc = dd_of(0.0);
            for (int u = 0; u < nx; ++u) acc = dd_fmad(acc, ld_dd(Xd, N * nx + u), Wg[(size_t)(N - 1) * nx2 + l * nx + u]);
            st_dd(psid, l, acc);
        }
        wsync();
        sweep(pp, [&](int k, const double* Ak) {
            const double* Bk = Ak + d.sA;
            const double* pa = psid + ((N - 1 - k) & 1) * 2 * nx;
            double* pb = psid + ((N - k) & 1) * 2 * nx;
            if constexpr (G::NX != 0) {
                // fixed dimensions, one instruction stream for both lane groups (the branches ran
                // one after the other): lanes < NU form out_k, lanes 32.. psi_k.  An out lane runs
                // the psi lanes' W X_k terms on zeros first: dd_fmad({+0, +0}, {0, 0}, w) is
                // {+0, +0} exactly, so its sums are the generic path's; every read is issued first.
                constexpr int NX = G::NX, NU = G::NU;
                const bool po = l < NU;
                const int t = l >= 32 && l < 32 + NX ? l - 32 : 0, lu = po ? l : 0;
                const double* cp = po ? Bk + lu : Ak + t;   // psi_{k+1} coefficients: B_k[:, l] | A_k[:, t]
                const int cs = po ? NU : NX;
                dd x[NX], ps[NX];
                double w[NX], cf[NX], v0[NU], vm[NU], vp[NU], r2[NU], d2[NU];
#pragma unroll
                for (int u = 0; u < NX; ++u) {
                    w[u] = Ak[d.sAB + t * NX + u];
                    x[u] = po ? dd_of(0.0) : ld_dd(Xd, k * NX + u);
                    ps[u] = ld_dd(pa, u);
                    cf[u] = cp[u * cs];
                }
#pragma unroll
                for (int j = 0; j < NU; ++j) {
                    v0[j] = v[k * NU + j];
                    vm[j] = k ? -v[(k - 1) * NU + j] : 0.0;
                    vp[j] = k + 1 < N ? v[(k + 1) * NU + j] : 0.0;
                    r2[j] = 2.0 * c.R[lu * NU + j];
                    d2[j] = 2.0 * c.dR[lu * NU + j];
                }
                const int rr = c.ms + 2 * (k * NU + lu);
                const double th0 = th[rr], th1 = th[rr + 1], vl = v[k * NU + lu], rl = rhs[k * NU + lu];
                __builtin_amdgcn_sched_barrier(0);
                dd acc = dd_of(0.0);
#pragma unroll
                for (int u = 0; u < NX; ++u) acc = dd_fmad(acc, x[u], w[u]);
#pragma unroll
                for (int s2 = 0; s2 < NX; ++s2) acc = dd_fmad(acc, ps[s2], cf[s2]);
                if (po) {
#pragma unroll
                    for (int j = 0; j < NU; ++j) {
                        const dd dk = dd_ts(v0[j], vm[j]);
                        const dd dn = (k + 1 < N) ? dd_ts(vp[j], -v0[j]) : dd_of(0.0);
                        acc = dd_fmadd(acc, r2[j], v0[j]);
                        acc = dd_fmad(acc, dd_sub(dk, dn), d2[j]);
                    }
                    acc = dd_fmad(acc, dd_ts(th0, th1), vl);
                    out[k * NU + l] = dd_sub(dd_of(rl), acc).hi;
                } else if (k > 0 && l >= 32 && l < 32 + NX) {
                    st_dd(pb, t, acc);
                }
            } else if (l < nu) {
                dd acc = dd_of(0.0);
                for (int s2 = 0; s2 < nx; ++s2) acc = dd_fmad(acc, ld_dd(pa, s2), Bk[s2 * nu + l]);
                for (int j = 0; j < nu; ++j) {
                    const double vk = v[k * nu + j];
                    const dd dk = dd_ts(vk, k ? -v[(k - 1) * nu + j] : 0.0);
                    const dd dn = (k + 1 < N) ? dd_ts(v[(k + 1) * nu + j], -vk) : dd_of(0.0);
                    acc = dd_fmadd(acc, 2.0 * c.R[l * nu + j], vk);
                    acc = dd_fmad(acc, dd_sub(dk, dn), 2.0 * c.dR[l * nu + j]);
                }
                const int rr = c.ms + 2 * (k * nu + l);
                acc = dd_fmad(acc, dd_ts(th[rr], th[rr + 1]), v[k * nu + l]);
                out[k * nu + l] = dd_sub(dd_of(rhs[k * nu + l]), acc).hi;
            } else if (k > 0 && l >= 32 && l < 32 + nx) {
                const int t = l - 32;
                dd acc = dd_of(0.0);
                for (int u = 0; u < nx; ++u) acc = dd_fmad(acc, ld_dd(Xd, k * nx + u), Ak[d.sAB + t * nx + u]);
                for (int s2 = 0; s2 < nx; ++s2) acc = dd_fmad(acc, ld_dd(pa, s2), Ak[s2 * nx + t]);
                st_dd(pb, t, acc);
            }
        });
    }
}

template <class G>
__global__ __launch_bounds__(kWave) void mpc_riccati_kernel(const MpcConst c_arg, const MpcPtrs P) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    // launch order (cmpc_opts.order): clamped into range, so a bad entry cannot address outside the batch
    const int b = P.order ? min(max(P.order[blockIdx.x], 0), (int)gridDim.x - 1) : (int)blockIdx.x;
    if (c_arg.rescue == 3) {  // the fp32 path's fp64 pass (mpc_launch): the agents it left short of tol only
        if (P.status[b] == CMPC_SOLVED) return;
    } else if (c_arg.rescue) {  // rescue pass: agents handed over at a breakdown, or left CMPC_UNSOLVED, only
        const RGlb g0 = r_glb(c_arg);
        if (P.ws[(size_t)b * g0.total + g0.hand] != 1.0 && P.status[b] != CMPC_UNSOLVED) return;
    }
    const int l = threadIdx.x;
    // rescue 3 runs at tol * 1e-3 of the fp32 solve's tol: its rounding floor is the requested tol
    const double tol_req = c_arg.rescue == 3 ? 1e3 * c_arg.tol : c_arg.tol;
    const int it_prev = (c_arg.rescue == 3 && P.iters) ? P.iters[b] : 0;
    const RLds L = r_layout(c_arg);
    // the weights are indexed by lane-dependent expressions: read them from an LDS copy (a
    // kernel-argument struct indexed that way is materialised in scratch)
    {
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&c_arg);
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(sm + L.cst);
        for (int i = l; i < mpc_const_used_doubles(c_arg); i += kWave) dst[i] = src[i];
        wsync();
    }
    const MpcConst& c = *reinterpret_cast<const MpcConst*>(sm + L.cst);
    const Dims d = dims_t<G>(c);
    const RGlb gl = r_glb(c);
    const int nx = d.nx, nu = d.nu, N = c.N, ns = c.ns, mc = mc_t<G>(c), n = c.n, ms = c.ms, m = c.m;

    const double* __restrict__ A = P.A + (size_t)b * N * nx * nx;
    const double* __restrict__ B = P.B + (size_t)b * N * nx * nu;
    const double* __restrict__ x0 = P.x0 + (size_t)b * nx;
    const double* __restrict__ up = P.up + (size_t)b * nu;
    const double* __restrict__ pl = P.p + (size_t)b * (N + 1) * nx;
    const double* __restrict__ C = P.C + (size_t)b * N * mc * nx;
    const double* __restrict__ h = P.h + (size_t)b * N * mc;
    double* __restrict__ ws = P.ws + (size_t)b * gl.total;
    double* dta = ws + gl.dta;
    double* dla = ws + gl.dla;
    double* F = ws + gl.F;
    double* bU = ws + gl.bU;
    double* bsig = ws + gl.bsig;
    double* Wg = ws + gl.Wk;

    constexpr bool GR = G::GR;  // lane-owned rows in the global scratch (cross-lane reads: gsync)
    double* t = GR ? ws + gl.t : sm + L.t;
    double* lam = GR ? ws + gl.lam : sm + L.lam;
    double* th = sm + L.th;
    double* rp = GR ? ws + gl.rp : sm + L.rp;
    double* rho = GR ? ws + gl.rho : sm + L.rho;
    double* rt = sm + L.rt;
    double* w = GR ? ws + gl.w : sm + L.w;
    double* GdU = GR ? ws + gl.GdU : sm + L.GdU;
    auto rsync = [&]() {
        if constexpr (GR) gsync(); else wsync();
    };
    double* X = sm + L.X;
    double* dX = sm + L.dX;
    double* yb = sm + L.yb;
    double* psi = sm + L.psi;
    double* U = sm + L.U;
    double* dU = sm + L.dU;
    double* rd = sm + L.rd;
    double* gU = sm + L.gU;
    double* rh = sm + L.rh;
    double* cr = sm + L.cr;
    double* sig = sm + L.sig;
    double* dsig = sm + L.dsig;
    double* Dsig = sm + L.Dsig;
    double* rsig = sm + L.rsig;
    double* sb = sm + L.sb;
    const StageSrc sAB{A, B, B, d.sA, d.sB, d.sF, 0};  // third segment unused (cnt = sAB); never null

    for (int i = l; i < L.cst; i += kWave) sm[i] = 0.0;
    wsync();
    // rescue pass: continue from the iterate a condensed kernel handed over at its breakdown
    // (hand_doubles, internal.h), or start cold; the flag is consumed here, so a second rescue
    // pass over an agent this one leaves CMPC_UNSOLVED starts cold
    double* hand = ws + gl.hand;
    const bool warm = (c_arg.rescue == 1 || c_arg.rescue == 2) && hand[0] == 1.0;
    // double-double near the solution: a continued (rescue) solve from the start, a cold one only
    // once the fp64 recursion stops making progress or breaks down (kDdStall)
    // (rescue 3, the fp32 path's last pass: double-double at every iteration above kDdTh from the start —
    // the robust rule of round 2 — for the agents whose fp32 solve and its fp64 restart both stopped short)
    bool dd_on = warm || c_arg.rescue == 3;
    bool f32_on = G::F32 && !warm;  // Cfg::F32: fp32 factorisation and recursions until kRicF32Stall
    const int it0 = warm ? (int)hand[1] : 0;
    if (warm) {
        for (int i = l; i < n; i += kWave) U[i] = hand[2 + i];
        for (int i = l; i < N * ns; i += kWave) sig[i] = hand[2 + n + i];
        wsync();
    }
    // diagnostic per-section clock sums (MpcPtrs::stamps; tools/ric_stamps.py):
    // 0 residuals, 1 stage weights, 2 factor, 3 factor (dd), 4 rhs, 5 solve, 6 refinement,
    // 7 rows / slacks / step, 8 update, 12 dd iterations, 13 refinement steps, 14 setup + output
    const bool stamp = P.stamps != nullptr;
    unsigned long long* tsum = reinterpret_cast<unsigned long long*>(sm + L.stamps);
    unsigned long long t_a = stamp ? clock64_() : 0, t_b = 0;
#define RSTAMP(slot)                          \
    if (stamp) {                              \
        t_b = clock64_();                     \
        if (l == 0) tsum[slot] += t_b - t_a;  \
        t_a = t_b;                            \
    }
#define RCOUNT(slot) \
    if (stamp && l == 0) tsum[slot] += 1;

    // Cfg::F32: an fp32-mode solve that ends short of tol restarts cold in fp64 (no fp32 stage) at
    // tol * 1e-3, so that its rounding floor is the requested tol: on 4 rounds of 8192 BASELINE cfg5
    // agents 2 solves ended at status 2 with KKT 4e-6 / 7e-6 (a dual residual the fp32 phase left,
    // then a breakdown at th ~ 1e25); restarted, all 32768 solve with KKT <= 1e-6 (tools/f32_lab.py,
    // oracle RIC_F32).  `tol` is the attempt's tolerance, it_done the iterations of the first attempt.
    double tol = c.tol;
    int it_done = 0;
    bool kkt_stop = false;  // rescue 3 stopped at kkt < the requested tol (merit not below it)
    double best_m, best_kkt, kkt;
    int best_it, stop, it;
    for (int attempt = 0;; ++attempt) {
    // ---- row right-hand sides; inactive rows carry w = +inf ----
    for (int r = l; r < m; r += kWave) {
        double v;
        if (r < ms) {
            v = h[r];
        } else {
            const int q = r - ms, i = (q >> 1) % nu;
            v = (q & 1) ? -c.u_lb[i] : c.u_ub[i];
        }
        w[r] = isfinite(v) ? v : INFINITY;
    }
    wsync();
    fwd_sim<G>(c, d, sAB, sb, x0, U, X);

    double mact_l = 0.0, sp_l = 1.0;
    const size_t ht = hand_t(c);
    for (int r = l; r < m; r += kWave) {
        if (isfinite(w[r])) {
            if (warm) {
                t[r] = hand[ht + r];
                lam[r] = hand[ht + m + r];
            } else {
                const double g = row_value<G>(c, C, r, X, U, sig);
                t[r] = fmax(w[r] - g, kT0Floor);
                lam[r] = 1.0;
            }
            mact_l += 1.0;
            sp_l = fmax(sp_l, fabs(w[r]));
        } else {
            t[r] = 1.0;
            lam[r] = 0.0;
        }
    }
    const double mact = fmax(wave_sum(mact_l), 1.0);
    const double scale_p = wave_max(sp_l);
    rsync();  // lam: read across lanes by the residuals
    if (warm && l == 0) hand[0] = 0.0;  // (every lane has read the flag: `warm` steered the loop above)

    best_m = INFINITY;
    best_kkt = INFINITY;
    best_it = 0;
    stop = kStopMaxIter;
    kkt = INFINITY;
    RSTAMP(14);
    double alpha_prev = 1;  // step of the previous iteration (kShortStep guard)
    for (it = it0 + 1; it <= c.max_iter; ++it) {
        // ================= residuals (as mpc_ipm.hip) =================
        for (int i = l; i < (N + 1) * nx; i += kWave) {
            const int k = i / nx, s = i - k * nx;
            double v = 2.0 * pl[i];
            for (int u = 0; u < nx; ++u) v = fma(2.0 * c.Q[s * nx + u], X[k * nx + u], v);
            yb[i] = v;
        }
        wsync();
        if constexpr (G::NX != 0) {
            // both residual adjoints in one sweep: gU from yb, rd from yb2 = yb + C' lambda (stages 1..N)
            double* yb2 = sm + L.yb2;
            for (int i = l; i < (N + 1) * nx; i += kWave) {
                const int k = i / nx, s = i - k * nx;
                double v = 0.0;
                if (k > 0)
                    for (int r = 0; r < mc; ++r) v = fma(lam[(k - 1) * mc + r], C[((size_t)(k - 1) * mc + r) * nx + s], v);
                yb2[i] = k > 0 ? yb[i] + v : yb[i];
            }
            wsync();
            adjoint2<G>(c, d, sAB, sb, yb, gU, yb2, rd, sm + L.psid);
        } else {
            adjoint<G>(c, d, sAB, sb, yb, gU, psi);
        }
        double gs_l = 1.0;
        for (int i = l; i < n; i += kWave) {
            gU[i] += rdr_grad<G>(c, U, up, i);
            gs_l = nmax(gs_l, fabs(gU[i]));
        }
        const double gscale = wave_max(gs_l);
        if constexpr (G::NX == 0) {
            for (int i = l; i < N * nx; i += kWave) {  // + C' lambda on stages 1..N
                const int k = i / nx, s = i - k * nx;
                double v = 0.0;
                for (int r = 0; r < mc; ++r) v = fma(lam[k * mc + r], C[((size_t)k * mc + r) * nx + s], v);
                yb[(k + 1) * nx + s] += v;
            }
            wsync();
            adjoint<G>(c, d, sAB, sb, yb, rd, psi);
        }
        double nrd_l = 0.0, nrs_l = 0.0, nrp_l = 0.0, mu_l = 0.0;
        for (int i = l; i < n; i += kWave) {
            const int r = ms + 2 * i;
            rd[i] += rdr_grad<G>(c, U, up, i) + lam[r] - lam[r + 1];
            nrd_l = nmax(nrd_l, fabs(rd[i]));
        }
        for (int i = l; i < N * ns; i += kWave) {
            const int k = i / ns, j = i - k * ns;
            double v = 2.0 * c.Qs[j] * sig[i];
            constexpr int MCB = G::MC ? G::MC : CMPC_MAX_MC;
            double lk[MCB];
#pragma unroll
            for (int r = 0; r < MCB; ++r) lk[r] = r < mc ? lam[k * mc + r] : 0.0;
#pragma unroll
            for (int r = 0; r < MCB; ++r)
                if (r < mc && c.row_slack[r] == j) v += c.row_sign[r] * lk[r];
            rsig[i] = v;
            nrs_l = nmax(nrs_l, fabs(v));
        }
        for (int r0 = l; r0 < m; r0 += kRowChunk * kWave) {
            double wv[kRowChunk], tv[kRowChunk], lv[kRowChunk], gv[kRowChunk];
#pragma unroll
            for (int i = 0; i < kRowChunk; ++i) {
                const int r = r0 + i * kWave, rc = r < m ? r : l;
                wv[i] = w[rc];
                tv[i] = t[rc];
                lv[i] = lam[rc];
                gv[i] = row_value<G>(c, C, rc, X, U, sig);
            }
#pragma unroll
            for (int i = 0; i < kRowChunk; ++i) {
                const int r = r0 + i * kWave;
                if (r >= m) break;
                if (isfinite(wv[i])) {
                    const double v = gv[i] + tv[i] - wv[i];
                    rp[r] = v;
                    nrp_l = nmax(nrp_l, fabs(v));
                    mu_l += tv[i] * lv[i];
                } else {
                    rp[r] = 0.0;
                }
            }
        }
        const double mu = wave_sum(mu_l) / mact;
        const double res = nmax(nmax(wave_max(nrd_l) / gscale, wave_max(nrs_l) / c.qs_max), wave_max(nrp_l) / scale_p);
        kkt = nmax(res, mu);
        const double merit = nmax(res, 1e4 * mu);
        if (!isfinite(merit)) {
            stop = kStopNonFinite;
            break;
        }
        if (merit < best_m) {
            best_m = merit;
            best_kkt = kkt;
            best_it = it;
            for (int i = l; i < n; i += kWave) bU[i] = U[i];
            for (int i = l; i < N * ns; i += kWave) bsig[i] = sig[i];
        }
        if (merit < tol) {
            stop = kStopConverged;
            break;
        }
        if (c_arg.rescue == 3 && kkt < tol_req) {  // the last pass stops at the KKT bar (status 2 below)
            kkt_stop = true;
            stop = kStopConverged;
            break;
        }
        if (best_m < 1e3 * tol && it - best_it >= kStallIters) {
            stop = kStopStalled;
            break;
        }
        if (warm && it - best_it >= kWarmStall) {  // continued solve without progress (internal.h)
            stop = kStopStalled;
            break;
        }
        wsync();

        RSTAMP(0);
        // ================= Newton system: Riccati factorisation =================
        for (int r0 = l; r0 < m; r0 += kRowChunk * kWave) {
            double wv[kRowChunk], tv[kRowChunk], lv[kRowChunk];
#pragma unroll
            for (int i = 0; i < kRowChunk; ++i) {
                const int r = r0 + i * kWave, rc = r < m ? r : l;
                wv[i] = w[rc];
                tv[i] = t[rc];
                lv[i] = lam[rc];
            }
#pragma unroll
            for (int i = 0; i < kRowChunk; ++i) {
                const int r = r0 + i * kWave;
                if (r < m) th[r] = isfinite(wv[i]) ? (c_arg.rescue == 3 ? fmin(lv[i] / tv[i], kThCapLast) : lv[i] / tv[i]) : 0.0;
            }
        }
        wsync();
        for (int i = l; i < N * ns; i += kWave) {
            const int k = i / ns, j = i - k * ns;
            double v = 2.0 * c.Qs[j];
            for (int r = 0; r < mc; ++r)
                if (c.row_slack[r] == j) v += th[k * mc + r];
            Dsig[i] = v;
        }
        wsync();
        stage_weights<G>(c, L, sm, C, Wg);
        gsync();  // W_k: stored by one lane, read by others
        double thm_l = 0.0;
        for (int r = l; r < m; r += kWave) thm_l = fmax(thm_l, th[r]);
        const bool above = wave_max(thm_l) > kDdTh;  // wave-uniform
        if (f32_on && it - best_it >= kRicF32Stall) f32_on = false;
        if (!f32_on && !dd_on && it - best_it >= kDdStall) dd_on = true;
        bool hp = above && dd_on && !f32_on;
        wsync();
        RSTAMP(1);
        bool fact_ok;
        if constexpr (G::F32) {
            fact_ok = f32_on ? riccati_factor<G, float>(c, d, L, sm, A, B, Wg, F)
                             : (hp ? riccati_factor_dd<G>(c, d, L, sm, A, B, Wg, F)
                                   : riccati_factor<G>(c, d, L, sm, A, B, Wg, F, stamp ? tsum : nullptr));
            if (!fact_ok && f32_on) {  // fp32 breakdown: this iteration and the rest in fp64
                gsync();
                f32_on = false;
                fact_ok = riccati_factor<G>(c, d, L, sm, A, B, Wg, F);
            }
        } else {
            fact_ok = hp ? riccati_factor_dd<G>(c, d, L, sm, A, B, Wg, F)
                         : riccati_factor<G>(c, d, L, sm, A, B, Wg, F, stamp ? tsum : nullptr);
        }
        if (!fact_ok && !hp && above) {  // fp64 breakdown above the threshold: this iteration and the rest in dd
            gsync();
            dd_on = hp = true;
            fact_ok = riccati_factor_dd<G>(c, d, L, sm, A, B, Wg, F);
        }
        gsync();  // gains F: stored by the factor's lanes, read by every lane of the solves
        if (!fact_ok) {
            stop = kStopBreakdown;
            break;
        }
        RSTAMP(hp ? 3 : 2);
        if (hp) RCOUNT(12);

        // ================= predictor / corrector =================
        double sig_c = 0.0, alpha = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            for (int r0 = l; r0 < m; r0 += kRowChunk * kWave) {
                double wv[kRowChunk], tv[kRowChunk], lv[kRowChunk], pv[kRowChunk], av[kRowChunk], bv[kRowChunk];
#pragma unroll
                for (int i = 0; i < kRowChunk; ++i) {
                    const int r = r0 + i * kWave, rc = r < m ? r : l;
                    wv[i] = w[rc];
                    tv[i] = t[rc];
                    lv[i] = lam[rc];
                    pv[i] = rp[rc];
                    av[i] = pass ? dta[rc] : 0.0;
                    bv[i] = pass ? dla[rc] : 0.0;
                }
#pragma unroll
                for (int i = 0; i < kRowChunk; ++i) {
                    const int r = r0 + i * kWave;
                    if (r >= m) break;
                    if (!isfinite(wv[i])) {
                        rho[r] = 0.0;
                        continue;
                    }
                    double rc = -tv[i] * lv[i];
                    if (pass) rc += sig_c * mu - av[i] * bv[i];
                    rho[r] = (rc + lv[i] * pv[i]) / tv[i];
                }
            }
            rsync();  // rho: read across lanes (same-stage rows, slack directions)
            for (int r = l; r < m; r += kWave) {
                double v = rho[r];
                if (r < ms) {
                    const int k = r / mc, rr = r - k * mc, j = c.row_slack[rr];
                    if (j >= 0) {
                        constexpr int MCB = G::MC ? G::MC : CMPC_MAX_MC;
                        double rk[MCB];  // the stage's rho, loaded together
#pragma unroll
                        for (int r2 = 0; r2 < MCB; ++r2) rk[r2] = r2 < mc ? rho[k * mc + r2] : 0.0;
                        const double q = 2.0 * c.Qs[j];
                        v = q * rho[r] - th[r] * c.row_sign[rr] * rsig[k * ns + j];
#pragma unroll
                        for (int r2 = 0; r2 < MCB; ++r2) {
                            if (r2 >= mc || r2 == rr || c.row_slack[r2] != j) continue;
                            const int R2 = k * mc + r2;
                            v += th[R2] * rho[r] - th[r] * c.row_sign[rr] * c.row_sign[r2] * rk[r2];
                        }
                        v /= Dsig[k * ns + j];
                    }
                }
                rt[r] = v;
            }
            wsync();
            for (int i = l; i < (N + 1) * nx; i += kWave) {
                const int k = i / nx, s = i - k * nx;
                double v = 0.0;
                if (k > 0)
                    for (int r = 0; r < mc; ++r) v = fma(rt[(k - 1) * mc + r], C[((size_t)(k - 1) * mc + r) * nx + s], v);
                yb[i] = v;
            }
            wsync();
            if (!hp) {
                RSTAMP(4);
                bool done = false;
                if constexpr (G::F32) {
                    if (f32_on) {
                        riccati_solve<G, float>(c, d, L, sm, A, B, F, nullptr, dU, dX, yb, rd, rt);
                        done = true;
                    }
                }
                if (!done) riccati_solve<G>(c, d, L, sm, A, B, F, nullptr, dU, dX, yb, rd, rt);  // rhs fused in
                RSTAMP(5);
            } else {
                adjoint<G>(c, d, sAB, sb, yb, rh, psi);
                // rhs = -rd - G' rt (kept: the refinement measures residuals against it)
                for (int i = l; i < n; i += kWave) rh[i] = -rd[i] - (rh[i] + rt[ms + 2 * i] - rt[ms + 2 * i + 1]);
                wsync();
                RSTAMP(4);
                riccati_solve<G>(c, d, L, sm, A, B, F, rh, dU, dX);
                RSTAMP(5);
                // refinement: dU += M^-1 (rhs - K dU), residual in double-double (gU, cr: free here)
                const int nref = warm ? kRefineMaxWarm : kRefineMax;
                for (int ir = 0; ir < nref; ++ir) {
                    kres_dd<G>(c, d, L, sm, A, B, Wg, dU, rh, gU);
                    riccati_solve<G>(c, d, L, sm, A, B, F, gU, cr, nullptr);
                    double cn_l = 0.0, un_l = 0.0;
                    for (int i = l; i < n; i += kWave) {
                        const double u = dU[i] + cr[i];
                        dU[i] = u;
                        cn_l = nmax(cn_l, fabs(cr[i]));
                        un_l = fmax(un_l, fabs(u));
                    }
                    const double cn = wave_max(cn_l), un = wave_max(un_l);
                    wsync();
                    RCOUNT(13);
                    if (!(cn > kRefineTol * un)) break;
                }
                fwd_sim<G>(c, d, sAB, sb, nullptr, dU, dX);
                RSTAMP(6);
            }
            for (int r0 = l; r0 < m; r0 += kRowChunk * kWave) {
                double gv[kRowChunk];
#pragma unroll
                for (int i = 0; i < kRowChunk; ++i) {
                    const int r = r0 + i * kWave;
                    gv[i] = row_value<G>(c, C, r < m ? r : l, dX, dU, nullptr);
                }
#pragma unroll
                for (int i = 0; i < kRowChunk; ++i)
                    if (r0 + i * kWave < m) GdU[r0 + i * kWave] = gv[i];
            }
            rsync();  // GdU: read across lanes by the slack directions
            for (int i = l; i < N * ns; i += kWave) {
                const int k = i / ns, j = i - k * ns;
                double v = rsig[i];
                constexpr int MCB = G::MC ? G::MC : CMPC_MAX_MC;
                double rk[MCB], gk[MCB];  // the stage's rho and GdU, loaded together
#pragma unroll
                for (int r = 0; r < MCB; ++r) {
                    rk[r] = r < mc ? rho[k * mc + r] : 0.0;
                    gk[r] = r < mc ? GdU[k * mc + r] : 0.0;
                }
#pragma unroll
                for (int r = 0; r < MCB; ++r)
                    if (r < mc && c.row_slack[r] == j) {
                        const int R1 = k * mc + r;
                        v += c.row_sign[r] * (rk[r] + th[R1] * gk[r]);
                    }
                dsig[i] = -v / Dsig[i];
            }
            wsync();
            double amax_l = 1.0e300;
            double* dtp = pass ? rho : dta;  // corrector reuses rho/rt storage for (dt, dl)
            double* dlp = pass ? rt : dla;
            for (int r0 = l; r0 < m; r0 += kRowChunk * kWave) {
                double wv[kRowChunk], rv[kRowChunk], pv[kRowChunk], gv[kRowChunk], tv[kRowChunk], lv[kRowChunk];
#pragma unroll
                for (int i = 0; i < kRowChunk; ++i) {
                    const int r = r0 + i * kWave, rc = r < m ? r : l;
                    wv[i] = w[rc];
                    rv[i] = rho[rc];
                    pv[i] = rp[rc];
                    gv[i] = GdU[rc];
                    tv[i] = t[rc];
                    lv[i] = lam[rc];
                }
#pragma unroll
                for (int i = 0; i < kRowChunk; ++i) {
                    const int r = r0 + i * kWave;
                    if (r >= m) break;
                    if (!isfinite(wv[i])) {
                        dtp[r] = 0.0;
                        dlp[r] = 0.0;
                        continue;
                    }
                    double sd = 0.0;
                    if (r < ms) {
                        const int k = r / mc, rr = r - k * mc, j = c.row_slack[rr];
                        if (j >= 0) sd = c.row_sign[rr] * dsig[k * ns + j];
                    }
                    const double rho_r = rv[i];
                    const double dtv = -pv[i] - gv[i] - sd;
                    const double dlv = rho_r + th[r] * (gv[i] + sd);
                    dtp[r] = dtv;
                    dlp[r] = dlv;
                    if (dtv < 0.0) amax_l = fmin(amax_l, -tv[i] / dtv);
                    if (dlv < 0.0) amax_l = fmin(amax_l, -lv[i] / dlv);
                }
            }
            const double amax = fmin(wave_min(amax_l), 1.0e300);
            wsync();
            if (!pass) {
                const double a = fmin(amax, 1.0);
                double mua_l = 0.0;
                for (int r0 = l; r0 < m; r0 += kRowChunk * kWave) {
                    double wv[kRowChunk], tv[kRowChunk], lv[kRowChunk], av[kRowChunk], bv[kRowChunk];
#pragma unroll
                    for (int i = 0; i < kRowChunk; ++i) {
                        const int r = r0 + i * kWave, rc = r < m ? r : l;
                        wv[i] = w[rc];
                        tv[i] = t[rc];
                        lv[i] = lam[rc];
                        av[i] = dta[rc];
                        bv[i] = dla[rc];
                    }
#pragma unroll
                    for (int i = 0; i < kRowChunk; ++i)
                        if (r0 + i * kWave < m && isfinite(wv[i])) mua_l += (tv[i] + a * av[i]) * (lv[i] + a * bv[i]);
                }
                const double mu_aff = wave_sum(mua_l) / mact;
                const double ratio = mu > 0.0 ? mu_aff / mu : 0.0;
                // e = 3; a warm continuation of a condensed solve keeps that method's e = 2 (internal.h)
                sig_c = warm ? ratio * ratio : ratio * ratio * ratio;
                if (alpha_prev < kShortStep) sig_c = fmax(sig_c, kSigmaMin);
            } else {
                alpha = fmin(1.0, 0.995 * amax);
                // stay in the wide neighbourhood t_r lam_r >= gamma mu(alpha) (see kNbhdGamma)
                for (int bt = 0; bt < kMaxBacktrack; ++bt) {
                    double mn_l = 0.0, pm_l = INFINITY;
                    for (int r0 = l; r0 < m; r0 += kRowChunk * kWave) {
                        double wv[kRowChunk], tv[kRowChunk], rv[kRowChunk], lv[kRowChunk], qv[kRowChunk];
#pragma unroll
                        for (int i = 0; i < kRowChunk; ++i) {
                            const int r = r0 + i * kWave, rc = r < m ? r : l;
                            wv[i] = w[rc];
                            tv[i] = t[rc];
                            rv[i] = rho[rc];
                            lv[i] = lam[rc];
                            qv[i] = rt[rc];
                        }
#pragma unroll
                        for (int i = 0; i < kRowChunk; ++i)
                            if (r0 + i * kWave < m && isfinite(wv[i])) {
                                const double pr = (tv[i] + alpha * rv[i]) * (lv[i] + alpha * qv[i]);
                                mn_l += pr;
                                pm_l = fmin(pm_l, pr);
                            }
                    }
                    if (wave_min(pm_l) >= kNbhdGamma * (wave_sum(mn_l) / mact)) break;
                    alpha *= 0.8;
                }
            }
            RSTAMP(7);
        }
        // ---- update (corrector direction: dU, dX, dsig, (rho, rt) = (dt, dl)) ----
        alpha_prev = alpha;
        for (int i = l; i < n; i += kWave) U[i] = fma(alpha, dU[i], U[i]);
        for (int i = l; i < N * ns; i += kWave) sig[i] = fma(alpha, dsig[i], sig[i]);
        for (int i = l; i < (N + 1) * nx; i += kWave) X[i] = fma(alpha, dX[i], X[i]);
        for (int r0 = l; r0 < m; r0 += kRowChunk * kWave) {
            double wv[kRowChunk], tv[kRowChunk], rv[kRowChunk], lv[kRowChunk], qv[kRowChunk];
#pragma unroll
            for (int i = 0; i < kRowChunk; ++i) {
                const int r = r0 + i * kWave, rc = r < m ? r : l;
                wv[i] = w[rc];
                tv[i] = t[rc];
                rv[i] = rho[rc];
                lv[i] = lam[rc];
                qv[i] = rt[rc];
            }
#pragma unroll
            for (int i = 0; i < kRowChunk; ++i) {
                const int r = r0 + i * kWave;
                if (r < m && isfinite(wv[i])) {
                    t[r] = fma(alpha, rv[i], tv[i]);
                    lam[r] = fma(alpha, qv[i], lv[i]);
                }
            }
        }
        rsync();  // lam: read across lanes by the next residuals
        RSTAMP(8);
    }
    if (it > c.max_iter) it = c.max_iter;
    wsync();
    if constexpr (G::F32) {
        if (attempt == 0 && !warm && stop != kStopConverged) {  // the fp64 restart (above)
            it_done = it;
            f32_on = dd_on = false;
            tol = c.tol * 1e-3;
            for (int i = l; i < n; i += kWave) U[i] = 0.0;
            for (int i = l; i < N * ns; i += kWave) sig[i] = 0.0;
            wsync();
            continue;
        }
    }
    break;
    }
    int status = kkt_stop ? CMPC_SOLVED_INACCURATE : CMPC_SOLVED;
    // polish (CMPC_FLAG_POLISH): a rescue-pass solve that stops short of tol for the last time — status 2 or
    // -2, or anything on the second (cold) pass, rescue == 2 — leaves its last iterate in the rescue image
    // with flag 2 and its best merit (mpc_polish.hip)
    const bool pol = c_arg.rescue && c.polish && stop != kStopConverged && stop != kStopNonFinite &&
                     (best_m < 1e3 * tol || stop == kStopMaxIter || c_arg.rescue == 2);
    if (pol) {
        const int ht = (int)hand_t(c);
        for (int i = l; i < n; i += kWave) hand[2 + i] = U[i];
        for (int i = l; i < N * ns; i += kWave) hand[2 + n + i] = sig[i];
        for (int r = l; r < m; r += kWave) {
            hand[ht + r] = t[r];
            hand[ht + m + r] = lam[r];
        }
        if (l == 0) {
            hand[0] = 2.0;
            hand[1] = best_m;
        }
    }
    if (stop != kStopConverged) {
        if (best_it > 0) {  // restore the best iterate
            for (int i = l; i < n; i += kWave) U[i] = bU[i];
            for (int i = l; i < N * ns; i += kWave) sig[i] = bsig[i];
            kkt = best_kkt;
        }
        // (an fp64 restart that ends with its best merit below the requested tol has met it)
        status = ((it_done || c_arg.rescue == 3) && best_m < tol_req) ? CMPC_SOLVED : stop_status(stop, best_m, tol_req);
    }
    wsync();

    // ---- output in the reference layout ----
    fwd_sim<G>(c, d, sAB, sb, x0, U, X);
    const int nxe = nx + ns;
    const size_t nz = (size_t)nxe * (N + 1) + 2 * (size_t)n;
    double* z = P.z + (size_t)b * nz;
    for (int i = l; i < (N + 1) * nxe; i += kWave) {
        const int k = i / nxe, s = i - k * nxe;
        z[i] = (s < nx) ? X[k * nx + s] : (k ? sig[(k - 1) * ns + (s - nx)] : 0.0);
    }
    for (int i = l; i < n; i += kWave) {
        const int k = i / nu, j = i - k * nu;
        z[(size_t)(N + 1) * nxe + i] = U[i];
        z[(size_t)(N + 1) * nxe + n + i] = U[i] - (k ? U[(k - 1) * nu + j] : up[j]);
    }
    if (l == 0) {
        if (P.kkt) P.kkt[b] = kkt;
        if (P.iters) P.iters[b] = it_prev + it_done + it;
        if (P.status) P.status[b] = status;
    }
    RSTAMP(14);
    if (stamp) {
        wsync();
        if (l < kStampSlots)
            P.stamps[(size_t)b * kStampSlots + l] = (l == kStampSlots - 1) ? (unsigned long long)(it_done + it) : tsum[l];
    }
#undef RSTAMP
#undef RCOUNT
}


// ---------------------------------------------------------------------------------------------------
// Latency mode: four wavefronts per agent (mpc_riccati_mw_kernel).
//
// At the reference's shipped horizon (config_LPV.py:13-24: N = 125, 3 agents) the LDS image of one agent
// is ~154 KB, so a CU holds one agent and three of its four SIMDs idle; a 3-agent step is then one serial
// wave per agent, no faster than a CPU core running the C restatement (round 5: 11.2 / 43.4 ms against
// 10.5 / 45.8 ms).  This kernel gives the agent's workgroup all four SIMDs:
//   * every per-row / per-stage item loop (rows, residual rows, th, Dsig, the stage weights W_k, the
//     right-hand sides rho / rt / C'rt, the row directions, the step bounds, the update) runs over the
//     256 threads;
//   * the residual adjoint sweep (wave 0) runs beside the Riccati factorisation (wave 1, its own stage
//     slots sb2) and the residual rows (waves 2, 3).  The factorisation's precision (double-double or
//     not) is decided in the one-wave kernel after this iteration's merit; here it is speculated from
//     the state before it ("no new best iterate") and the factorisation is redone in the rare iteration
//     where the merit says otherwise;
//   * the Newton solves (serial in the stages) run on wave 0.
// Every value is computed by the same expressions in the same order as in mpc_riccati_kernel; the sums
// that cross rows (mu, mu_aff, the neighbourhood test) are accumulated by wave 0 in the one-wave
// kernel's lane order, so the iterates are those of the one-wave kernel (GPU test
// test_riccati_latency_mode_matches_one_wave).  CMPC_FLAG_ONE_WAVE keeps the one-wave kernel.
constexpr int kMW = 4;  // wavefronts per agent

__host__ __device__ inline RLds r_layout_mw(const MpcConst& c) {
    RLds L = r_layout_ex(c, false);
    const Dims d = dims_of(c);
    L.sb2 = L.total;
    L.red = L.sb2 + 2 * d.Sl;
    L.ring = L.red + 16;
    L.total = L.ring + ((kRing * d.sF + 1) & ~1);
    return L;
}

// rt of the rows (the slack groups' Schur form of rho; mpc_riccati_kernel's loop) over nt threads
template <class G>
__device__ __forceinline__ void mw_rt(const MpcConst& c, int tid, int nt, const double* rho, const double* th,
                                      const double* rsig, const double* Dsig, double* rt) {
    constexpr int MC = G::MC;
    const int ms = c.ms, mc = MC, ns = c.ns, m = c.m;
    for (int r = tid; r < m; r += nt) {
        double v = rho[r];
        if (r < ms) {
            const int k = r / mc, rr = r - k * mc, j = c.row_slack[rr];
            if (j >= 0) {
                double rk[MC];
#pragma unroll
                for (int r2 = 0; r2 < MC; ++r2) rk[r2] = rho[k * mc + r2];
                const double q = 2.0 * c.Qs[j];
                v = q * rho[r] - th[r] * c.row_sign[rr] * rsig[k * ns + j];
#pragma unroll
                for (int r2 = 0; r2 < MC; ++r2) {
                    if (r2 == rr || c.row_slack[r2] != j) continue;
                    const int R2 = k * mc + r2;
                    v += th[R2] * rho[r] - th[r] * c.row_sign[rr] * c.row_sign[r2] * rk[r2];
                }
                v /= Dsig[k * ns + j];
            }
        }
        rt[r] = v;
    }
}

template <class G>
__global__ __launch_bounds__(kMW * kWave) void mpc_riccati_mw_kernel(const MpcConst c_arg, const MpcPtrs P) {
    static_assert(G::NX != 0 && !G::GR && !G::F32, "latency mode: fixed dimensions, rows in LDS, fp64");
    constexpr int NT = kMW * kWave;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int b = P.order ? min(max(P.order[blockIdx.x], 0), (int)gridDim.x - 1) : (int)blockIdx.x;
    if (c_arg.rescue) {  // (as mpc_riccati_kernel; the whole workgroup returns)
        const RGlb g0 = r_glb(c_arg);
        if (P.ws[(size_t)b * g0.total + g0.hand] != 1.0 && P.status[b] != CMPC_UNSOLVED) return;
    }
    const int tid = threadIdx.x, l = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const RLds L = r_layout_mw(c_arg);
    {
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&c_arg);
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(sm + L.cst);
        for (int i = tid; i < mpc_const_used_doubles(c_arg); i += NT) dst[i] = src[i];
    }
    __syncthreads();
    const MpcConst& c = *reinterpret_cast<const MpcConst*>(sm + L.cst);
    const Dims d = dims_t<G>(c);
    const RGlb gl = r_glb(c);
    constexpr int NX = G::NX, MC = G::MC;
    const int nx = NX, nu = G::NU, N = c.N, ns = c.ns, mc = MC, n = c.n, ms = c.ms, m = c.m;

    const double* __restrict__ A = P.A + (size_t)b * N * nx * nx;
    const double* __restrict__ B = P.B + (size_t)b * N * nx * nu;
    const double* __restrict__ x0 = P.x0 + (size_t)b * nx;
    const double* __restrict__ up = P.up + (size_t)b * nu;
    const double* __restrict__ pl = P.p + (size_t)b * (N + 1) * nx;
    const double* __restrict__ C = P.C + (size_t)b * N * mc * nx;
    const double* __restrict__ h = P.h + (size_t)b * N * mc;
    double* __restrict__ ws = P.ws + (size_t)b * gl.total;
    double* dta = ws + gl.dta;
    double* dla = ws + gl.dla;
    double* F = ws + gl.F;
    double* bU = ws + gl.bU;
    double* bsig = ws + gl.bsig;
    double* Wg = ws + gl.Wk;
    double* t = sm + L.t;
    double* lam = sm + L.lam;
    double* th = sm + L.th;
    double* rp = sm + L.rp;
    double* rho = sm + L.rho;
    double* rt = sm + L.rt;
    double* w = sm + L.w;
    double* GdU = sm + L.GdU;
    double* X = sm + L.X;
    double* dX = sm + L.dX;
    double* yb = sm + L.yb;
    double* yb2 = sm + L.yb2;
    double* psi = sm + L.psi;
    double* U = sm + L.U;
    double* dU = sm + L.dU;
    double* rd = sm + L.rd;
    double* gU = sm + L.gU;
    double* rh = sm + L.rh;
    double* cr = sm + L.cr;
    double* sig = sm + L.sig;
    double* dsig = sm + L.dsig;
    double* Dsig = sm + L.Dsig;
    double* rsig = sm + L.rsig;
    double* sb = sm + L.sb;
    double* red = sm + L.red;  // [0, 4): block reductions; 8..: values handed between waves
    RLds L1 = L;
    L1.sb = L.sb2;  // wave 1's stage slots: the factorisation runs beside wave 0's adjoint sweep
    const StageSrc sAB{A, B, B, d.sA, d.sB, d.sF, 0};

    // block reductions (max / min are order-free; the cross-row SUMS are wave 0's, below)
    auto bred = [&](double v, int op) __attribute__((always_inline)) -> double {
        v = op == 0 ? wave_max(v) : wave_min(v);
        if (l == 0) red[wv] = v;
        __syncthreads();
        double r = red[0];
        for (int q = 1; q < kMW; ++q) r = op == 0 ? nmax(r, red[q]) : fmin(r, red[q]);
        __syncthreads();
        return r;
    };
    // a value of wave 0 to every thread
    auto from0 = [&](double v, int slot) __attribute__((always_inline)) -> double {
        if (wv == 0 && l == 0) red[slot] = v;
        __syncthreads();
        const double r = red[slot];
        __syncthreads();
        return r;
    };

    for (int i = tid; i < L.cst; i += NT) sm[i] = 0.0;
    __syncthreads();
    double* hand = ws + gl.hand;
    const bool warm = c_arg.rescue && hand[0] == 1.0;
    bool dd_on = warm;
    const int it0 = warm ? (int)hand[1] : 0;
    if (warm) {
        for (int i = tid; i < n; i += NT) U[i] = hand[2 + i];
        for (int i = tid; i < N * ns; i += NT) sig[i] = hand[2 + n + i];
    }
    __syncthreads();
    // per-section clocks (wave 0's view; the overlapped residual / factor phase is slot 0, a redone
    // factorisation slot 2 / 3)
    const bool stamp = P.stamps != nullptr;
    unsigned long long* tsum = reinterpret_cast<unsigned long long*>(sm + L.stamps);
    unsigned long long t_a = stamp ? clock64_() : 0, t_b = 0;
#define MSTAMP(slot)                                    \
    if (stamp && wv == 0) {                             \
        t_b = clock64_();                               \
        if (l == 0) tsum[slot] += t_b - t_a;            \
        t_a = t_b;                                      \
    }
#define MCOUNT(slot) \
    if (stamp && tid == 0) tsum[slot] += 1;

    for (int r = tid; r < m; r += NT) {
        double v;
        if (r < ms) {
            v = h[r];
        } else {
            const int q = r - ms, i = (q >> 1) % nu;
            v = (q & 1) ? -c.u_lb[i] : c.u_ub[i];
        }
        w[r] = isfinite(v) ? v : INFINITY;
    }
    __syncthreads();
    if (wv == 0) fwd_sim<G>(c, d, sAB, sb, x0, U, X);
    __syncthreads();
    double mact_l = 0.0, sp_l = 1.0;
    const size_t ht = hand_t(c);
    for (int r = tid; r < m; r += NT) {
        if (isfinite(w[r])) {
            if (warm) {
                t[r] = hand[ht + r];
                lam[r] = hand[ht + m + r];
            } else {
                const double g = row_value<G>(c, C, r, X, U, sig);
                t[r] = fmax(w[r] - g, kT0Floor);
                lam[r] = 1.0;
            }
            mact_l += 1.0;
            sp_l = fmax(sp_l, fabs(w[r]));
        } else {
            t[r] = 1.0;
            lam[r] = 0.0;
        }
    }
    // the active-row count: integer-valued, exact in any order
    const double mact_w = wave_sum(mact_l);  // (every lane: a cross-lane sum)
    if (l == 0) red[4 + wv] = mact_w;
    __syncthreads();
    const double mact = fmax(red[4] + red[5] + red[6] + red[7], 1.0);
    const double scale_p = bred(sp_l, 0);  // (its barriers: every thread has read `warm` and the rows)
    if (warm && tid == 0) hand[0] = 0.0;
    if (tid == 0) red[15] = 0.0;  // a timed-out wait between the waves

    double best_m = INFINITY, best_kkt = INFINITY;
    int best_it = 0, stop = kStopMaxIter, it;
    double kkt = INFINITY;
    MSTAMP(14);
    double alpha_prev = 1;
    bool hp = false;
    for (it = it0 + 1; it <= c.max_iter; ++it) {
        // ---- item phases (all waves): the residual adjoints' right-hand sides, th, the residual rows, Dsig,
        // the stage weights W_k, and the predictor's right-hand side (rho, rt, C'rt: they need only the
        // iterate, so wave 2 can run its backward pass beside the factorisation) ----
        if (tid == 0) red[12] = red[13] = red[14] = 0.0;  // progress: factorisation, adjoint sweep, piped pass
        for (int i = tid; i < (N + 1) * nx; i += NT) {
            const int k = i / nx, s = i - k * nx;
            double v = 2.0 * pl[i];
            for (int u = 0; u < nx; ++u) v = fma(2.0 * c.Q[s * nx + u], X[k * nx + u], v);
            yb[i] = v;
        }
        for (int r = tid; r < m; r += NT) {
            th[r] = isfinite(w[r]) ? lam[r] / t[r] : 0.0;
            rp[r] = isfinite(w[r]) ? row_value<G>(c, C, r, X, U, sig) + t[r] - w[r] : 0.0;
        }
        for (int i = tid; i < N * ns; i += NT) {
            const int k = i / ns, j = i - k * ns;
            double v = 2.0 * c.Qs[j] * sig[i];
            for (int r = 0; r < mc; ++r)
                if (c.row_slack[r] == j) v += c.row_sign[r] * lam[k * mc + r];
            rsig[i] = v;
        }
        __syncthreads();
        for (int i = tid; i < (N + 1) * nx; i += NT) {
            const int k = i / nx, s = i - k * nx;
            double v = 0.0;
            if (k > 0)
                for (int r = 0; r < mc; ++r) v = fma(lam[(k - 1) * mc + r], C[((size_t)(k - 1) * mc + r) * nx + s], v);
            yb2[i] = k > 0 ? yb[i] + v : yb[i];
        }
        for (int i = tid; i < N * ns; i += NT) {
            const int k = i / ns, j = i - k * ns;
            double v = 2.0 * c.Qs[j];
            for (int r = 0; r < mc; ++r)
                if (c.row_slack[r] == j) v += th[k * mc + r];
            Dsig[i] = v;
        }
        for (int r = tid; r < m; r += NT) {  // pass 0's rho (the one-wave kernel's statements)
            if (!isfinite(w[r])) {
                rho[r] = 0.0;
                continue;
            }
            double rc = -t[r] * lam[r];
            rho[r] = (rc + lam[r] * rp[r]) / t[r];
        }
        __syncthreads();
        stage_weights<G>(c, L, sm, C, Wg, tid, NT);
        double thm_l = 0.0;
        for (int r = tid; r < m; r += NT) thm_l = fmax(thm_l, th[r]);
        mw_rt<G>(c, tid, NT, rho, th, rsig, Dsig, rt);
        gsync();  // W_k (global): stored here by every wave, read by wave 1's factorisation
        const bool above = bred(thm_l, 0) > kDdTh;
        double* ybC = dX;  // pass 0's C'rt (dX is free until pass 0's forward pass writes it)
        for (int i = tid; i < (N + 1) * nx; i += NT) {
            const int k = i / nx, s = i - k * nx;
            double v = 0.0;
            if (k > 0)
                for (int r = 0; r < mc; ++r) v = fma(rt[(k - 1) * mc + r], C[((size_t)(k - 1) * mc + r) * nx + s], v);
            ybC[i] = v;
        }
        __syncthreads();
        // ---- wave 0: both residual adjoints; wave 1: the factorisation (speculative precision); wave 2
        // (fp64 guess): the predictor's backward pass, stage by stage behind them ----
        const bool hp_spec = above && (dd_on || it - best_it >= kDdStall);
#ifdef RIC_MW_NOPIPE  // lab: no backward pass beside the factorisation
        const bool piped = false;
#else
        const bool piped = !hp_spec;
#endif
        MSTAMP(1);  // (slot 1: the item phases before the waves' roles)
        const unsigned long long t_role = stamp ? clock64_() : 0;
        auto factor = [&](bool hp_want, bool ring_on) __attribute__((always_inline)) {
            bool ok = hp_want ? riccati_factor_dd<G>(c, d, L1, sm, A, B, Wg, F)
                              : riccati_factor<G>(c, d, L1, sm, A, B, Wg, F, nullptr, ring_on ? sm + L.ring : nullptr,
                                                  red + 12, red + 14, red + 15);
            bool hp_f = hp_want;
            if (!ok && !hp_want && above) {  // fp64 breakdown above the threshold: double-double (as the one-wave kernel)
                gsync();
                hp_f = true;
                ok = riccati_factor_dd<G>(c, d, L1, sm, A, B, Wg, F);
            }
            gsync();  // the gains F (global), read by wave 0's solves
            if (l == 0) {
                red[8] = ok ? 1.0 : 0.0;
                red[9] = hp_f ? 1.0 : 0.0;
            }
        };
        if (wv == 0) {
            adjoint2<G>(c, d, sAB, sb, yb, gU, yb2, rd, sm + L.psid, red + 13);
        } else if (wv == 1) {
            factor(hp_spec, piped);
        } else if (wv == 2 && piped) {
            if (!riccati_back_piped<G>(c, A, B, sm + L.ring, d.sF, red + 12, red + 13, red + 14, ybC, rd, rt, lam, U, up,
                                       sm + L.pv, dU, ms) && l == 0)
                red[15] = 1.0;
        }
        if (stamp && l == 0 && wv < 3) tsum[9 + wv] += clock64_() - t_role;  // slots 9-11: each role's own clocks
        __syncthreads();
        double gs_l = 1.0, nrd_l = 0.0, nrs_l = 0.0, nrp_l = 0.0;
        for (int i = tid; i < n; i += NT) {
            gU[i] += rdr_grad<G>(c, U, up, i);
            gs_l = nmax(gs_l, fabs(gU[i]));
            const int r = ms + 2 * i;
            rd[i] += rdr_grad<G>(c, U, up, i) + lam[r] - lam[r + 1];
            nrd_l = nmax(nrd_l, fabs(rd[i]));
        }
        for (int i = tid; i < N * ns; i += NT) nrs_l = nmax(nrs_l, fabs(rsig[i]));
        for (int r = tid; r < m; r += NT)
            if (isfinite(w[r])) nrp_l = nmax(nrp_l, fabs(rp[r]));
        double mu_l = 0.0;  // wave 0, in the one-wave kernel's lane order
        if (wv == 0)
            for (int r = l; r < m; r += kWave)
                if (isfinite(w[r])) mu_l += t[r] * lam[r];
        const double mu = from0(wave_sum(mu_l) / mact, 10);
        const double gscale = bred(gs_l, 0);
        const double nrd = bred(nrd_l, 0), nrs = bred(nrs_l, 0), nrp = bred(nrp_l, 0);
        const double res = nmax(nmax(nrd / gscale, nrs / c.qs_max), nrp / scale_p);
        kkt = nmax(res, mu);
        const double merit = nmax(res, 1e4 * mu);
        if (!isfinite(merit)) {
            stop = kStopNonFinite;
            break;
        }
        if (red[15] != 0.0) {  // a wait between the waves timed out (never expected): give the agent up
            stop = kStopBreakdown;
            break;
        }
        if (merit < best_m) {
            best_m = merit;
            best_kkt = kkt;
            best_it = it;
            for (int i = tid; i < n; i += NT) bU[i] = U[i];
            for (int i = tid; i < N * ns; i += NT) bsig[i] = sig[i];
        }
        if (merit < c.tol) {
            stop = kStopConverged;
            break;
        }
        if (best_m < 1e3 * c.tol && it - best_it >= kStallIters) {
            stop = kStopStalled;
            break;
        }
        if (warm && it - best_it >= kWarmStall) {
            stop = kStopStalled;
            break;
        }
        // the precision the one-wave kernel picks now (this iteration's best_it); redo on a miss
        if (!dd_on && it - best_it >= kDdStall) dd_on = true;
        hp = above && dd_on;
        MSTAMP(0);
        if (hp != hp_spec) {
            if (wv == 1) factor(hp, false);
            __syncthreads();
        }
        const bool fact_ok = red[8] != 0.0;
        if (red[9] != 0.0 && !hp) dd_on = hp = true;
        __syncthreads();  // (red[8], red[9] read by every thread before the next writes)
        if (!fact_ok) {
            stop = kStopBreakdown;
            break;
        }
        MSTAMP(hp ? 3 : 2);
        if (hp) MCOUNT(12);

        // ================= predictor / corrector =================
        double sig_c = 0.0, alpha = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            if (pass) {  // (pass 0's rho, rt and C'rt were formed before the factorisation)
                for (int r = tid; r < m; r += NT) {
                    if (!isfinite(w[r])) {
                        rho[r] = 0.0;
                        continue;
                    }
                    double rc = -t[r] * lam[r];
                    rc += sig_c * mu - dta[r] * dla[r];
                    rho[r] = (rc + lam[r] * rp[r]) / t[r];
                }
                __syncthreads();
                mw_rt<G>(c, tid, NT, rho, th, rsig, Dsig, rt);
                __syncthreads();
                for (int i = tid; i < (N + 1) * nx; i += NT) {
                    const int k = i / nx, s = i - k * nx;
                    double v = 0.0;
                    if (k > 0)
                        for (int r = 0; r < mc; ++r) v = fma(rt[(k - 1) * mc + r], C[((size_t)(k - 1) * mc + r) * nx + s], v);
                    yb[i] = v;
                }
                __syncthreads();
            }
            const double* yrt = pass ? yb : ybC;
            MSTAMP(4);
            if (wv == 0) {  // the Newton solve: serial in the stages
                if (!hp) {  // (pass 0 with wave 2's backward pass: the forward pass only)
                    riccati_solve<G>(c, d, L, sm, A, B, F, nullptr, dU, dX, yrt, rd, rt, (!pass && piped) ? 2 : 3);
                } else {
                    adjoint<G>(c, d, sAB, sb, yrt, rh, psi);
                    for (int i = l; i < n; i += kWave) rh[i] = -rd[i] - (rh[i] + rt[ms + 2 * i] - rt[ms + 2 * i + 1]);
                    wsync();
                    riccati_solve<G>(c, d, L, sm, A, B, F, rh, dU, dX);
                    const int nref = warm ? kRefineMaxWarm : kRefineMax;
                    for (int ir = 0; ir < nref; ++ir) {
                        kres_dd<G>(c, d, L, sm, A, B, Wg, dU, rh, gU);
                        riccati_solve<G>(c, d, L, sm, A, B, F, gU, cr, nullptr);
                        double cn_l = 0.0, un_l = 0.0;
                        for (int i = l; i < n; i += kWave) {
                            const double u = dU[i] + cr[i];
                            dU[i] = u;
                            cn_l = nmax(cn_l, fabs(cr[i]));
                            un_l = fmax(un_l, fabs(u));
                        }
                        const double cn = wave_max(cn_l), un = wave_max(un_l);
                        wsync();
                        MCOUNT(13);
                        if (!(cn > kRefineTol * un)) break;
                    }
                    fwd_sim<G>(c, d, sAB, sb, nullptr, dU, dX);
                }
            }
            __syncthreads();
            MSTAMP(hp ? 6 : 5);
            for (int r = tid; r < m; r += NT) GdU[r] = row_value<G>(c, C, r, dX, dU, nullptr);
            __syncthreads();
            for (int i = tid; i < N * ns; i += NT) {
                const int k = i / ns, j = i - k * ns;
                double v = rsig[i];
#pragma unroll
                for (int r = 0; r < MC; ++r)
                    if (c.row_slack[r] == j) {
                        const int R1 = k * mc + r;
                        v += c.row_sign[r] * (rho[R1] + th[R1] * GdU[R1]);
                    }
                dsig[i] = -v / Dsig[i];
            }
            __syncthreads();
            double amax_l = 1.0e300;
            double* dtp = pass ? rho : dta;  // corrector reuses rho/rt storage for (dt, dl)
            double* dlp = pass ? rt : dla;
            for (int r = tid; r < m; r += NT) {
                if (!isfinite(w[r])) {
                    dtp[r] = 0.0;
                    dlp[r] = 0.0;
                    continue;
                }
                double sd = 0.0;
                if (r < ms) {
                    const int k = r / mc, rr = r - k * mc, j = c.row_slack[rr];
                    if (j >= 0) sd = c.row_sign[rr] * dsig[k * ns + j];
                }
                const double rho_r = rho[r];
                const double dtv = -rp[r] - GdU[r] - sd;
                const double dlv = rho_r + th[r] * (GdU[r] + sd);
                dtp[r] = dtv;
                dlp[r] = dlv;
                if (dtv < 0.0) amax_l = fmin(amax_l, -t[r] / dtv);
                if (dlv < 0.0) amax_l = fmin(amax_l, -lam[r] / dlv);
            }
            gsync();  // (dta, dla: global)
            const double amax = fmin(bred(amax_l, 1), 1.0e300);
            if (!pass) {
                const double a = fmin(amax, 1.0);
                double mua_l = 0.0;
                if (wv == 0)
                    for (int r = l; r < m; r += kWave)
                        if (isfinite(w[r])) mua_l += (t[r] + a * dta[r]) * (lam[r] + a * dla[r]);
                const double mu_aff = from0(wave_sum(mua_l) / mact, 11);
                const double ratio = mu > 0.0 ? mu_aff / mu : 0.0;
                sig_c = warm ? ratio * ratio : ratio * ratio * ratio;
                if (alpha_prev < kShortStep) sig_c = fmax(sig_c, kSigmaMin);
            } else {
                alpha = fmin(1.0, 0.995 * amax);
                if (wv == 0) {  // the neighbourhood backtracking, in the one-wave kernel's order
                    for (int bt = 0; bt < kMaxBacktrack; ++bt) {
                        double mn_l = 0.0, pm_l = INFINITY;
                        for (int r = l; r < m; r += kWave)
                            if (isfinite(w[r])) {
                                const double pr = (t[r] + alpha * rho[r]) * (lam[r] + alpha * rt[r]);
                                mn_l += pr;
                                pm_l = fmin(pm_l, pr);
                            }
                        if (wave_min(pm_l) >= kNbhdGamma * (wave_sum(mn_l) / mact)) break;
                        alpha *= 0.8;
                    }
                }
                alpha = from0(alpha, 12);
            }
            MSTAMP(7);
        }
        alpha_prev = alpha;
        for (int i = tid; i < n; i += NT) U[i] = fma(alpha, dU[i], U[i]);
        for (int i = tid; i < N * ns; i += NT) sig[i] = fma(alpha, dsig[i], sig[i]);
        for (int i = tid; i < (N + 1) * nx; i += NT) X[i] = fma(alpha, dX[i], X[i]);
        for (int r = tid; r < m; r += NT)
            if (isfinite(w[r])) {
                t[r] = fma(alpha, rho[r], t[r]);
                lam[r] = fma(alpha, rt[r], lam[r]);
            }
        __syncthreads();
        MSTAMP(8);
    }
    if (it > c.max_iter) it = c.max_iter;
    gsync();
    __syncthreads();
    int status = CMPC_SOLVED;
    const bool pol = c_arg.rescue && c.polish && stop != kStopConverged && stop != kStopNonFinite &&
                     (best_m < 1e3 * c.tol || stop == kStopMaxIter || c_arg.rescue == 2);
    if (pol) {
        const int ht2 = (int)hand_t(c);
        for (int i = tid; i < n; i += NT) hand[2 + i] = U[i];
        for (int i = tid; i < N * ns; i += NT) hand[2 + n + i] = sig[i];
        for (int r = tid; r < m; r += NT) {
            hand[ht2 + r] = t[r];
            hand[ht2 + m + r] = lam[r];
        }
        if (tid == 0) {
            hand[0] = 2.0;
            hand[1] = best_m;
        }
    }
    __syncthreads();
    if (stop != kStopConverged) {
        if (best_it > 0) {  // restore the best iterate
            for (int i = tid; i < n; i += NT) U[i] = bU[i];
            for (int i = tid; i < N * ns; i += NT) sig[i] = bsig[i];
            kkt = best_kkt;
        }
        status = stop_status(stop, best_m, c.tol);
    }
    __syncthreads();
    if (wv == 0) fwd_sim<G>(c, d, sAB, sb, x0, U, X);
    __syncthreads();
    const int nxe = nx + ns;
    const size_t nz = (size_t)nxe * (N + 1) + 2 * (size_t)n;
    double* z = P.z + (size_t)b * nz;
    for (int i = tid; i < (N + 1) * nxe; i += NT) {
        const int k = i / nxe, s = i - k * nxe;
        z[i] = (s < nx) ? X[k * nx + s] : (k ? sig[(k - 1) * ns + (s - nx)] : 0.0);
    }
    for (int i = tid; i < n; i += NT) {
        const int k = i / nu, j = i - k * nu;
        z[(size_t)(N + 1) * nxe + i] = U[i];
        z[(size_t)(N + 1) * nxe + n + i] = U[i] - (k ? U[(k - 1) * nu + j] : up[j]);
    }
    if (tid == 0) {
        if (P.kkt) P.kkt[b] = kkt;
        if (P.iters) P.iters[b] = it;
        if (P.status) P.status[b] = status;
    }
    MSTAMP(14);
    if (stamp) {
        __syncthreads();
        if (tid < kStampSlots) P.stamps[(size_t)b * kStampSlots + tid] = (tid == kStampSlots - 1) ? (unsigned long long)it : tsum[tid];
    }
#undef MSTAMP
#undef MCOUNT
}

}  // namespace

bool mpc_riccati_f32_supported(const MpcConst& c) { return c.nx == 6 && c.nu == 3 && c.mc == 6; }

size_t mpc_riccati_lds_bytes(const MpcConst& c) {
    return sizeof(double) * (size_t)(mpc_riccati_mw(c) ? r_layout_mw(c) : r_layout(c)).total;
}

// The latency mode (mpc_riccati_mw_kernel) where it applies: the PlannerLPV agent with two neighbours
// (nx 9, nu 2, 6 rows per stage: the reference's shipped N = 125), fp64, an LDS image that leaves a CU
// to one agent (over half of it: three SIMDs of the CU would idle), unless CMPC_FLAG_ONE_WAVE.
bool mpc_riccati_mw(const MpcConst& c) {
    if (c.f32 || c.waves == 1 || !(c.nx == 9 && c.nu == 2 && c.mc == 6) || r_rows_global(c)) return false;
    const size_t one = sizeof(double) * (size_t)r_layout(c).total, mw = sizeof(double) * (size_t)r_layout_mw(c).total;
    return 2 * one > kMaxLdsBytes && mw <= kMaxLdsBytes;
}

size_t mpc_riccati_ws_doubles(const MpcConst& c) { return r_glb(c).total; }

hipError_t mpc_riccati_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    if (!p.ws) return hipErrorInvalidValue;
    const size_t lds = mpc_riccati_lds_bytes(c);
    const Dims d = dims_of(c);
    const bool small = d.S <= kPerSmall * kWave;
    // instantiations: the PlannerLPV agent (nx 9, nu 2, 4 + nb rows per stage), the synthetic
    // double integrator (nx 4, nu 2; the 3-D one of cfg5: nx 6, nu 3, nb 2), runtime dimensions
    auto go = [&](auto g) -> hipError_t {
        using G = decltype(g);
        hipError_t e = hipFuncSetAttribute((const void*)mpc_riccati_kernel<G>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(mpc_riccati_kernel<G>, dim3(batch), dim3(kWave), lds, s, c, p);
        return hipSuccess;
    };
    hipError_t e;
    if (mpc_riccati_mw(c)) {  // the latency mode: four wavefronts per agent
        using G = Cfg<kPerSmall, 9, 2, 6>;
        e = hipFuncSetAttribute((const void*)mpc_riccati_mw_kernel<G>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(mpc_riccati_mw_kernel<G>, dim3(batch), dim3(kMW * kWave), lds, s, c, p);
        return hipGetLastError();
    }
#ifdef RIC_LAB_ONLY_MW  // lab builds: the latency-mode kernel alone (a fast compile)
    (void)small;
    return hipErrorInvalidValue;
#else
    if (c.f32) {  // BASELINE cfg5's fp32 path (mpc_riccati_f32_supported)
        if (!mpc_riccati_f32_supported(c)) return hipErrorInvalidValue;
        e = r_rows_global(c) ? go(Cfg<kPerSmall, 6, 3, 6, true, true>{}) : go(Cfg<kPerSmall, 6, 3, 6, false, true>{});
    } else if (c.nx == 9 && c.nu == 2 && c.mc == 5) e = go(Cfg<kPerSmall, 9, 2, 5>{});
    else if (c.nx == 9 && c.nu == 2 && c.mc == 6) e = go(Cfg<kPerSmall, 9, 2, 6>{});
    else if (c.nx == 9 && c.nu == 2 && c.mc == 7) e = go(Cfg<kPerSmall, 9, 2, 7>{});
    else if (c.nx == 4 && c.nu == 2) e = go(Cfg<kPerSmall, 4, 2, 0>{});
    else if (c.nx == 6 && c.nu == 3 && c.mc == 6)   // BASELINE cfg5
        e = r_rows_global(c) ? go(Cfg<kPerSmall, 6, 3, 6, true>{}) : go(Cfg<kPerSmall, 6, 3, 6>{});
    else if (small) e = go(Cfg<kPerSmall, 0, 0, 0>{});
    else e = go(Cfg<kPerMax, 0, 0, 0>{});
#endif
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

}  // namespace cmpc
