// Lane-per-agent solver body (mpc_lane.hip): included by the kernel and by the host check
// tools/lane_cpu.cpp.
#pragma once
#include <cmath>
#ifdef LANE_TRACE
#include <cstdio>
#endif

#include "internal.h"

namespace cmpc {

namespace {

constexpr int kF32Stall = 2;  // fp32 iterations without a new best iterate before an agent goes fp64

// Lane-interleaved view, in PAIRS: elements 2p and 2p+1 of agent b sit side by side at double
// index (p * batch + b) * 2 (+1) of the scratch (floats in quads: (q * batch + b) * 4 + w), so that
// one 16-byte load per lane brings two elements of that lane's OWN agent — the stage images below
// are filled per lane, and a lane whose agent has converged (inactive) does not leave a hole in
// another agent's image.  On the device every access is a raw buffer load / store whose element
// offset is a wave-uniform SGPR and whose lane offset (b * 16 bytes) is one VGPR for all arrays; on
// the host (tools/lane_cpu.cpp) a pointer.  Accesses go through a small proxy (read / assign).
template <class T>
struct LV {
    static constexpr unsigned G = 16 / sizeof(T);  // elements per 16-byte group
#if defined(__HIP_DEVICE_COMPILE__)
    __amdgpu_buffer_rsrc_t r;
    unsigned base, s, vo;  // region start (elements of T, a multiple of G), batch, lane byte offset b * 16
    __device__ __forceinline__ int soff(int i) const {
        const unsigned a = base + (unsigned)i;
        return (int)((a / G) * s * 16u + (a % G) * (unsigned)sizeof(T));
    }
    __device__ __forceinline__ T ld(int i) const {
        if constexpr (sizeof(T) == 8)
            return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, (int)vo, soff(i), 0));
        else
            return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, (int)vo, soff(i), 0));
    }
    __device__ __forceinline__ void st(int i, T v) const {
        if constexpr (sizeof(T) == 8)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), r,
                                                  (int)vo, soff(i), 0);
        else
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)vo, soff(i), 0);
    }
#else
    T* p;        // the region's group 0 of agent b
    size_t s;    // batch
    size_t idx(int i) const { return ((size_t)i / G) * s * G + (size_t)i % G; }
    T ld(int i) const { return p[idx(i)]; }
    void st(int i, T v) const { p[idx(i)] = v; }
#endif
    struct Ref {
        const LV* v;
        int i;
        __host__ __device__ __forceinline__ operator T() const { return v->ld(i); }
        __host__ __device__ __forceinline__ const Ref& operator=(T x) const {
            v->st(i, x);
            return *this;
        }
        __host__ __device__ __forceinline__ const Ref& operator=(const Ref& o) const {
            v->st(i, (T)o);
            return *this;
        }
    };
    __host__ __device__ __forceinline__ Ref operator[](int i) const { return Ref{this, i}; }
};

struct LaneLayout {
    size_t X, U, sig, t, lam, bU, bsig, rd, dUp, Fd, dta, dla, dU, dX, dsig, dt, dl, Ff;
    size_t iA, iB, iC, ih, ip;  // the inputs, pair-interleaved by lane_pack (mpc_lane.hip)
    size_t total;
    int nup, nsp;               // per-stage strides of the input-like (U, dU, rd, dUp) and slack arrays
};

__host__ __device__ constexpr int lane_ev(int x) { return (x + 1) & ~1; }

__host__ __device__ inline LaneLayout lane_layout(const MpcConst& c) {
    LaneLayout L;
    const size_t N = c.N, nx = c.nx, nu = c.nu, m = c.m;
    const size_t nup = lane_ev(c.nu), nsp = lane_ev(c.ns);
    L.nup = (int)nup;
    L.nsp = (int)nsp;
    const size_t sF = nu * (nx + nu) + nu * nu;
    size_t o = 0;
    auto take = [&](size_t cnt) {  // regions start on a pair
        const size_t r = o;
        o += (cnt + 1) & ~(size_t)1;
        return r;
    };
    L.X = take((N + 1) * nx);
    L.U = take(N * nup);
    L.sig = take(N * nsp);
    L.t = take(m);
    L.lam = take(m);
    L.bU = take(N * nup);
    L.bsig = take(N * nsp);
    L.rd = take(N * nup);
    L.dUp = take(N * nup);
    L.Fd = take(N * sF);
    L.dta = take(m);
    L.dla = take(m);
    L.dU = take(N * nup);
    L.dX = take((N + 1) * nx);
    L.dsig = take(N * nsp);
    L.dt = take(m);
    L.dl = take(m);
    L.Ff = take((N * sF + 3) / 4 * 2);  // floats, in quads (Ff * 2 is a multiple of 4)
    L.iA = take(N * nx * nx);
    L.iB = take(N * nx * nu);
    L.iC = take(N * c.mc * nx);
    L.ih = take(N * c.mc);
    L.ip = take((N + 1) * nx);
    L.total = o;
    return L;
}

// NaN-propagating max (a NaN residual must never look converged)
__host__ __device__ inline double lane_nmax(double a, double b) { return (a > b || a != a) ? a : b; }

// scheduling fence between the phases of a stage (keeps the compiler from hoisting one phase's loads
// into the previous phase, which multiplies the live registers); nothing on the host
#if defined(__HIP_DEVICE_COMPILE__)
#define LANE_PHASE() __builtin_amdgcn_sched_barrier(0)
#else
#define LANE_PHASE() ((void)0)
#endif

// packed lower-triangle index (i >= j) and its symmetric accessor
__host__ __device__ constexpr int sy(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// Stage images.  Every sweep step reads its stage's data (inputs, iterate, direction, gains) from an
// LDS image that the step before filled with buffer_load ... lds (no VGPRs, the load latency hidden
// behind a whole step of arithmetic): two images, ping-pong.  A wavefront serves kLaneAP agents
// (the other 32 lanes exit at once): an image row is one element for those agents, 256 bytes, and
// one dwordx4 LDS load of 32 lanes fills two rows.  The map below (rows; runs start on even rows,
// float runs on multiples of 4 float rows) is the union of what the sweeps fetch.
constexpr int kLaneAP = 32;  // agents per wavefront (measured at 8192 agents: 32 -> 106 ms, 8 -> 129 ms, 4 -> 208 ms)

template <int NX, int NU, int MC, int NS>
struct IMap {
    static constexpr int SF = NU * (NX + NU) + NU * NU;
    static constexpr int ev(int x) { return (x + 1) & ~1; }
    static constexpr int A = 0, B = A + ev(NX * NX), C = B + ev(NX * NU), h = C + ev(MC * NX), p = h + ev(MC);
    static constexpr int X = p + ev(NX), U = X + ev(NX), sig = U + ev(NU), tB = sig + ev(NS), lB = tB + ev(MC);
    static_assert(NX % 2 == 0 && MC % 2 == 0 && SF % 4 == 0, "pair layout: even NX, MC; SF a multiple of 4");
    static constexpr int tI = lB + ev(MC), lI = tI + ev(2 * NU), dX = lI + ev(2 * NU), dsig = dX + ev(NX);
    static constexpr int dtB = dsig + ev(NS), dlB = dtB + ev(MC), dU = dlB + ev(MC), dtI = dU + ev(NU);
    static constexpr int dlI = dtI + ev(2 * NU), rd = dlI + ev(2 * NU), dUp = rd + ev(NU), aB = dUp + ev(NU);
    static constexpr int alB = aB + ev(MC), aI = alB + ev(MC), alI = aI + ev(2 * NU), Fd = alI + ev(2 * NU);
    static constexpr int rows = Fd + ev(SF);
    static constexpr int frows = (SF + 3) & ~3;                     // fp32 gains
    static constexpr int bytes = rows * kLaneAP * 8 + frows * kLaneAP * 4;  // one image
};

// Residual and factorisation accumulators of one S1 sweep.
struct S1Out {
    double gsc, nrd, nrs, nrp, mu;
    bool broke;
};

}  // namespace

// One agent's solve (lane j = b % kLaneAP of its wavefront).  __host__ __device__: the kernel runs it
// per lane; tools/lane_cpu.cpp runs the same code on the host (images emulated per agent) to check it
// against the C restatement.  `smem`: the two stage images of this wavefront (device).  `b` is the
// agent's slot in the packed scratch; `ag` (default: b) its index in the caller's arrays (x0, u_prev
// and the outputs): they differ under a launch order (cmpc_opts.order, packed by lane_pack).
template <int NX, int NU, int MC, int NS, bool MIXED>
__host__ __device__ inline void lane_agent(const MpcConst& c, const MpcPtrs& P, int batch, int b, char* smem,
                                           int ag = -1) {
    const size_t a_ = (size_t)(ag < 0 ? b : ag);
    using M = IMap<NX, NU, MC, NS>;
    constexpr int NA = NX + NU, SF = M::SF;
    constexpr int NUP = lane_ev(NU), NSP = lane_ev(NS);  // per-stage strides of U-like / slack arrays
    const int N = c.N, ms = c.ms, m = c.m;
    const LaneLayout L = lane_layout(c);
    const size_t S = (size_t)batch;
    double* ws = P.ws;
    const int j = b % kLaneAP;  // lane within the wavefront's agents
#if defined(__HIP_DEVICE_COMPILE__)
    // one buffer resource over the launch's scratch (mpc_lane_launch splits batches whose scratch
    // would reach 2 GiB into sub-launches, so the 32-bit offsets never wrap)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(ws, 0, (int)(L.total * S * 8 < 0x7fffffffull ? L.total * S * 8 : 0x7fffffffull),
                                          0x00020000);
    const unsigned Su = (unsigned)S;
    auto mk = [&](size_t region) { return LV<double>{rs, (unsigned)region, Su, (unsigned)b * 16u}; };
    const LV<float> Ff{rs, (unsigned)(2 * L.Ff), Su, (unsigned)b * 16u};  // float elements from float index 2 * Ff
    // image fills: per lane 16 bytes of its own agent (a pair of double rows / a quad of float rows)
    const int vo = (int)((unsigned)b * 16u);
    auto fd = [&](int buf, int row, size_t ge, int cnt) {  // ge, row even
        char* dst = smem + buf * M::bytes + (row >> 1) * (kLaneAP * 16);
        for (int q = 0; q < cnt; q += 2)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + (q >> 1) * (kLaneAP * 16)),
                                                     16, vo, (int)((ge + q) / 2 * Su * 16u), 0, 0);
    };
    auto ff = [&](int buf, size_t gf, int cnt) {  // gf a multiple of 4
        char* dst = smem + buf * M::bytes + M::rows * (kLaneAP * 8);
        for (int q = 0; q < cnt; q += 4)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + (q >> 2) * (kLaneAP * 16)),
                                                     16, vo, (int)((gf + q) / 4 * Su * 16u), 0, 0);
    };
    const double* imd0 = reinterpret_cast<const double*>(smem);
    auto im = [&](int buf, int row) -> double {
        return imd0[buf * (M::bytes / 8) + (row >> 1) * (2 * kLaneAP) + 2 * j + (row & 1)];
    };
    auto imf = [&](int buf, int row) -> float {
        return reinterpret_cast<const float*>(smem + buf * M::bytes + M::rows * (kLaneAP * 8))[(row >> 2) * (4 * kLaneAP) +
                                                                                               4 * j + (row & 3)];
    };
    // every image fill (and store) of this wavefront retired and every LDS read of the image done; a
    // compiler memory barrier too, so no image read moves above it (the LDS-DMA writes are invisible
    // to the compiler's dependence tracking)
    auto img_wait = [&]() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); };
#else
    (void)smem;
    auto mk = [&](size_t region) { return LV<double>{ws + region * S + 2 * (size_t)b, S}; };
    const LV<float> Ff{reinterpret_cast<float*>(ws + L.Ff * S) + 4 * (size_t)b, S};
    double hd[2][M::rows];
    float hf[2][M::frows];
    auto fd = [&](int buf, int row, size_t ge, int cnt) {
        const LV<double> v{ws + 2 * (size_t)b, S};
        for (int q = 0; q < cnt; ++q) hd[buf][row + q] = v.ld((int)(ge + q));
    };
    auto ff = [&](int buf, size_t gf, int cnt) {
        const LV<float> v{reinterpret_cast<float*>(ws) + 4 * (size_t)b, S};
        for (int q = 0; q < cnt; ++q) hf[buf][q] = v.ld((int)(gf + q));
    };
    auto im = [&](int buf, int row) -> double { return hd[buf][row]; };
    auto imf = [&](int buf, int row) -> float { return hf[buf][row]; };
    auto img_wait = [&]() {};
#endif
    (void)j;
    const LV<double> X = mk(L.X), U = mk(L.U), sig = mk(L.sig), t = mk(L.t), lam = mk(L.lam), bU = mk(L.bU);
    const LV<double> bsig = mk(L.bsig), rd = mk(L.rd), dUp = mk(L.dUp), Fd = mk(L.Fd), dta = mk(L.dta);
    const LV<double> dla = mk(L.dla), dU = mk(L.dU), dX = mk(L.dX), dsig = mk(L.dsig), dt = mk(L.dt), dl = mk(L.dl);
    const LV<double> gA = mk(L.iA), gB = mk(L.iB), gC = mk(L.iC), gh = mk(L.ih);
    double x0[NX], up[NU];
#pragma unroll
    for (int s = 0; s < NX; ++s) x0[s] = P.x0[a_ * NX + s];
#pragma unroll
    for (int i = 0; i < NU; ++i) up[i] = P.up[a_ * NU + i];
    // input-row bound of row q (0: u <= ub, 1: -u <= -lb) of input i
    auto w_in = [&](int i, int q) -> double { return q ? -c.u_lb[i] : c.u_ub[i]; };

    // ---------------- start: U = 0, sig = 0, X = simulation, t = max(w - g, floor), lam = 1 ----------------
    int mact = 0;
    double scale_p = 1.0;
    {
        double x[NX];
#pragma unroll
        for (int s = 0; s < NX; ++s) {
            x[s] = x0[s];
            X[s] = x[s];
        }
        for (int k = 0; k < N; ++k) {
            double xn[NX];
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                double v = 0.0;
#pragma unroll
                for (int q = 0; q < NX; ++q) v = fma((double)gA[k * NX * NX + s * NX + q], x[q], v);
                xn[s] = v;
            }
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                x[s] = xn[s];
                X[(k + 1) * NX + s] = xn[s];
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) U[k * NUP + i] = 0.0;
#pragma unroll
            for (int q = 0; q < NS; ++q) sig[k * NSP + q] = 0.0;
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                const int R = k * MC + r;
                const double hr = gh[R];
                if (__builtin_isfinite(hr)) {
                    double g = 0.0;
#pragma unroll
                    for (int s = 0; s < NX; ++s) g = fma((double)gC[k * MC * NX + r * NX + s], x[s], g);
                    const double s0 = hr - g;
                    t[R] = s0 > kT0Floor ? s0 : kT0Floor;
                    lam[R] = 1.0;
                    ++mact;
                    scale_p = fmax(scale_p, fabs(hr));
                } else {
                    t[R] = 1.0;
                    lam[R] = 0.0;
                }
            }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int R = ms + 2 * (k * NU + i) + q;
                    const double wv = w_in(i, q);
                    if (__builtin_isfinite(wv)) {
                        t[R] = wv > kT0Floor ? wv : kT0Floor;  // g = +-u = 0
                        lam[R] = 1.0;
                        ++mact;
                        scale_p = fmax(scale_p, fabs(wv));
                    } else {
                        t[R] = 1.0;
                        lam[R] = 0.0;
                    }
                }
        }
    }
    const double qs_max = c.qs_max, tol = c.tol;
    const double mactd = mact ? (double)mact : 1.0;

    // ---- row algebra of one block (the MC rows of stage kb, acting on X_{kb+1}) ----
    // th, the slack-group Schur terms Dsig, the slack residual rsig (oracle solve_one); the block's
    // data come from a stage image (C rows at M::C, h at M::h) and the caller's t / lam / x / sigma
    struct Blk {
        double th[MC], rp[MC], tt[MC], ll[MC], Dsig[NS], rsig[NS];
        bool act[MC];
    };
    auto blk_rows = [&](int buf, const double* xn, const double* sg, const double* tt, const double* ll, Blk& q) {
#pragma unroll
        for (int r = 0; r < MC; ++r) {
            const double hr = im(buf, M::h + r);
            q.act[r] = __builtin_isfinite(hr);
            q.tt[r] = tt[r];
            q.ll[r] = ll[r];
            double g = 0.0;
#pragma unroll
            for (int s = 0; s < NX; ++s) g = fma(im(buf, M::C + r * NX + s), xn[s], g);
            const int jj = c.row_slack[r];
            if (jj >= 0) g += (double)c.row_sign[r] * sg[jj];
            q.rp[r] = q.act[r] ? g + q.tt[r] - hr : 0.0;
            q.th[r] = q.act[r] ? q.ll[r] / q.tt[r] : 0.0;
        }
#pragma unroll
        for (int jj = 0; jj < NS; ++jj) {
            double v = 2.0 * c.Qs[jj], rsv = 2.0 * c.Qs[jj] * sg[jj];
#pragma unroll
            for (int r = 0; r < MC; ++r)
                if (c.row_slack[r] == jj) {
                    v += q.th[r];
                    rsv += (double)c.row_sign[r] * q.ll[r];
                }
            q.Dsig[jj] = v;
            q.rsig[jj] = rsv;
        }
    };
    // rho (rows of the block) from the complementarity rhs rc, and rt (stable group form)
    auto blk_rho = [&](const Blk& q, const double* rc, double* rho, double* rt) {
#pragma unroll
        for (int r = 0; r < MC; ++r) rho[r] = q.act[r] ? (rc[r] + q.ll[r] * q.rp[r]) / q.tt[r] : 0.0;
#pragma unroll
        for (int r = 0; r < MC; ++r) {
            const int jj = c.row_slack[r];
            if (jj < 0) {
                rt[r] = rho[r];
                continue;
            }
            double v = 2.0 * c.Qs[jj] * rho[r] - q.th[r] * (double)c.row_sign[r] * q.rsig[jj];
#pragma unroll
            for (int r2 = 0; r2 < MC; ++r2) {
                if (r2 == r || c.row_slack[r2] != jj) continue;
                v += q.th[r2] * rho[r] - q.th[r] * (double)(c.row_sign[r] * c.row_sign[r2]) * rho[r2];
            }
            rt[r] = v / q.Dsig[jj];
        }
    };
    // W = 2Q + M (stable group Schur form) of the block (oracle stage_w); lower triangle, packed
    auto blk_w = [&](int buf, const Blk& q, double* W) {
#pragma unroll
        for (int s = 0; s < NX; ++s)
#pragma unroll
            for (int u = 0; u <= s; ++u) W[sy(s, u)] = 2.0 * c.Q[s * NX + u];
#pragma unroll
        for (int r = 0; r < MC; ++r) {
            double c1[NX];
#pragma unroll
            for (int s = 0; s < NX; ++s) c1[s] = im(buf, M::C + r * NX + s);
            const double th1 = q.th[r];
            const int jj = c.row_slack[r];
            if (jj < 0) {
#pragma unroll
                for (int s = 0; s < NX; ++s)
#pragma unroll
                    for (int u = 0; u <= s; ++u) W[sy(s, u)] += th1 * c1[s] * c1[u];
                continue;
            }
            const double inv = 1.0 / q.Dsig[jj], qq = 2.0 * c.Qs[jj];
#pragma unroll
            for (int s = 0; s < NX; ++s)
#pragma unroll
                for (int u = 0; u <= s; ++u) W[sy(s, u)] += qq * th1 * c1[s] * c1[u] * inv;
#pragma unroll
            for (int r2 = r + 1; r2 < MC; ++r2) {
                if (c.row_slack[r2] != jj) continue;
                double c2[NX];
#pragma unroll
                for (int s = 0; s < NX; ++s) c2[s] = im(buf, M::C + r2 * NX + s);
                const double th2 = q.th[r2], s1 = c.row_sign[r], s2 = c.row_sign[r2];
#pragma unroll
                for (int s = 0; s < NX; ++s)
#pragma unroll
                    for (int u = 0; u <= s; ++u)
                        W[sy(s, u)] += th1 * th2 * (s1 * c1[s] - s2 * c2[s]) * (s1 * c1[u] - s2 * c2[u]) * inv;
            }
        }
    };
    // 2R u_k + 2dR (du_k - du_{k+1}) (the input part of the gradient), entry i, from u_{k-1}, u_k, u_{k+1}
    auto rdr = [&](int k, int i, const double* um, const double* uk, const double* un) -> double {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < NU; ++q) {
            const double duk = uk[q] - um[q];
            const double dun = (k + 1 < N) ? un[q] - uk[q] : 0.0;
            v += 2.0 * c.R[i * NU + q] * uk[q] + 2.0 * c.dR[i * NU + q] * (duk - dun);
        }
        return v;
    };
    // gains store (RF precision; fp32 in Ff, fp64 in Fd) and image fetch / read
    auto storeF = [&](int k, const auto* K, const auto* Hi) {
        using RF = std::remove_cv_t<std::remove_reference_t<decltype(K[0])>>;
#pragma unroll
        for (int e = 0; e < NU * NA; ++e) {
            if constexpr (std::is_same_v<RF, float>) Ff[k * SF + e] = K[e];
            else Fd[k * SF + e] = K[e];
        }
#pragma unroll
        for (int e = 0; e < NU * NU; ++e) {
            if constexpr (std::is_same_v<RF, float>) Ff[k * SF + NU * NA + e] = Hi[e];
            else Fd[k * SF + NU * NA + e] = Hi[e];
        }
    };
    auto fetchF = [&](auto rf_tag, int buf, int k) {
        using RF = decltype(rf_tag);
        if constexpr (std::is_same_v<RF, float>) ff(buf, 2 * L.Ff + (size_t)k * SF, SF);
        else fd(buf, M::Fd, L.Fd + (size_t)k * SF, SF);
    };
    auto imF = [&](auto rf_tag, int buf, int e) {
        using RF = decltype(rf_tag);
        if constexpr (std::is_same_v<RF, float>) return imf(buf, e);
        else return im(buf, M::Fd + e);
    };
    // backward solve step at stage k (oracle ric_solve): g = p_u - rhs + B'p_x, dUp = -Hi g,
    // p <- [A'p_x; 0] + K'g; A, B, K, Hi from the image
    auto bsolve_img = [&](auto rf_tag, int buf, const double* rhs, auto* pv, double* dup) {
        using RF = decltype(rf_tag);
        RF g[NU], pn[NA];
#pragma unroll
        for (int cc = 0; cc < NU; ++cc) {
            RF v = pv[NX + cc] - (RF)rhs[cc];
#pragma unroll
            for (int s = 0; s < NX; ++s) v += (RF)im(buf, M::B + s * NU + cc) * pv[s];
            g[cc] = v;
        }
#pragma unroll
        for (int cc = 0; cc < NU; ++cc) {
            RF v = 0;
#pragma unroll
            for (int e = 0; e < NU; ++e) v -= imF(rf_tag, buf, NU * NA + cc * NU + e) * g[e];
            dup[cc] = (double)v;
        }
#pragma unroll
        for (int jj = 0; jj < NA; ++jj) {
            RF v = 0;
            if (jj < NX)
#pragma unroll
                for (int s = 0; s < NX; ++s) v += (RF)im(buf, M::A + s * NX + jj) * pv[s];
#pragma unroll
            for (int cc = 0; cc < NU; ++cc) v += imF(rf_tag, buf, cc * NA + jj) * g[cc];
            pn[jj] = v;
        }
#pragma unroll
        for (int jj = 0; jj < NA; ++jj) pv[jj] = pn[jj];
    };

    // ============ S1: lazy update, residuals, factorisation, predictor backward solve ============
    // Step jb = N .. 0: the block part of block kb = jb - 1 (jb >= 1; the previous step's update of
    // its rows, X_jb, sigma_kb, u_kb, then its residual terms, W_jb and y_jb) and the stage part of
    // stage k = jb (jb <= N-1: rows of u_k, dual residual, predictor rhs, factorisation, backward
    // solve).  u_{k+1}, u_k and the rows of u_k come from the two previous steps (registers): the
    // image of a step is fetched before the step before it stores its update.
    auto s1_fetch = [&](int buf, int jb, bool apply) {
        if (jb <= N - 1) {
            fd(buf, M::A, L.iA + (size_t)jb * NX * NX, NX * NX);
            fd(buf, M::B, L.iB + (size_t)jb * NX * NU, NX * NU);
        }
        if (jb >= 1) {
            const int kb = jb - 1;
            fd(buf, M::C, L.iC + (size_t)kb * MC * NX, MC * NX);
            fd(buf, M::h, L.ih + (size_t)kb * MC, MC);
            fd(buf, M::p, L.ip + (size_t)jb * NX, NX);
            fd(buf, M::X, L.X + (size_t)jb * NX, NX);
            fd(buf, M::sig, L.sig + (size_t)kb * NSP, NS);
            fd(buf, M::tB, L.t + (size_t)kb * MC, MC);
            fd(buf, M::lB, L.lam + (size_t)kb * MC, MC);
            fd(buf, M::U, L.U + (size_t)kb * NUP, NU);
            fd(buf, M::tI, L.t + ms + (size_t)kb * 2 * NU, 2 * NU);
            fd(buf, M::lI, L.lam + ms + (size_t)kb * 2 * NU, 2 * NU);
            if (apply) {
                fd(buf, M::dX, L.dX + (size_t)jb * NX, NX);
                fd(buf, M::dsig, L.dsig + (size_t)kb * NSP, NS);
                fd(buf, M::dtB, L.dt + (size_t)kb * MC, MC);
                fd(buf, M::dlB, L.dl + (size_t)kb * MC, MC);
                fd(buf, M::dU, L.dU + (size_t)kb * NUP, NU);
                fd(buf, M::dtI, L.dt + ms + (size_t)kb * 2 * NU, 2 * NU);
                fd(buf, M::dlI, L.dl + ms + (size_t)kb * 2 * NU, 2 * NU);
            }
        }
    };
    auto sweep1 = [&](auto rf_tag, bool apply, double al) __attribute__((always_inline)) -> S1Out {
        using RF = decltype(rf_tag);
        S1Out o{1.0, 0.0, 0.0, 0.0, 0.0, false};
        RF Pm[NA * (NA + 1) / 2], pv[NA];  // cost-to-go P_{k+1}, lower triangle packed
        double psf[NX], ps[NX], ps3[NX];
        double un[NU], uk[NU], tIk[2 * NU], lIk[2 * NU];  // u_{k+1}, u_k, rows of u_k
#pragma unroll
        for (int i = 0; i < NU; ++i) un[i] = uk[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 2 * NU; ++i) tIk[i] = lIk[i] = 0.0;
        s1_fetch(N & 1, N, apply);
        img_wait();
        for (int jb = N; jb >= 0; --jb) {
            const int buf = jb & 1, k = jb, kb = jb - 1;
            if (jb >= 1) s1_fetch(buf ^ 1, jb - 1, apply);
            // ---- block part, phase 0: the lazy update of block kb ----
            double xn[NX], sg[NS], tB[MC], lB[MC], um[NU], tIm[2 * NU], lIm[2 * NU];
            if (jb >= 1) {
#pragma unroll
                for (int s = 0; s < NX; ++s) xn[s] = im(buf, M::X + s);
#pragma unroll
                for (int q = 0; q < NS; ++q) sg[q] = im(buf, M::sig + q);
#pragma unroll
                for (int r = 0; r < MC; ++r) {
                    tB[r] = im(buf, M::tB + r);
                    lB[r] = im(buf, M::lB + r);
                }
#pragma unroll
                for (int i = 0; i < NU; ++i) um[i] = im(buf, M::U + i);
#pragma unroll
                for (int i = 0; i < 2 * NU; ++i) {
                    tIm[i] = im(buf, M::tI + i);
                    lIm[i] = im(buf, M::lI + i);
                }
                if (apply) {
#pragma unroll
                    for (int s = 0; s < NX; ++s) {
                        xn[s] = fma(al, im(buf, M::dX + s), xn[s]);
                        X[jb * NX + s] = xn[s];
                    }
#pragma unroll
                    for (int q = 0; q < NS; ++q) {
                        sg[q] = fma(al, im(buf, M::dsig + q), sg[q]);
                        sig[kb * NSP + q] = sg[q];
                    }
#pragma unroll
                    for (int r = 0; r < MC; ++r)
                        if (__builtin_isfinite(im(buf, M::h + r))) {
                            tB[r] = fma(al, im(buf, M::dtB + r), tB[r]);
                            lB[r] = fma(al, im(buf, M::dlB + r), lB[r]);
                            t[kb * MC + r] = tB[r];
                            lam[kb * MC + r] = lB[r];
                        }
#pragma unroll
                    for (int i = 0; i < NU; ++i) {
                        um[i] = fma(al, im(buf, M::dU + i), um[i]);
                        U[kb * NUP + i] = um[i];
                    }
#pragma unroll
                    for (int i = 0; i < 2 * NU; ++i)
                        if (__builtin_isfinite(w_in(i >> 1, i & 1))) {
                            tIm[i] = fma(al, im(buf, M::dtI + i), tIm[i]);
                            lIm[i] = fma(al, im(buf, M::dlI + i), lIm[i]);
                            t[ms + kb * 2 * NU + i] = tIm[i];
                            lam[ms + kb * 2 * NU + i] = lIm[i];
                        }
                }
            } else {
#pragma unroll
                for (int i = 0; i < NU; ++i) um[i] = up[i];
            }
            LANE_PHASE();
            // ---- stage part, phase 1: rows of u_k, gradient, dual residual and predictor rhs ----
            double thu[NU], rhs[NU];  // th_ub + th_lb; -rd - (B'psi3 + rt_ub - rt_lb)
            if (jb <= N - 1) {
                double rtu[NU], lamu[NU];
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    thu[i] = 0.0;
                    rtu[i] = 0.0;
                    lamu[i] = 0.0;
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const double wv = w_in(i, q);
                        const double tt = tIk[2 * i + q], ll = lIk[2 * i + q];
                        lamu[i] += q ? -ll : ll;
                        if (!__builtin_isfinite(wv)) continue;
                        const double rp = (q ? -uk[i] : uk[i]) + tt - wv;
                        o.nrp = lane_nmax(o.nrp, fabs(rp));
                        o.mu += tt * ll;
                        thu[i] += ll / tt;
                        const double rho = (-tt * ll + ll * rp) / tt;
                        rtu[i] += q ? -rho : rho;
                    }
                }
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    double gf = 0.0, gd = 0.0, g3 = 0.0;
#pragma unroll
                    for (int s = 0; s < NX; ++s) {
                        const double bs = im(buf, M::B + s * NU + i);
                        gf = fma(bs, psf[s], gf);
                        gd = fma(bs, ps[s], gd);
                        g3 = fma(bs, ps3[s], g3);
                    }
                    const double rr = rdr(k, i, um, uk, un);
                    o.gsc = lane_nmax(o.gsc, fabs(gf + rr));
                    const double rdv = gd + rr + lamu[i];
                    o.nrd = lane_nmax(o.nrd, fabs(rdv));
                    rd[k * NUP + i] = rdv;
                    rhs[i] = -rdv - (g3 + rtu[i]);
                }
            }
            LANE_PHASE();
            // ---- block part, phase 2: residual terms, W, y and the adjoints psi_jb = y_jb + A_jb' psi ----
            double W[NX * (NX + 1) / 2];
            if (jb >= 1) {
                Blk q;
                blk_rows(buf, xn, sg, tB, lB, q);
                double rc[MC], rho[MC], rt[MC];
#pragma unroll
                for (int r = 0; r < MC; ++r) {
                    rc[r] = -q.tt[r] * q.ll[r];
                    if (q.act[r]) {
                        o.nrp = lane_nmax(o.nrp, fabs(q.rp[r]));
                        o.mu += q.tt[r] * q.ll[r];
                    }
                }
#pragma unroll
                for (int qq = 0; qq < NS; ++qq) o.nrs = lane_nmax(o.nrs, fabs(q.rsig[qq]));
                blk_rho(q, rc, rho, rt);
                blk_w(buf, q, W);
                double yf[NX], y[NX], y3[NX];
#pragma unroll
                for (int s = 0; s < NX; ++s) {
                    double v = 2.0 * im(buf, M::p + s);
#pragma unroll
                    for (int u = 0; u < NX; ++u) v = fma(2.0 * c.Q[s * NX + u], xn[u], v);
                    yf[s] = v;
                    double vl = v, v3 = 0.0;
#pragma unroll
                    for (int r = 0; r < MC; ++r) {
                        const double cr = im(buf, M::C + r * NX + s);
                        vl = fma(q.ll[r], cr, vl);
                        v3 = fma(rt[r], cr, v3);
                    }
                    y[s] = vl;
                    y3[s] = v3;
                }
                if (jb == N) {
#pragma unroll
                    for (int s = 0; s < NX; ++s) {
                        psf[s] = yf[s];
                        ps[s] = y[s];
                        ps3[s] = y3[s];
                    }
                } else {
                    double nf[NX], nd[NX], n3[NX];
#pragma unroll
                    for (int jj = 0; jj < NX; ++jj) {
                        double a1 = yf[jj], a2 = y[jj], a3 = y3[jj];
#pragma unroll
                        for (int s = 0; s < NX; ++s) {
                            const double as = im(buf, M::A + s * NX + jj);
                            a1 = fma(as, psf[s], a1);
                            a2 = fma(as, ps[s], a2);
                            a3 = fma(as, ps3[s], a3);
                        }
                        nf[jj] = a1;
                        nd[jj] = a2;
                        n3[jj] = a3;
                    }
#pragma unroll
                    for (int jj = 0; jj < NX; ++jj) {
                        psf[jj] = nf[jj];
                        ps[jj] = nd[jj];
                        ps3[jj] = n3[jj];
                    }
                }
            }
            LANE_PHASE();
            if (jb == N) {  // P_N = blkdiag(W_N, 0), p = 0
#pragma unroll
                for (int i = 0; i < NA; ++i)
#pragma unroll
                    for (int jj = 0; jj <= i; ++jj) Pm[sy(i, jj)] = (i < NX) ? (RF)W[sy(i, jj)] : (RF)0;
#pragma unroll
                for (int jj = 0; jj < NA; ++jj) pv[jj] = 0;
            } else if (!o.broke) {
                // ---- stage part, phase 3: factorisation at stage k (oracle ric_factor), gains stored,
                // predictor backward solve step, T = Hy'K ----
                RF T[NA * (NA + 1) / 2];
                {
                    RF K[NU * NA], Hi[NU * NU], Hy[NU * NA];
                    {
                        RF PB[NA * NU], H[NU * NU], Lf[NU * NU];
#pragma unroll
                        for (int i = 0; i < NA; ++i)
#pragma unroll
                            for (int cc = 0; cc < NU; ++cc) {
                                RF v = Pm[sy(i, NX + cc)];
#pragma unroll
                                for (int s = 0; s < NX; ++s) v += Pm[sy(i, s)] * (RF)im(buf, M::B + s * NU + cc);
                                PB[i * NU + cc] = v;
                            }
#pragma unroll
                        for (int cc = 0; cc < NU; ++cc)
#pragma unroll
                            for (int e = 0; e < NU; ++e) {
                                RF v = (RF)(2.0 * c.R[cc * NU + e] + 2.0 * c.dR[cc * NU + e]) + PB[(NX + cc) * NU + e];
#pragma unroll
                                for (int s = 0; s < NX; ++s) v += (RF)im(buf, M::B + s * NU + cc) * PB[s * NU + e];
                                if (cc == e) v += (RF)thu[cc];
                                H[cc * NU + e] = v;
                            }
#pragma unroll
                        for (int cc = 0; cc < NU; ++cc)
#pragma unroll
                            for (int jj = 0; jj < NA; ++jj) {
                                RF v = 0;
                                if (jj < NX) {
#pragma unroll
                                    for (int s = 0; s < NX; ++s) v += PB[s * NU + cc] * (RF)im(buf, M::A + s * NX + jj);
                                } else {
                                    v = (RF)(-2.0 * c.dR[cc * NU + (jj - NX)]);
                                }
                                Hy[cc * NA + jj] = v;
                            }
#pragma unroll
                        for (int jj = 0; jj < NU; ++jj) {
                            RF d = H[jj * NU + jj];
#pragma unroll
                            for (int qq = 0; qq < jj; ++qq) d -= Lf[jj * NU + qq] * Lf[jj * NU + qq];
                            if (!(d > (RF)0)) {
                                o.broke = true;
                                d = (RF)1;
                            }
                            d = sqrt(d);
                            Lf[jj * NU + jj] = d;
#pragma unroll
                            for (int i = jj + 1; i < NU; ++i) {
                                RF v = H[i * NU + jj];
#pragma unroll
                                for (int qq = 0; qq < jj; ++qq) v -= Lf[i * NU + qq] * Lf[jj * NU + qq];
                                Lf[i * NU + jj] = v / d;
                            }
                        }
#pragma unroll
                        for (int cc = 0; cc < NU; ++cc) {
                            RF e[NU];
#pragma unroll
                            for (int i = 0; i < NU; ++i) e[i] = (i == cc) ? (RF)1 : (RF)0;
#pragma unroll
                            for (int i = 0; i < NU; ++i) {
                                RF v = e[i];
#pragma unroll
                                for (int qq = 0; qq < i; ++qq) v -= Lf[i * NU + qq] * e[qq];
                                e[i] = v / Lf[i * NU + i];
                            }
#pragma unroll
                            for (int i = NU - 1; i >= 0; --i) {
                                RF v = e[i];
#pragma unroll
                                for (int qq = i + 1; qq < NU; ++qq) v -= Lf[qq * NU + i] * e[qq];
                                e[i] = v / Lf[i * NU + i];
                            }
#pragma unroll
                            for (int i = 0; i < NU; ++i) Hi[i * NU + cc] = e[i];
                        }
                    }
#pragma unroll
                    for (int cc = 0; cc < NU; ++cc)
#pragma unroll
                        for (int jj = 0; jj < NA; ++jj) {
                            RF v = 0;
#pragma unroll
                            for (int e = 0; e < NU; ++e) v -= Hi[cc * NU + e] * Hy[e * NA + jj];
                            K[cc * NA + jj] = v;
                        }
                    storeF(k, K, Hi);
                    {   // backward solve step: g = p_u - rhs + B'p_x, dUp = -Hi g, p <- [A'p_x; 0] + K'g
                        RF g[NU], pn[NA];
#pragma unroll
                        for (int cc = 0; cc < NU; ++cc) {
                            RF v = pv[NX + cc] - (RF)rhs[cc];
#pragma unroll
                            for (int s = 0; s < NX; ++s) v += (RF)im(buf, M::B + s * NU + cc) * pv[s];
                            g[cc] = v;
                        }
#pragma unroll
                        for (int cc = 0; cc < NU; ++cc) {
                            RF v = 0;
#pragma unroll
                            for (int e = 0; e < NU; ++e) v -= Hi[cc * NU + e] * g[e];
                            dUp[k * NUP + cc] = (double)v;
                        }
#pragma unroll
                        for (int jj = 0; jj < NA; ++jj) {
                            RF v = 0;
                            if (jj < NX)
#pragma unroll
                                for (int s = 0; s < NX; ++s) v += (RF)im(buf, M::A + s * NX + jj) * pv[s];
#pragma unroll
                            for (int cc = 0; cc < NU; ++cc) v += K[cc * NA + jj] * g[cc];
                            pn[jj] = v;
                        }
#pragma unroll
                        for (int jj = 0; jj < NA; ++jj) pv[jj] = pn[jj];
                    }
                    if (jb >= 1) {
#pragma unroll
                        for (int i = 0; i < NA; ++i)
#pragma unroll
                            for (int jj = 0; jj <= i; ++jj) {
                                RF v = 0;
#pragma unroll
                                for (int cc = 0; cc < NU; ++cc) v += Hy[cc * NA + i] * K[cc * NA + jj];
                                T[sy(i, jj)] = v;
                            }
                    }
                }
                LANE_PHASE();
                // ---- phase 4: P_k = blkdiag(W_k + A'P_xx A, 2dR) + Hy'K over P_{k+1} ----
                if (jb >= 1) {
                    RF PA[NX * NX];
#pragma unroll
                    for (int s = 0; s < NX; ++s)
#pragma unroll
                        for (int jj = 0; jj < NX; ++jj) {
                            RF v = 0;
#pragma unroll
                            for (int qq = 0; qq < NX; ++qq) v += Pm[sy(s, qq)] * (RF)im(buf, M::A + qq * NX + jj);
                            PA[s * NX + jj] = v;
                        }
#pragma unroll
                    for (int i = 0; i < NA; ++i)
#pragma unroll
                        for (int jj = 0; jj <= i; ++jj) {
                            RF v;
                            if (i < NX) {
                                v = (RF)W[sy(i, jj)];
#pragma unroll
                                for (int s = 0; s < NX; ++s) v += (RF)im(buf, M::A + s * NX + i) * PA[s * NX + jj];
                            } else {
                                v = (jj >= NX) ? (RF)(2.0 * c.dR[(i - NX) * NU + (jj - NX)]) : (RF)0;
                            }
                            Pm[sy(i, jj)] = v + T[sy(i, jj)];
                        }
                }
            }
            // registers for the next step: u_{k+1} <- u_k, u_k <- u_kb, rows of u_k <- rows of u_kb
            if (jb >= 1) {
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    un[i] = uk[i];
                    uk[i] = um[i];
                }
#pragma unroll
                for (int i = 0; i < 2 * NU; ++i) {
                    tIk[i] = tIm[i];
                    lIk[i] = lIm[i];
                }
            }
            img_wait();
            LANE_PHASE();
        }
        return o;
    };

    // ============ S2 / S4: forward feedback solve, row steps ============
    // pass 0 (predictor): stores dta / dla, returns the step bound and the mu_aff polynomial;
    // pass 1 (corrector, rc of sig_mu): stores dU, dX, dsig, dt, dl.
    struct FwdOut {
        double amax, s0, s1, s2;
    };
    auto fwd_fetch = [&](auto rf_tag, int buf, int k, int pass) {
        fd(buf, M::A, L.iA + (size_t)k * NX * NX, NX * NX);
        fd(buf, M::B, L.iB + (size_t)k * NX * NU, NX * NU);
        fd(buf, M::C, L.iC + (size_t)k * MC * NX, MC * NX);
        fd(buf, M::h, L.ih + (size_t)k * MC, MC);
        fd(buf, M::X, L.X + (size_t)(k + 1) * NX, NX);
        fd(buf, M::U, L.U + (size_t)k * NUP, NU);
        fd(buf, M::sig, L.sig + (size_t)k * NSP, NS);
        fd(buf, M::tB, L.t + (size_t)k * MC, MC);
        fd(buf, M::lB, L.lam + (size_t)k * MC, MC);
        fd(buf, M::tI, L.t + ms + (size_t)k * 2 * NU, 2 * NU);
        fd(buf, M::lI, L.lam + ms + (size_t)k * 2 * NU, 2 * NU);
        fd(buf, M::dUp, L.dUp + (size_t)k * NUP, NU);
        fetchF(rf_tag, buf, k);
        if (pass) {
            fd(buf, M::aB, L.dta + (size_t)k * MC, MC);
            fd(buf, M::alB, L.dla + (size_t)k * MC, MC);
            fd(buf, M::aI, L.dta + ms + (size_t)k * 2 * NU, 2 * NU);
            fd(buf, M::alI, L.dla + ms + (size_t)k * 2 * NU, 2 * NU);
        }
    };
    auto sweep_fwd = [&](auto rf_tag, int pass, double sm) __attribute__((always_inline)) -> FwdOut {
        using RF = decltype(rf_tag);
        FwdOut o{INFINITY, 0.0, 0.0, 0.0};
        double dx[NX];
        RF dup_prev[NU];
#pragma unroll
        for (int s = 0; s < NX; ++s) dx[s] = 0.0;
#pragma unroll
        for (int i = 0; i < NU; ++i) dup_prev[i] = 0;
        if (pass) {
#pragma unroll
            for (int s = 0; s < NX; ++s) dX[s] = 0.0;
        }
        auto step_row = [&](int R, double tt, double ll, double dtv, double dlv) {
            if (dtv < 0.0) o.amax = fmin(o.amax, -tt / dtv);
            if (dlv < 0.0) o.amax = fmin(o.amax, -ll / dlv);
            o.s0 += tt * ll;
            o.s1 += tt * dlv + ll * dtv;
            o.s2 += dtv * dlv;
            if (pass) {
                dt[R] = dtv;
                dl[R] = dlv;
            } else {
                dta[R] = dtv;
                dla[R] = dlv;
            }
        };
        fwd_fetch(rf_tag, 0, 0, pass);
        img_wait();
        for (int k = 0; k < N; ++k) {
            const int buf = k & 1;
            if (k + 1 < N) fwd_fetch(rf_tag, buf ^ 1, k + 1, pass);
            double du[NU];
            RF dcur[NU];
#pragma unroll
            for (int cc = 0; cc < NU; ++cc) {
                RF v = (RF)im(buf, M::dUp + cc);
#pragma unroll
                for (int jj = 0; jj < NX; ++jj) v += imF(rf_tag, buf, cc * NA + jj) * (RF)dx[jj];
                if (k > 0)
#pragma unroll
                    for (int e = 0; e < NU; ++e) v += imF(rf_tag, buf, cc * NA + NX + e) * dup_prev[e];
                dcur[cc] = v;
                du[cc] = (double)v;
            }
#pragma unroll
            for (int cc = 0; cc < NU; ++cc) dup_prev[cc] = dcur[cc];
            double dxn[NX];
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                double v = 0.0;
#pragma unroll
                for (int qq = 0; qq < NX; ++qq) v = fma(im(buf, M::A + s * NX + qq), dx[qq], v);
#pragma unroll
                for (int cc = 0; cc < NU; ++cc) v = fma(im(buf, M::B + s * NU + cc), du[cc], v);
                dxn[s] = v;
            }
#pragma unroll
            for (int s = 0; s < NX; ++s) dx[s] = dxn[s];
            if (pass) {
#pragma unroll
                for (int cc = 0; cc < NU; ++cc) dU[k * NUP + cc] = du[cc];
#pragma unroll
                for (int s = 0; s < NX; ++s) dX[(k + 1) * NX + s] = dx[s];
            }
            // input rows of u_k: GdU = +-du
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                const double ukv = im(buf, M::U + i);
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int R = ms + 2 * (k * NU + i) + q;
                    const double wv = w_in(i, q);
                    if (!__builtin_isfinite(wv)) {
                        if (pass) {
                            dt[R] = 0.0;
                            dl[R] = 0.0;
                        }
                        continue;
                    }
                    const double tt = im(buf, M::tI + 2 * i + q), ll = im(buf, M::lI + 2 * i + q);
                    const double rp = (q ? -ukv : ukv) + tt - wv;
                    double rc = -tt * ll;
                    if (pass) rc += sm - im(buf, M::aI + 2 * i + q) * im(buf, M::alI + 2 * i + q);
                    const double rho = (rc + ll * rp) / tt;
                    const double gdu = q ? -du[i] : du[i];
                    step_row(R, tt, ll, -rp - gdu, rho + (ll / tt) * gdu);
                }
            }
            // block k rows at X_{k+1}
            double xn[NX], sg[NS], tB[MC], lB[MC];
#pragma unroll
            for (int s = 0; s < NX; ++s) xn[s] = im(buf, M::X + s);
#pragma unroll
            for (int qq = 0; qq < NS; ++qq) sg[qq] = im(buf, M::sig + qq);
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                tB[r] = im(buf, M::tB + r);
                lB[r] = im(buf, M::lB + r);
            }
            Blk q;
            blk_rows(buf, xn, sg, tB, lB, q);
            double rho[MC], gdu[MC];
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                double rc = -q.tt[r] * q.ll[r];
                if (pass && q.act[r]) rc += sm - im(buf, M::aB + r) * im(buf, M::alB + r);
                rho[r] = q.act[r] ? (rc + q.ll[r] * q.rp[r]) / q.tt[r] : 0.0;
                double g = 0.0;
#pragma unroll
                for (int s = 0; s < NX; ++s) g = fma(im(buf, M::C + r * NX + s), dx[s], g);
                gdu[r] = g;
            }
            double ds[NS];
#pragma unroll
            for (int qq = 0; qq < NS; ++qq) {
                double v = q.rsig[qq];
#pragma unroll
                for (int r = 0; r < MC; ++r)
                    if (c.row_slack[r] == qq) v += (double)c.row_sign[r] * (rho[r] + q.th[r] * gdu[r]);
                ds[qq] = -v / q.Dsig[qq];
                if (pass) dsig[k * NSP + qq] = ds[qq];
            }
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                const int R = k * MC + r;
                if (!q.act[r]) {
                    if (pass) {
                        dt[R] = 0.0;
                        dl[R] = 0.0;
                    }
                    continue;
                }
                const int jj = c.row_slack[r];
                const double sd = jj >= 0 ? (double)c.row_sign[r] * ds[jj] : 0.0;
                step_row(R, q.tt[r], q.ll[r], -q.rp[r] - gdu[r] - sd, rho[r] + q.th[r] * (gdu[r] + sd));
            }
            img_wait();
            LANE_PHASE();
        }
        return o;
    };

    // ============ S3: corrector right-hand side and backward solve ============
    // step jb = N .. 0: block part kb = jb - 1 (rt of its rows -> psi3_jb) after the stage part k = jb
    // (rows of u_k, rhs, backward solve step with the stored gains)
    auto s3_fetch = [&](auto rf_tag, int buf, int jb) {
        if (jb <= N - 1) {
            fd(buf, M::A, L.iA + (size_t)jb * NX * NX, NX * NX);
            fd(buf, M::B, L.iB + (size_t)jb * NX * NU, NX * NU);
            fd(buf, M::rd, L.rd + (size_t)jb * NUP, NU);
            fd(buf, M::U, L.U + (size_t)jb * NUP, NU);
            fd(buf, M::tI, L.t + ms + (size_t)jb * 2 * NU, 2 * NU);
            fd(buf, M::lI, L.lam + ms + (size_t)jb * 2 * NU, 2 * NU);
            fd(buf, M::aI, L.dta + ms + (size_t)jb * 2 * NU, 2 * NU);
            fd(buf, M::alI, L.dla + ms + (size_t)jb * 2 * NU, 2 * NU);
            fetchF(rf_tag, buf, jb);
        }
        if (jb >= 1) {
            const int kb = jb - 1;
            fd(buf, M::C, L.iC + (size_t)kb * MC * NX, MC * NX);
            fd(buf, M::h, L.ih + (size_t)kb * MC, MC);
            fd(buf, M::X, L.X + (size_t)jb * NX, NX);
            fd(buf, M::sig, L.sig + (size_t)kb * NSP, NS);
            fd(buf, M::tB, L.t + (size_t)kb * MC, MC);
            fd(buf, M::lB, L.lam + (size_t)kb * MC, MC);
            fd(buf, M::aB, L.dta + (size_t)kb * MC, MC);
            fd(buf, M::alB, L.dla + (size_t)kb * MC, MC);
        }
    };
    auto sweep3 = [&](auto rf_tag, double sm) __attribute__((always_inline)) {
        using RF = decltype(rf_tag);
        RF pv[NA];
        double ps3[NX];
#pragma unroll
        for (int jj = 0; jj < NA; ++jj) pv[jj] = 0;
        s3_fetch(rf_tag, N & 1, N);
        img_wait();
        for (int jb = N; jb >= 0; --jb) {
            const int buf = jb & 1, k = jb;
            if (jb >= 1) s3_fetch(rf_tag, buf ^ 1, jb - 1);
            if (jb <= N - 1) {
                double rtu[NU];
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    rtu[i] = 0.0;
                    const double ukv = im(buf, M::U + i);
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const double wv = w_in(i, q);
                        if (!__builtin_isfinite(wv)) continue;
                        const double tt = im(buf, M::tI + 2 * i + q), ll = im(buf, M::lI + 2 * i + q);
                        const double rp = (q ? -ukv : ukv) + tt - wv;
                        const double rc = -tt * ll + sm - im(buf, M::aI + 2 * i + q) * im(buf, M::alI + 2 * i + q);
                        const double rho = (rc + ll * rp) / tt;
                        rtu[i] += q ? -rho : rho;
                    }
                }
                double rhs[NU];
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    double g3 = 0.0;
#pragma unroll
                    for (int s = 0; s < NX; ++s) g3 = fma(im(buf, M::B + s * NU + i), ps3[s], g3);
                    rhs[i] = -im(buf, M::rd + i) - (g3 + rtu[i]);
                }
                double dup[NU];
                bsolve_img(rf_tag, buf, rhs, pv, dup);
#pragma unroll
                for (int i = 0; i < NU; ++i) dUp[k * NUP + i] = dup[i];
            }
            if (jb >= 1) {
                double xn[NX], sg[NS], tB[MC], lB[MC];
#pragma unroll
                for (int s = 0; s < NX; ++s) xn[s] = im(buf, M::X + s);
#pragma unroll
                for (int qq = 0; qq < NS; ++qq) sg[qq] = im(buf, M::sig + qq);
#pragma unroll
                for (int r = 0; r < MC; ++r) {
                    tB[r] = im(buf, M::tB + r);
                    lB[r] = im(buf, M::lB + r);
                }
                Blk q;
                blk_rows(buf, xn, sg, tB, lB, q);
                double rc[MC], rho[MC], rt[MC];
#pragma unroll
                for (int r = 0; r < MC; ++r)
                    rc[r] = q.act[r] ? -q.tt[r] * q.ll[r] + sm - im(buf, M::aB + r) * im(buf, M::alB + r) : 0.0;
                blk_rho(q, rc, rho, rt);
                double y3[NX];
#pragma unroll
                for (int s = 0; s < NX; ++s) {
                    double v3 = 0.0;
#pragma unroll
                    for (int r = 0; r < MC; ++r) v3 = fma(rt[r], im(buf, M::C + r * NX + s), v3);
                    y3[s] = v3;
                }
                if (jb == N) {
#pragma unroll
                    for (int s = 0; s < NX; ++s) ps3[s] = y3[s];
                } else {
                    double n3[NX];
#pragma unroll
                    for (int jj = 0; jj < NX; ++jj) {
                        double a3 = y3[jj];
#pragma unroll
                        for (int s = 0; s < NX; ++s) a3 = fma(im(buf, M::A + s * NX + jj), ps3[s], a3);
                        n3[jj] = a3;
                    }
#pragma unroll
                    for (int jj = 0; jj < NX; ++jj) ps3[jj] = n3[jj];
                }
            }
            img_wait();
            LANE_PHASE();
        }
    };

    // ================= Mehrotra iterations =================
    bool f32 = MIXED;  // this agent still factors in fp32
    double best_m = INFINITY, best_kkt = INFINITY, kkt = INFINITY;
    int best_it = 0, stop = kStopMaxIter, it;
    double alpha_prev = 1.0, alpha = 0.0;
    bool pending = false;  // a step (alpha, dU, dX, dsig, dt, dl) waits to be applied by S1
    // the sweeps in this agent's current precision (the fp32 instantiations exist only when MIXED)
    auto run1 = [&](bool apply, double al) __attribute__((always_inline)) -> S1Out {
        if constexpr (MIXED) {
            if (f32) return sweep1(0.0f, apply, al);
        }
        return sweep1(0.0, apply, al);
    };
    auto run_fwd = [&](int pass, double sm) __attribute__((always_inline)) -> FwdOut {
        if constexpr (MIXED) {
            if (f32) return sweep_fwd(0.0f, pass, sm);
        }
        return sweep_fwd(0.0, pass, sm);
    };
    auto run3 = [&](double sm) __attribute__((always_inline)) {
        if constexpr (MIXED) {
            if (f32) {
                sweep3(0.0f, sm);
                return;
            }
        }
        sweep3(0.0, sm);
    };
    for (it = 1; it <= c.max_iter; ++it) {
        S1Out o = run1(pending, alpha);
        pending = false;
        const double mu = o.mu / mactd;
        const double res = lane_nmax(lane_nmax(o.nrd / o.gsc, o.nrs / qs_max), o.nrp / scale_p);
        kkt = lane_nmax(res, mu);
        const double merit = lane_nmax(res, 1e4 * mu);
#ifdef LANE_TRACE
        printf("it %2d mu %.3e res %.3e (rd %.2e rs %.2e rp %.2e) merit %.3e alpha %.3e\n", it, mu, res, o.nrd / o.gsc,
               o.nrs / qs_max, o.nrp / scale_p, merit, alpha);
#endif
        if (!__builtin_isfinite(merit)) {
            stop = kStopNonFinite;
            break;
        }
        if (merit < best_m) {
            best_m = merit;
            best_kkt = kkt;
            best_it = it;
            for (int i = 0; i < N * NUP; ++i) bU[i] = U[i];
            for (int i = 0; i < N * NSP; ++i) bsig[i] = sig[i];
        }
        if (merit < tol) {
            stop = kStopConverged;
            break;
        }
        if (best_m < 1e3 * tol && it - best_it >= kStallIters) {
            stop = kStopStalled;
            break;
        }
        if (MIXED && f32 && (o.broke || it - best_it >= kF32Stall)) {
            f32 = false;  // this agent continues in fp64: refactor this iteration
            o = run1(false, 0.0);
        }
        if (o.broke) {
            stop = kStopBreakdown;
            break;
        }
        // ---- predictor ----
        FwdOut fp = run_fwd(0, 0.0);
        double aa = fp.amax < 1.0 ? fp.amax : 1.0;
        const double mu_aff = (fp.s0 + aa * fp.s1 + aa * aa * fp.s2) / mactd;
        double sig_c = mu > 0.0 ? pow(mu_aff / mu, 3.0) : 0.0;
        if (alpha_prev < kShortStep) sig_c = fmax(sig_c, kSigmaMin);
        const double sm = sig_c * mu;
        // ---- corrector ----
        run3(sm);
        FwdOut fc = run_fwd(1, sm);
        double al = 0.995 * fc.amax;
        if (al > 1.0) al = 1.0;
        // ---- wide-neighbourhood backtracking: t_r lam_r >= gamma mu(al) after the step ----
        for (int bt = 0; bt < kMaxBacktrack && mact; ++bt) {
            double mn = 0.0, pmin = INFINITY;
            for (int R = 0; R < m; ++R) {
                const bool act = R < ms ? __builtin_isfinite((double)gh[R]) : __builtin_isfinite(w_in(((R - ms) >> 1) % NU, (R - ms) & 1));
                if (!act) continue;
                const double pr = (t[R] + al * dt[R]) * (lam[R] + al * dl[R]);
                mn += pr;
                pmin = fmin(pmin, pr);
            }
            if (pmin >= kNbhdGamma * (mn / mactd)) break;
            al *= 0.8;
        }
        alpha_prev = al;
        alpha = al;
        pending = true;
    }
    if (it > c.max_iter) it = c.max_iter;
    int status = CMPC_SOLVED;
    if (stop != kStopConverged) {
        if (best_it > 0) {
            for (int i = 0; i < N * NUP; ++i) U[i] = bU[i];
            for (int i = 0; i < N * NSP; ++i) sig[i] = bsig[i];
            kkt = best_kkt;
        }
        status = stop_status(stop, best_m, tol);
    }
    // ---- output: exact re-simulation of the states from U, slacks, inputs, input increments ----
    const int nxe = NX + NS;
    const size_t nz = (size_t)nxe * (N + 1) + 2 * (size_t)c.n;
    double* z = P.z + a_ * nz;
    double x[NX];
#pragma unroll
    for (int s = 0; s < NX; ++s) {
        x[s] = x0[s];
        z[s] = x[s];
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) z[NX + j] = 0.0;
    for (int k = 0; k < N; ++k) {
        double u[NU];
#pragma unroll
        for (int i = 0; i < NU; ++i) u[i] = U[k * NUP + i];
        double xn[NX];
#pragma unroll
        for (int s = 0; s < NX; ++s) {
            double v = 0.0;
#pragma unroll
            for (int q = 0; q < NX; ++q) v += (double)gA[k * NX * NX + s * NX + q] * x[q];
#pragma unroll
            for (int i = 0; i < NU; ++i) v += (double)gB[k * NX * NU + s * NU + i] * u[i];
            xn[s] = v;
        }
#pragma unroll
        for (int s = 0; s < NX; ++s) {
            x[s] = xn[s];
            z[(size_t)(k + 1) * nxe + s] = x[s];
        }
#pragma unroll
        for (int j = 0; j < NS; ++j) z[(size_t)(k + 1) * nxe + NX + j] = sig[k * NSP + j];
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            z[(size_t)(N + 1) * nxe + k * NU + i] = u[i];
            z[(size_t)(N + 1) * nxe + c.n + k * NU + i] = u[i] - (k ? U[(k - 1) * NUP + i] : up[i]);
        }
    }
    if (P.kkt) P.kkt[a_] = kkt;
    if (P.iters) P.iters[a_] = it;
    if (P.status) P.status[a_] = status;
}

}  // namespace cmpc
