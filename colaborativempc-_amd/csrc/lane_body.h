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

// lane-interleaved view: element i of this lane's agent at p[i * s]
template <class T>
struct LV {
    T* p;
    size_t s;
    __host__ __device__ __forceinline__ T& operator[](int i) const { return p[(size_t)i * s]; }
};

struct LaneLayout {
    size_t X, U, sig, t, lam, bU, bsig, rd, dUp, Fd, dta, dla, dU, dX, dsig, dt, dl, Ff;
    size_t iA, iB, iC, ih, ip;  // the inputs, lane-interleaved by lane_pack (mpc_lane.hip)
    size_t total;
};

__host__ __device__ inline LaneLayout lane_layout(const MpcConst& c) {
    LaneLayout L;
    const size_t N = c.N, nx = c.nx, nu = c.nu, ns = c.ns, m = c.m, n = c.n;
    const size_t sF = nu * (nx + nu) + nu * nu;
    size_t o = 0;
    auto take = [&](size_t cnt) {
        const size_t r = o;
        o += cnt;
        return r;
    };
    L.X = take((N + 1) * nx);
    L.U = take(n);
    L.sig = take(N * ns);
    L.t = take(m);
    L.lam = take(m);
    L.bU = take(n);
    L.bsig = take(N * ns);
    L.rd = take(n);
    L.dUp = take(n);
    L.Fd = take(N * sF);
    L.dta = take(m);
    L.dla = take(m);
    L.dU = take(n);
    L.dX = take((N + 1) * nx);
    L.dsig = take(N * ns);
    L.dt = take(m);
    L.dl = take(m);
    L.Ff = take((N * sF + 1) / 2);  // floats
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

// packed lower-triangle index (i >= j) and its symmetric accessor
__host__ __device__ constexpr int sy(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// Residual and factorisation accumulators of one S1 sweep.
struct S1Out {
    double gsc, nrd, nrs, nrp, mu;
    bool broke;
};

}  // namespace

// One agent's solve (lane b of the batch).  __host__ __device__: the kernel below runs it per lane,
// and tools/lane_cpu.cpp runs the same code on the host to check it against the C restatement.
template <int NX, int NU, int MC, int NS, bool MIXED>
__host__ __device__ inline void lane_agent(const MpcConst& c, const MpcPtrs& P, int batch, int b) {
    constexpr int NA = NX + NU, SF = NU * NA + NU * NU;
    const int N = c.N, ms = c.ms, m = c.m;
    const LaneLayout L = lane_layout(c);
    const size_t S = (size_t)batch;
    double* ws = P.ws;
    const LV<double> X{ws + L.X * S + b, S}, U{ws + L.U * S + b, S}, sig{ws + L.sig * S + b, S};
    const LV<double> t{ws + L.t * S + b, S}, lam{ws + L.lam * S + b, S}, bU{ws + L.bU * S + b, S};
    const LV<double> bsig{ws + L.bsig * S + b, S}, rd{ws + L.rd * S + b, S}, dUp{ws + L.dUp * S + b, S};
    const LV<double> Fd{ws + L.Fd * S + b, S}, dta{ws + L.dta * S + b, S}, dla{ws + L.dla * S + b, S};
    const LV<double> dU{ws + L.dU * S + b, S}, dX{ws + L.dX * S + b, S}, dsig{ws + L.dsig * S + b, S};
    const LV<double> dt{ws + L.dt * S + b, S}, dl{ws + L.dl * S + b, S};
    const LV<float> Ff{reinterpret_cast<float*>(ws + L.Ff * S) + b, S};

    // inputs in the lane-interleaved copy lane_pack made (coalesced across the wavefront)
    const LV<double> gA{ws + L.iA * S + b, S}, gB{ws + L.iB * S + b, S}, gC{ws + L.iC * S + b, S};
    const LV<double> gh{ws + L.ih * S + b, S}, gp{ws + L.ip * S + b, S};
    double x0[NX], up[NU];
#pragma unroll
    for (int s = 0; s < NX; ++s) x0[s] = P.x0[(size_t)b * NX + s];
#pragma unroll
    for (int i = 0; i < NU; ++i) up[i] = P.up[(size_t)b * NU + i];

    auto loadA = [&](int k, double* A) {
#pragma unroll
        for (int i = 0; i < NX * NX; ++i) A[i] = gA[k * NX * NX + i];
    };
    auto loadB = [&](int k, double* Bm) {
#pragma unroll
        for (int i = 0; i < NX * NU; ++i) Bm[i] = gB[k * NX * NU + i];
    };
    auto loadC = [&](int k, double* C, double* h) {
#pragma unroll
        for (int i = 0; i < MC * NX; ++i) C[i] = gC[k * MC * NX + i];
#pragma unroll
        for (int r = 0; r < MC; ++r) h[r] = gh[k * MC + r];
    };
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
            double A[NX * NX], C[MC * NX], h[MC];
            loadA(k, A);
            loadC(k, C, h);
            double xn[NX];
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                double v = 0.0;
#pragma unroll
                for (int q = 0; q < NX; ++q) v = fma(A[s * NX + q], x[q], v);
                xn[s] = v;
            }
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                x[s] = xn[s];
                X[(k + 1) * NX + s] = xn[s];
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) U[k * NU + i] = 0.0;
#pragma unroll
            for (int j = 0; j < NS; ++j) sig[k * NS + j] = 0.0;
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                const int R = k * MC + r;
                if (__builtin_isfinite(h[r])) {
                    double g = 0.0;
#pragma unroll
                    for (int s = 0; s < NX; ++s) g = fma(C[r * NX + s], x[s], g);
                    const double s0 = h[r] - g;
                    t[R] = s0 > kT0Floor ? s0 : kT0Floor;
                    lam[R] = 1.0;
                    ++mact;
                    scale_p = fmax(scale_p, fabs(h[r]));
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
    // th, the slack-group Schur terms Dsig, the slack residual rsig, and for rc (the complementarity
    // right-hand side per row) rho and its stable-form rt (oracle solve_one).
    struct Blk {
        double th[MC], rp[MC], tt[MC], ll[MC], Dsig[NS], rsig[NS];
        bool act[MC];
    };
    auto blk_rows = [&](int kb, const double* xn, const double* sg, const double* C, const double* h, Blk& q) {
#pragma unroll
        for (int r = 0; r < MC; ++r) {
            const int R = kb * MC + r;
            q.act[r] = __builtin_isfinite(h[r]);
            q.tt[r] = t[R];
            q.ll[r] = lam[R];
            double g = 0.0;
#pragma unroll
            for (int s = 0; s < NX; ++s) g = fma(C[r * NX + s], xn[s], g);
            const int j = c.row_slack[r];
            if (j >= 0) g += (double)c.row_sign[r] * sg[j];
            q.rp[r] = q.act[r] ? g + q.tt[r] - h[r] : 0.0;
            q.th[r] = q.act[r] ? q.ll[r] / q.tt[r] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            double v = 2.0 * c.Qs[j], rs = 2.0 * c.Qs[j] * sg[j];
#pragma unroll
            for (int r = 0; r < MC; ++r)
                if (c.row_slack[r] == j) {
                    v += q.th[r];
                    rs += (double)c.row_sign[r] * q.ll[r];
                }
            q.Dsig[j] = v;
            q.rsig[j] = rs;
        }
    };
    // rho (rows of the block) from the complementarity rhs rc, and rt (stable group form)
    auto blk_rho = [&](const Blk& q, const double* rc, double* rho, double* rt) {
#pragma unroll
        for (int r = 0; r < MC; ++r) rho[r] = q.act[r] ? (rc[r] + q.ll[r] * q.rp[r]) / q.tt[r] : 0.0;
#pragma unroll
        for (int r = 0; r < MC; ++r) {
            const int j = c.row_slack[r];
            if (j < 0) {
                rt[r] = rho[r];
                continue;
            }
            double v = 2.0 * c.Qs[j] * rho[r] - q.th[r] * (double)c.row_sign[r] * q.rsig[j];
#pragma unroll
            for (int r2 = 0; r2 < MC; ++r2) {
                if (r2 == r || c.row_slack[r2] != j) continue;
                v += q.th[r2] * rho[r] - q.th[r] * (double)(c.row_sign[r] * c.row_sign[r2]) * rho[r2];
            }
            rt[r] = v / q.Dsig[j];
        }
    };
    // W = 2Q + M (stable group Schur form) of the block (oracle stage_w); lower triangle, packed
    auto blk_w = [&](const Blk& q, const double* C, double* W) {
#pragma unroll
        for (int s = 0; s < NX; ++s)
#pragma unroll
            for (int u = 0; u <= s; ++u) W[sy(s, u)] = 2.0 * c.Q[s * NX + u];
#pragma unroll
        for (int r = 0; r < MC; ++r) {
            const double* c1 = C + r * NX;
            const double th1 = q.th[r];
            const int j = c.row_slack[r];
            if (j < 0) {
#pragma unroll
                for (int s = 0; s < NX; ++s)
#pragma unroll
                    for (int u = 0; u <= s; ++u) W[sy(s, u)] += th1 * c1[s] * c1[u];
                continue;
            }
            const double inv = 1.0 / q.Dsig[j], qq = 2.0 * c.Qs[j];
#pragma unroll
            for (int s = 0; s < NX; ++s)
#pragma unroll
                for (int u = 0; u <= s; ++u) W[sy(s, u)] += qq * th1 * c1[s] * c1[u] * inv;
#pragma unroll
            for (int r2 = r + 1; r2 < MC; ++r2) {
                if (c.row_slack[r2] != j) continue;
                const double* c2 = C + r2 * NX;
                const double th2 = q.th[r2], s1 = c.row_sign[r], s2 = c.row_sign[r2];
#pragma unroll
                for (int s = 0; s < NX; ++s)
#pragma unroll
                    for (int u = 0; u <= s; ++u)
                        W[sy(s, u)] += th1 * th2 * (s1 * c1[s] - s2 * c2[s]) * (s1 * c1[u] - s2 * c2[u]) * inv;
            }
        }
    };
    // 2R u_k + 2dR (du_k - du_{k+1}) (the input part of the gradient), entry i
    auto rdr = [&](int k, int i) -> double {
        double v = 0.0;
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            const double uk = U[k * NU + j];
            const double duk = uk - (k ? U[(k - 1) * NU + j] : up[j]);
            const double dun = (k + 1 < N) ? U[(k + 1) * NU + j] - uk : 0.0;
            v += 2.0 * c.R[i * NU + j] * uk + 2.0 * c.dR[i * NU + j] * (duk - dun);
        }
        return v;
    };
    // gains store / load (RF precision; fp32 in Ff, fp64 in Fd)
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
    auto loadF = [&](int k, auto* K, auto* Hi) {
        using RF = std::remove_reference_t<decltype(K[0])>;
#pragma unroll
        for (int e = 0; e < NU * NA; ++e) {
            if constexpr (std::is_same_v<RF, float>) K[e] = Ff[k * SF + e];
            else K[e] = Fd[k * SF + e];
        }
#pragma unroll
        for (int e = 0; e < NU * NU; ++e) {
            if constexpr (std::is_same_v<RF, float>) Hi[e] = Ff[k * SF + NU * NA + e];
            else Hi[e] = Fd[k * SF + NU * NA + e];
        }
    };
    // backward solve step at stage k (oracle ric_solve): g = p_u - rhs + B'p_x, dUp = -Hi g,
    // p <- [A'p_x; 0] + K'g
    auto bsolve = [&](const auto* K, const auto* Hi, const double* A, const double* Bm, const double* rhs, auto* pv,
                      double* dup) {
        using RF = std::remove_cv_t<std::remove_reference_t<decltype(K[0])>>;
        RF g[NU], pn[NA];
#pragma unroll
        for (int cc = 0; cc < NU; ++cc) {
            RF v = pv[NX + cc] - (RF)rhs[cc];
#pragma unroll
            for (int s = 0; s < NX; ++s) v += (RF)Bm[s * NU + cc] * pv[s];
            g[cc] = v;
        }
#pragma unroll
        for (int cc = 0; cc < NU; ++cc) {
            RF v = 0;
#pragma unroll
            for (int e = 0; e < NU; ++e) v -= Hi[cc * NU + e] * g[e];
            dup[cc] = (double)v;
        }
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            RF v = 0;
            if (j < NX)
#pragma unroll
                for (int s = 0; s < NX; ++s) v += (RF)A[s * NX + j] * pv[s];
#pragma unroll
            for (int cc = 0; cc < NU; ++cc) v += K[cc * NA + j] * g[cc];
            pn[j] = v;
        }
#pragma unroll
        for (int j = 0; j < NA; ++j) pv[j] = pn[j];
    };

    // ============ S1: lazy update, residuals, factorisation, predictor backward solve ============
    auto sweep1 = [&](auto rf_tag, bool apply, double al) -> S1Out {
        using RF = decltype(rf_tag);
        S1Out o{1.0, 0.0, 0.0, 0.0, 0.0, false};
        RF Pm[NA * (NA + 1) / 2], pv[NA];  // cost-to-go P_{k+1}, lower triangle packed
        double psf[NX], ps[NX], ps3[NX];
        // lazy update of block kb: X_{kb+1}, sig_kb, its rows, U_kb and the rows of u_kb
        auto update_blk = [&](int kb) {
            if (!apply) return;
#pragma unroll
            for (int s = 0; s < NX; ++s) X[(kb + 1) * NX + s] = fma(al, dX[(kb + 1) * NX + s], X[(kb + 1) * NX + s]);
#pragma unroll
            for (int j = 0; j < NS; ++j) sig[kb * NS + j] = fma(al, dsig[kb * NS + j], sig[kb * NS + j]);
#pragma unroll
            for (int i = 0; i < NU; ++i) U[kb * NU + i] = fma(al, dU[kb * NU + i], U[kb * NU + i]);
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                const int R = kb * MC + r;
                if (__builtin_isfinite(gh[R])) {
                    t[R] = fma(al, dt[R], t[R]);
                    lam[R] = fma(al, dl[R], lam[R]);
                }
            }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int R = ms + 2 * (kb * NU + i) + q;
                    if (__builtin_isfinite(w_in(i, q))) {
                        t[R] = fma(al, dt[R], t[R]);
                        lam[R] = fma(al, dl[R], lam[R]);
                    }
                }
        };
        // rows of block kb at X_{kb+1}: residual terms, W, and the three adjoint loads y
        auto block = [&](int kb, const double* C, const double* h, double* W, double* yf, double* y, double* y3) {
            double xn[NX], sg[NS];
#pragma unroll
            for (int s = 0; s < NX; ++s) xn[s] = X[(kb + 1) * NX + s];
#pragma unroll
            for (int j = 0; j < NS; ++j) sg[j] = sig[kb * NS + j];
            Blk q;
            blk_rows(kb, xn, sg, C, h, q);
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
            for (int j = 0; j < NS; ++j) o.nrs = lane_nmax(o.nrs, fabs(q.rsig[j]));
            blk_rho(q, rc, rho, rt);
            blk_w(q, C, W);
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                double v = 2.0 * gp[(kb + 1) * NX + s];
#pragma unroll
                for (int u = 0; u < NX; ++u) v = fma(2.0 * c.Q[s * NX + u], xn[u], v);
                yf[s] = v;
                double vl = v, v3 = 0.0;
#pragma unroll
                for (int r = 0; r < MC; ++r) {
                    vl = fma(q.ll[r], C[r * NX + s], vl);
                    v3 = fma(rt[r], C[r * NX + s], v3);
                }
                y[s] = vl;
                y3[s] = v3;
            }
        };
        {   // prologue: block N-1 (X_N): psi_N = y_N, P_N = blkdiag(W_N, 0), p = 0
            update_blk(N - 1);
            double C[MC * NX], h[MC], W[NX * (NX + 1) / 2];
            loadC(N - 1, C, h);
            block(N - 1, C, h, W, psf, ps, ps3);
#pragma unroll
            for (int i = 0; i < NA; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j) Pm[sy(i, j)] = (i < NX) ? (RF)W[sy(i, j)] : (RF)0;
#pragma unroll
            for (int j = 0; j < NA; ++j) pv[j] = 0;
        }
        for (int k = N - 1; k >= 0; --k) {
            if (k >= 1) update_blk(k - 1);
            double A[NX * NX], Bm[NX * NU];
            loadA(k, A);
            loadB(k, Bm);
            // ---- input rows of u_k ----
            double thu[NU], rtu[NU];  // th_ub + th_lb, rt_ub - rt_lb
            double lamu[NU];          // lam_ub - lam_lb
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                thu[i] = 0.0;
                rtu[i] = 0.0;
                lamu[i] = 0.0;
                const double uk = U[k * NU + i];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int R = ms + 2 * (k * NU + i) + q;
                    const double wv = w_in(i, q);
                    const double tt = t[R], ll = lam[R];
                    lamu[i] += q ? -ll : ll;
                    if (!__builtin_isfinite(wv)) continue;
                    const double rp = (q ? -uk : uk) + tt - wv;
                    o.nrp = lane_nmax(o.nrp, fabs(rp));
                    o.mu += tt * ll;
                    const double th = ll / tt;
                    thu[i] += th;
                    const double rho = (-tt * ll + ll * rp) / tt;
                    rtu[i] += q ? -rho : rho;
                }
            }
            // ---- gradient / dual residual / predictor rhs of u_k ----
            double rhs[NU];
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                double gf = 0.0, gd = 0.0, g3 = 0.0;
#pragma unroll
                for (int s = 0; s < NX; ++s) {
                    gf = fma(Bm[s * NU + i], psf[s], gf);
                    gd = fma(Bm[s * NU + i], ps[s], gd);
                    g3 = fma(Bm[s * NU + i], ps3[s], g3);
                }
                const double rr = rdr(k, i);
                o.gsc = lane_nmax(o.gsc, fabs(gf + rr));
                const double rdv = gd + rr + lamu[i];
                o.nrd = lane_nmax(o.nrd, fabs(rdv));
                rd[k * NU + i] = rdv;
                rhs[i] = -rdv - (g3 + rtu[i]);
            }
            // ---- Riccati factorisation at stage k (oracle ric_factor, standard form) ----
            RF K[NU * NA], Hi[NU * NU], Hy[NU * NA];
            if (!o.broke) {
                RF PB[NA * NU], H[NU * NU], Lf[NU * NU];
#pragma unroll
                for (int i = 0; i < NA; ++i)
#pragma unroll
                    for (int cc = 0; cc < NU; ++cc) {
                        RF v = Pm[sy(i, NX + cc)];
#pragma unroll
                        for (int s = 0; s < NX; ++s) v += Pm[sy(i, s)] * (RF)Bm[s * NU + cc];
                        PB[i * NU + cc] = v;
                    }
#pragma unroll
                for (int cc = 0; cc < NU; ++cc)
#pragma unroll
                    for (int e = 0; e < NU; ++e) {
                        RF v = (RF)(2.0 * c.R[cc * NU + e] + 2.0 * c.dR[cc * NU + e]) + PB[(NX + cc) * NU + e];
#pragma unroll
                        for (int s = 0; s < NX; ++s) v += (RF)Bm[s * NU + cc] * PB[s * NU + e];
                        if (cc == e) v += (RF)thu[cc];
                        H[cc * NU + e] = v;
                    }
#pragma unroll
                for (int cc = 0; cc < NU; ++cc)
#pragma unroll
                    for (int j = 0; j < NA; ++j) {
                        RF v = 0;
                        if (j < NX) {
#pragma unroll
                            for (int s = 0; s < NX; ++s) v += PB[s * NU + cc] * (RF)A[s * NX + j];
                        } else {
                            v = (RF)(-2.0 * c.dR[cc * NU + (j - NX)]);
                        }
                        Hy[cc * NA + j] = v;
                    }
#pragma unroll
                for (int j = 0; j < NU; ++j) {
                    RF d = H[j * NU + j];
#pragma unroll
                    for (int q = 0; q < j; ++q) d -= Lf[j * NU + q] * Lf[j * NU + q];
                    if (!(d > (RF)0)) {
                        o.broke = true;
                        d = (RF)1;
                    }
                    d = sqrt(d);
                    Lf[j * NU + j] = d;
#pragma unroll
                    for (int i = j + 1; i < NU; ++i) {
                        RF v = H[i * NU + j];
#pragma unroll
                        for (int q = 0; q < j; ++q) v -= Lf[i * NU + q] * Lf[j * NU + q];
                        Lf[i * NU + j] = v / d;
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
                        for (int q = 0; q < i; ++q) v -= Lf[i * NU + q] * e[q];
                        e[i] = v / Lf[i * NU + i];
                    }
#pragma unroll
                    for (int i = NU - 1; i >= 0; --i) {
                        RF v = e[i];
#pragma unroll
                        for (int q = i + 1; q < NU; ++q) v -= Lf[q * NU + i] * e[q];
                        e[i] = v / Lf[i * NU + i];
                    }
#pragma unroll
                    for (int i = 0; i < NU; ++i) Hi[i * NU + cc] = e[i];
                }
#pragma unroll
                for (int cc = 0; cc < NU; ++cc)
#pragma unroll
                    for (int j = 0; j < NA; ++j) {
                        RF v = 0;
#pragma unroll
                        for (int e = 0; e < NU; ++e) v -= Hi[cc * NU + e] * Hy[e * NA + j];
                        K[cc * NA + j] = v;
                    }
                storeF(k, K, Hi);
                double dup[NU];
                bsolve(K, Hi, A, Bm, rhs, pv, dup);
#pragma unroll
                for (int i = 0; i < NU; ++i) dUp[k * NU + i] = dup[i];
            }
            if (k == 0) break;
            // ---- block k-1 (X_k): residual terms, W_k, adjoints psi_k = y_k + A_k' psi_{k+1}, P_k ----
            double C[MC * NX], h[MC], W[NX * (NX + 1) / 2], yf[NX], y[NX], y3[NX];
            loadC(k - 1, C, h);
            block(k - 1, C, h, W, yf, y, y3);
            double nf[NX], nd[NX], n3[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) {
                double a1 = yf[j], a2 = y[j], a3 = y3[j];
#pragma unroll
                for (int s = 0; s < NX; ++s) {
                    a1 = fma(A[s * NX + j], psf[s], a1);
                    a2 = fma(A[s * NX + j], ps[s], a2);
                    a3 = fma(A[s * NX + j], ps3[s], a3);
                }
                nf[j] = a1;
                nd[j] = a2;
                n3[j] = a3;
            }
#pragma unroll
            for (int j = 0; j < NX; ++j) {
                psf[j] = nf[j];
                ps[j] = nd[j];
                ps3[j] = n3[j];
            }
            if (!o.broke) {
                // P_k = blkdiag(W_k + A'P_xx A, 2dR) + Hy'K, written over P_{k+1} once P_xx A is formed
                RF PA[NX * NX];
#pragma unroll
                for (int s = 0; s < NX; ++s)
#pragma unroll
                    for (int j = 0; j < NX; ++j) {
                        RF v = 0;
#pragma unroll
                        for (int q = 0; q < NX; ++q) v += Pm[sy(s, q)] * (RF)A[q * NX + j];
                        PA[s * NX + j] = v;
                    }
#pragma unroll
                for (int i = 0; i < NA; ++i)
#pragma unroll
                    for (int j = 0; j <= i; ++j) {
                        RF v;
                        if (i < NX) {
                            v = (RF)W[sy(i, j)];
#pragma unroll
                            for (int s = 0; s < NX; ++s) v += (RF)A[s * NX + i] * PA[s * NX + j];
                        } else {
                            v = (j >= NX) ? (RF)(2.0 * c.dR[(i - NX) * NU + (j - NX)]) : (RF)0;
                        }
#pragma unroll
                        for (int cc = 0; cc < NU; ++cc) v += Hy[cc * NA + i] * K[cc * NA + j];
                        Pm[sy(i, j)] = v;
                    }
            }
        }
        return o;
    };

    // ============ S2 / S4: forward feedback solve, row steps ============
    // pass 0 (predictor): stores dta / dla, returns the step bound and the mu_aff polynomial;
    // pass 1 (corrector, rc of sig_mu): stores dU, dX, dsig, dt, dl.
    struct FwdOut {
        double amax, s0, s1, s2;
    };
    auto sweep_fwd = [&](auto rf_tag, int pass, double sm) -> FwdOut {
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
        for (int k = 0; k < N; ++k) {
            double A[NX * NX], Bm[NX * NU], C[MC * NX], h[MC];
            loadA(k, A);
            loadB(k, Bm);
            loadC(k, C, h);
            RF K[NU * NA], Hi[NU * NU];
            loadF(k, K, Hi);
            double du[NU];
            RF dcur[NU];
#pragma unroll
            for (int cc = 0; cc < NU; ++cc) {
                RF v = (RF)dUp[k * NU + cc];
#pragma unroll
                for (int j = 0; j < NX; ++j) v += K[cc * NA + j] * (RF)dx[j];
                if (k > 0)
#pragma unroll
                    for (int e = 0; e < NU; ++e) v += K[cc * NA + NX + e] * dup_prev[e];
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
                for (int q = 0; q < NX; ++q) v = fma(A[s * NX + q], dx[q], v);
#pragma unroll
                for (int cc = 0; cc < NU; ++cc) v = fma(Bm[s * NU + cc], du[cc], v);
                dxn[s] = v;
            }
#pragma unroll
            for (int s = 0; s < NX; ++s) dx[s] = dxn[s];
#ifdef LANE_TRACE
            if (k < 2 || k == N - 1) printf("  pass %d k %d du %.10e %.10e %.10e\n", pass, k, du[0], du[1 % NU], du[2 % NU]);
#endif
            if (pass) {
#pragma unroll
                for (int cc = 0; cc < NU; ++cc) dU[k * NU + cc] = du[cc];
#pragma unroll
                for (int s = 0; s < NX; ++s) dX[(k + 1) * NX + s] = dx[s];
            }
            // input rows of u_k: GdU = +-du
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                const double uk = U[k * NU + i];
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
                    const double tt = t[R], ll = lam[R];
                    const double rp = (q ? -uk : uk) + tt - wv;
                    double rc = -tt * ll;
                    if (pass) rc += sm - dta[R] * dla[R];
                    const double rho = (rc + ll * rp) / tt;
                    const double gdu = q ? -du[i] : du[i];
                    step_row(R, tt, ll, -rp - gdu, rho + (ll / tt) * gdu);
                }
            }
            // block k rows at X_{k+1}
            double xn[NX], sg[NS];
#pragma unroll
            for (int s = 0; s < NX; ++s) xn[s] = X[(k + 1) * NX + s];
#pragma unroll
            for (int j = 0; j < NS; ++j) sg[j] = sig[k * NS + j];
            Blk q;
            blk_rows(k, xn, sg, C, h, q);
            double rc[MC], rho[MC], gdu[MC];
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                const int R = k * MC + r;
                rc[r] = -q.tt[r] * q.ll[r];
                if (pass && q.act[r]) rc[r] += sm - dta[R] * dla[R];
                rho[r] = q.act[r] ? (rc[r] + q.ll[r] * q.rp[r]) / q.tt[r] : 0.0;
                double g = 0.0;
#pragma unroll
                for (int s = 0; s < NX; ++s) g = fma(C[r * NX + s], dx[s], g);
                gdu[r] = g;
            }
            double ds[NS];
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                double v = q.rsig[j];
#pragma unroll
                for (int r = 0; r < MC; ++r)
                    if (c.row_slack[r] == j) v += (double)c.row_sign[r] * (rho[r] + q.th[r] * gdu[r]);
                ds[j] = -v / q.Dsig[j];
                if (pass) dsig[k * NS + j] = ds[j];
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
                const int j = c.row_slack[r];
                const double sd = j >= 0 ? (double)c.row_sign[r] * ds[j] : 0.0;
                step_row(R, q.tt[r], q.ll[r], -q.rp[r] - gdu[r] - sd, rho[r] + q.th[r] * (gdu[r] + sd));
            }
        }
        return o;
    };

    // ============ S3: corrector right-hand side and backward solve ============
    auto sweep3 = [&](auto rf_tag, double sm) {
        using RF = decltype(rf_tag);
        RF pv[NA];
        double ps3[NX];
        auto y3_of = [&](int kb, const double* C, const double* h, double* y3) {
            double xn[NX], sg[NS];
#pragma unroll
            for (int s = 0; s < NX; ++s) xn[s] = X[(kb + 1) * NX + s];
#pragma unroll
            for (int j = 0; j < NS; ++j) sg[j] = sig[kb * NS + j];
            Blk q;
            blk_rows(kb, xn, sg, C, h, q);
            double rc[MC], rho[MC], rt[MC];
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                const int R = kb * MC + r;
                rc[r] = q.act[r] ? -q.tt[r] * q.ll[r] + sm - dta[R] * dla[R] : 0.0;
            }
            blk_rho(q, rc, rho, rt);
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                double v3 = 0.0;
#pragma unroll
                for (int r = 0; r < MC; ++r) v3 = fma(rt[r], C[r * NX + s], v3);
                y3[s] = v3;
            }
        };
        {
            double C[MC * NX], h[MC];
            loadC(N - 1, C, h);
            y3_of(N - 1, C, h, ps3);
#pragma unroll
            for (int j = 0; j < NA; ++j) pv[j] = 0;
        }
        for (int k = N - 1; k >= 0; --k) {
            double A[NX * NX], Bm[NX * NU];
            loadA(k, A);
            loadB(k, Bm);
            double rtu[NU];
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                rtu[i] = 0.0;
                const double uk = U[k * NU + i];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int R = ms + 2 * (k * NU + i) + q;
                    const double wv = w_in(i, q);
                    if (!__builtin_isfinite(wv)) continue;
                    const double tt = t[R], ll = lam[R];
                    const double rp = (q ? -uk : uk) + tt - wv;
                    const double rc = -tt * ll + sm - dta[R] * dla[R];
                    const double rho = (rc + ll * rp) / tt;
                    rtu[i] += q ? -rho : rho;
                }
            }
            double rhs[NU];
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                double g3 = 0.0;
#pragma unroll
                for (int s = 0; s < NX; ++s) g3 = fma(Bm[s * NU + i], ps3[s], g3);
                rhs[i] = -rd[k * NU + i] - (g3 + rtu[i]);
            }
            RF K[NU * NA], Hi[NU * NU];
            loadF(k, K, Hi);
            double dup[NU];
            bsolve(K, Hi, A, Bm, rhs, pv, dup);
#pragma unroll
            for (int i = 0; i < NU; ++i) dUp[k * NU + i] = dup[i];
            if (k == 0) break;
            double C[MC * NX], h[MC], y3[NX];
            loadC(k - 1, C, h);
            y3_of(k - 1, C, h, y3);
            double n3[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) {
                double a3 = y3[j];
#pragma unroll
                for (int s = 0; s < NX; ++s) a3 = fma(A[s * NX + j], ps3[s], a3);
                n3[j] = a3;
            }
#pragma unroll
            for (int j = 0; j < NX; ++j) ps3[j] = n3[j];
        }
    };

    // ================= Mehrotra iterations =================
    bool f32 = MIXED;  // this agent still factors in fp32
    double best_m = INFINITY, best_kkt = INFINITY, kkt = INFINITY;
    int best_it = 0, stop = kStopMaxIter, it;
    double alpha_prev = 1.0, alpha = 0.0;
    bool pending = false;  // a step (alpha, dU, dX, dsig, dt, dl) waits to be applied by S1
    // the sweeps in this agent's current precision (the fp32 instantiations exist only when MIXED)
    auto run1 = [&](bool apply, double al) -> S1Out {
        if constexpr (MIXED) {
            if (f32) return sweep1(0.0f, apply, al);
        }
        return sweep1(0.0, apply, al);
    };
    auto run_fwd = [&](int pass, double sm) -> FwdOut {
        if constexpr (MIXED) {
            if (f32) return sweep_fwd(0.0f, pass, sm);
        }
        return sweep_fwd(0.0, pass, sm);
    };
    auto run3 = [&](double sm) {
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
            for (int i = 0; i < c.n; ++i) bU[i] = U[i];
            for (int i = 0; i < N * NS; ++i) bsig[i] = sig[i];
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
                const bool act = R < ms ? __builtin_isfinite(gh[R]) : __builtin_isfinite(w_in(((R - ms) >> 1) % NU, (R - ms) & 1));
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
            for (int i = 0; i < c.n; ++i) U[i] = bU[i];
            for (int i = 0; i < N * NS; ++i) sig[i] = bsig[i];
            kkt = best_kkt;
        }
        status = stop_status(stop, best_m, tol);
    }
    // ---- output: exact re-simulation of the states from U, slacks, inputs, input increments ----
    const int nxe = NX + NS;
    const size_t nz = (size_t)nxe * (N + 1) + 2 * (size_t)c.n;
    double* z = P.z + (size_t)b * nz;
    double x[NX];
#pragma unroll
    for (int s = 0; s < NX; ++s) {
        x[s] = x0[s];
        z[s] = x[s];
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) z[NX + j] = 0.0;
    for (int k = 0; k < N; ++k) {
        double A[NX * NX], Bm[NX * NU], u[NU];
        loadA(k, A);
        loadB(k, Bm);
#pragma unroll
        for (int i = 0; i < NU; ++i) u[i] = U[k * NU + i];
        double xn[NX];
#pragma unroll
        for (int s = 0; s < NX; ++s) {
            double v = 0.0;
#pragma unroll
            for (int q = 0; q < NX; ++q) v += A[s * NX + q] * x[q];
#pragma unroll
            for (int i = 0; i < NU; ++i) v += Bm[s * NU + i] * u[i];
            xn[s] = v;
        }
#pragma unroll
        for (int s = 0; s < NX; ++s) {
            x[s] = xn[s];
            z[(size_t)(k + 1) * nxe + s] = x[s];
        }
#pragma unroll
        for (int j = 0; j < NS; ++j) z[(size_t)(k + 1) * nxe + NX + j] = sig[k * NS + j];
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            z[(size_t)(N + 1) * nxe + k * NU + i] = u[i];
            z[(size_t)(N + 1) * nxe + c.n + k * NU + i] = u[i] - (k ? U[(k - 1) * NU + i] : up[i]);
        }
    }
    if (P.kkt) P.kkt[b] = kkt;
    if (P.iters) P.iters[b] = it;
    if (P.status) P.status[b] = status;
}

}  // namespace cmpc
