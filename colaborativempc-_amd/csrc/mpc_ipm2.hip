// Specialised batched condensed IPM ("v2"): same algorithm and results as the
// generic kernel in mpc_ipm.hip (the QP of PlannerLPV.solve, reference
// planner/lib/plan_lib/distributedPlanner/LPV_Planner.py:279-475), laid out for
// latency on CDNA4 with compile-time (NX, NU, MC) and T = ceil(N*NU/16) tiles:
//
//  * one 64-lane wavefront per agent; every per-agent input (A_k, B_k, C_k,
//    qlin, x0, u_prev) is staged into LDS once, and the LDS footprint is kept
//    under 40 KB so four agents share a CU (1024 agents resident on 256 CUs);
//  * lane k owns the constraint rows of stage k+1 (and input rows of u_k) in
//    registers, so every slack-group Schur term is lane-local;
//  * K = Gamma' W Gamma + ... is accumulated on V_MFMA_F64_16X16X4_F64 and
//    never leaves the accumulator registers: a blocked right-looking Cholesky
//    (16x16 diagonal factor by lane-per-row readlane broadcast, panel TRSM by
//    substitution, trailing SYRK on MFMA) factors it in place, and the
//    triangular solves run block-wise on the register tiles;
//  * the dynamics recursions (x_{k+1} = A x + B u, adjoint) broadcast the
//    state vector with v_readlane instead of LDS round trips.
#include <cmath>

#include "internal.h"
#include "wave_ops.h"

namespace cmpc {

struct Lds2 {
    int A, B, C, H, Pq, x0, up, W, X, dX, yb0, U, dU, rd, gU, vb, thin, bU, G0, G1, Y, S0, SP, red, total;
};

template <int T, int NX, int NU, int MC>
__host__ __device__ inline Lds2 lds2_layout(int N) {
    constexpr int NP = 16 * T, NXP = (NX + 3) & ~3;
    Lds2 L;
    int o = 0;
    auto take = [&](int cnt) {
        int r = o;
        o += (cnt + 1) & ~1;
        return r;
    };
    L.A = take(N * NX * NX);
    L.B = take(N * NX * NU);
    L.C = take(N * MC * NX);
    L.H = take(N * MC);
    L.Pq = take((N + 1) * NX);
    L.x0 = take(NX);
    L.up = take(NU);
    L.W = take(N * NX * NX);
    L.X = take((N + 1) * NX);
    L.dX = take((N + 1) * NX);  // also the second adjoint input (yb1) during residuals
    L.yb0 = take((N + 1) * NX);
    L.U = take(NP);
    L.dU = take(NP);
    L.rd = take(NP);
    L.gU = take(NP);
    L.vb = take(NP);
    L.thin = take(NP);
    L.bU = take(NP);
    L.G0 = take(NXP * NP);
    L.G1 = take(NXP * NP);
    L.Y = take(NXP * NP);
    L.S0 = take(16 * 17);
    L.SP = take(16 * 17 * (T > 1 ? T - 1 : 1));
    L.red = take(64);
    L.total = o;
    return L;
}

// x_0 = x0 (LDS, or 0), x_{k+1} = A_k x_k + B_k u_k ; lane s < NX carries x_s, broadcast by readlane
template <int NX, int NU>
__device__ __forceinline__ void fwd2(int N, const double* A, const double* B, const double* x0, const double* U,
                                     double* X) {
    const int l = threadIdx.x;
    const int s = l < NX ? l : 0;
    double xr = x0 ? x0[s] : 0.0;
    if (l < NX) X[l] = xr;
    for (int k = 0; k < N; ++k) {
        const double* Ak = A + (k * NX + s) * NX;
        const double* Bk = B + (k * NX + s) * NU;
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < NU; ++i) v = fma(Bk[i], U[k * NU + i], v);
#pragma unroll
        for (int t = 0; t < NX; ++t) v = fma(Ak[t], readlane_d(xr, t), v);
        xr = v;
        if (l < NX) X[(k + 1) * NX + l] = v;
    }
}

// Two adjoints at once (lanes 0-31 on y0 -> o0, lanes 32-63 on y1 -> o1):
// o_k = B_k' psi_{k+1}, psi_N = y_N, psi_k = y_k + A_k' psi_{k+1}.
template <int NX, int NU>
__device__ __forceinline__ void adj2(int N, const double* A, const double* B, const double* y0, const double* y1,
                                     double* o0, double* o1) {
    const int l = threadIdx.x, h = l >> 5, s = l & 31;
    const int sx = s < NX ? s : 0;
    const double* y = h ? y1 : y0;
    double* o = h ? o1 : o0;
    double pr = y[N * NX + sx];
    for (int k = N - 1; k >= 0; --k) {
        double ps[NX];
#pragma unroll
        for (int t = 0; t < NX; ++t) {
            const double a0 = readlane_d(pr, t), a1 = readlane_d(pr, 32 + t);
            ps[t] = h ? a1 : a0;
        }
        if (s < NU) {
            double v = 0.0;
#pragma unroll
            for (int t = 0; t < NX; ++t) v = fma(B[(k * NX + t) * NU + s], ps[t], v);
            o[k * NU + s] = v;
        }
        if (k > 0) {
            double v = y[k * NX + sx];
#pragma unroll
            for (int t = 0; t < NX; ++t) v = fma(A[(k * NX + t) * NX + sx], ps[t], v);
            pr = v;
        }
    }
}

template <int T, int NX, int NU, int MC>
__global__ __launch_bounds__(64, 1) void mpc_ipm2_kernel(const MpcConst c, const MpcPtrs P) {
    constexpr int NS = 3, NT = T * (T + 1) / 2, NP = 16 * T, NXP = (NX + 3) & ~3, RX = MC + 2 * NU;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int l = threadIdx.x, b = blockIdx.x, N = c.N, n = N * NU, ms = N * MC;
    const Lds2 L = lds2_layout<T, NX, NU, MC>(N);
    double* sA = sm + L.A;
    double* sB = sm + L.B;
    double* sC = sm + L.C;
    double* sH = sm + L.H;
    double* sP = sm + L.Pq;
    double* sx0 = sm + L.x0;
    double* sup = sm + L.up;
    double* sW = sm + L.W;
    double* X = sm + L.X;
    double* dX = sm + L.dX;
    double* yb0 = sm + L.yb0;
    double* U = sm + L.U;
    double* dU = sm + L.dU;
    double* rd = sm + L.rd;
    double* gU = sm + L.gU;
    double* vb = sm + L.vb;
    double* thin = sm + L.thin;
    double* bU = sm + L.bU;
    double* S0 = sm + L.S0;
    double* SP = sm + L.SP;
    double* red = sm + L.red;
    const bool stamp = P.stamps != nullptr && !c.debug;
    unsigned long long tsum[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long t_a = stamp ? clock64_() : 0, t_b = 0;
#define STAMP(slot)                        \
    if (stamp) {                           \
        t_b = clock64_();                  \
        tsum[slot] += t_b - t_a;           \
        t_a = t_b;                         \
    }

    // ---------------- stage the agent's data into LDS ----------------
    {
        const double* gA = P.A + (size_t)b * N * NX * NX;
        const double* gB = P.B + (size_t)b * N * NX * NU;
        const double* gC = P.C + (size_t)b * N * MC * NX;
        const double* gP = P.p + (size_t)b * (N + 1) * NX;
        for (int i = l; i < N * NX * NX; i += 64) sA[i] = gA[i];
        for (int i = l; i < N * NX * NU; i += 64) sB[i] = gB[i];
        for (int i = l; i < N * MC * NX; i += 64) sC[i] = gC[i];
        for (int i = l; i < N * MC; i += 64) sH[i] = P.h[(size_t)b * ms + i];
        for (int i = l; i < (N + 1) * NX; i += 64) sP[i] = gP[i];
        if (l < NX) sx0[l] = P.x0[(size_t)b * NX + l];
        if (l < NU) sup[l] = P.up[(size_t)b * NU + l];
        for (int i = l; i < NP; i += 64) {
            U[i] = 0.0;
            dU[i] = 0.0;
            vb[i] = 0.0;
            thin[i] = 0.0;
        }
    }
    // ---- rows owned by this lane: stage k+1 state rows (r < MC) and input rows of u_k ----
    const bool own = l < N;
    const int k = own ? l : 0;
    double t[RX], lam[RX], rp[RX], rho[RX], dtdl[RX], gdu[RX];
    unsigned actm = 0;  // bit r: row r of this lane is active (finite bound)
    auto wv = [&](int r) -> double {
        if (r < MC) return sH[k * MC + r];
        const int q = r - MC, i = q >> 1;
        return (q & 1) ? -c.u_lb[i] : c.u_ub[i];
    };
    double sg[NS] = {0.0, 0.0, 0.0};
    bar();
    if (own) {
#pragma unroll
        for (int r = 0; r < RX; ++r)
            if (isfinite(wv(r))) actm |= 1u << r;
    }
#define ACT(r) ((actm >> (r)) & 1u)
    fwd2<NX, NU>(N, sA, sB, sx0, U, X);
    bar();

    // row value at (X, U, sig) for this lane's rows
    auto rowval = [&](int r, const double* Xv, const double* Uv, bool with_sig) -> double {
        if (r < MC) {
            const double* cr = sC + (k * MC + r) * NX;
            const double* xk = Xv + (k + 1) * NX;
            double v = 0.0;
#pragma unroll
            for (int s = 0; s < NX; ++s) v = fma(cr[s], xk[s], v);
            const int j = c.row_slack[r];
            if (with_sig && j >= 0) v += c.row_sign[r] * sg[j];
            return v;
        }
        const int q = r - MC;
        const double u = Uv[k * NU + (q >> 1)];
        return (q & 1) ? -u : u;
    };

    double mact_l = 0.0, sp_l = 1.0;
#pragma unroll
    for (int r = 0; r < RX; ++r) {
        if (ACT(r)) {
            const double w = wv(r);
            t[r] = fmax(w - rowval(r, X, U, true), 1.0);
            lam[r] = 1.0;
            mact_l += 1.0;
            sp_l = fmax(sp_l, fabs(w));
        } else {
            t[r] = 1.0;
            lam[r] = 0.0;
        }
        dtdl[r] = rp[r] = rho[r] = gdu[r] = 0.0;
    }
    const double mact = fmax(wave_sum(mact_l), 1.0);
    const double scale_p = wave_max(sp_l);
    STAMP(0);

    // best iterate by merit max(res, 1e4 mu) (< tol <=> converged), returned when the method
    // stops short of convergence (iteration cap, factorisation breakdown, stagnation)
    double best_m = INFINITY, best_kkt = INFINITY, bsg[NS] = {0.0, 0.0, 0.0};
    int best_it = 0, stop = kStopMaxIter, it;
    double kkt = INFINITY;
    double th[RX], Dsig[NS], rsig[NS];
    v4d acc[NT];
    double Lrow[16], Lcol[16];
    for (it = 1; it <= c.max_iter; ++it) {
        // ================= residuals =================
        for (int i = l; i < (N + 1) * NX; i += 64) {
            const int kk = i / NX, s = i - kk * NX;
            double v = 2.0 * sP[i];
#pragma unroll
            for (int u = 0; u < NX; ++u) v = fma(2.0 * c.Q[s * NX + u], X[kk * NX + u], v);
            yb0[i] = v;
        }
        bar();
        // yb1 (in dX) = yb0 + C' lambda on stages 1..N
        if (own) {
#pragma unroll
            for (int s = 0; s < NX; ++s) {
                double v = yb0[(k + 1) * NX + s];
#pragma unroll
                for (int r = 0; r < MC; ++r) v = fma(lam[r], sC[(k * MC + r) * NX + s], v);
                dX[(k + 1) * NX + s] = v;
            }
        }
        if (l < NX) dX[l] = yb0[l];
        bar();
        adj2<NX, NU>(N, sA, sB, yb0, dX, gU, rd);
        bar();
        double gs_l = 1.0, nrd_l = 0.0, nrs_l = 0.0, nrp_l = 0.0, mu_l = 0.0;
        if (own) {
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                const int ci = k * NU + i;
                double v = 0.0;
#pragma unroll
                for (int j = 0; j < NU; ++j) {
                    const double uk = U[k * NU + j];
                    const double duk = uk - (k ? U[(k - 1) * NU + j] : sup[j]);
                    const double dun = (k + 1 < N) ? U[(k + 1) * NU + j] - uk : 0.0;
                    v += 2.0 * c.R[i * NU + j] * uk + 2.0 * c.dR[i * NU + j] * (duk - dun);
                }
                const double g = gU[ci] + v;
                const double rdv = rd[ci] + v + lam[MC + 2 * i] - lam[MC + 2 * i + 1];
                rd[ci] = rdv;
                gs_l = nmax(gs_l, fabs(g));
                nrd_l = nmax(nrd_l, fabs(rdv));
            }
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                double v = 2.0 * c.Qs[j] * sg[j];
#pragma unroll
                for (int r = 0; r < MC; ++r)
                    if (c.row_slack[r] == j) v += c.row_sign[r] * lam[r];
                rsig[j] = v;
                nrs_l = nmax(nrs_l, fabs(v));
            }
        }
#pragma unroll
        for (int r = 0; r < RX; ++r) {
            if (ACT(r)) {
                rp[r] = rowval(r, X, U, true) + t[r] - wv(r);
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
        STAMP(0);
        const double merit = nmax(res, 1e4 * mu);
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

        // ================= Newton matrix K = Gamma' W Gamma + Hc + diag =================
#pragma unroll
        for (int r = 0; r < RX; ++r) th[r] = ACT(r) ? lam[r] / t[r] : 0.0;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            double v = 2.0 * c.Qs[j];
#pragma unroll
            for (int r = 0; r < MC; ++r)
                if (c.row_slack[r] == j) v += th[r];
            Dsig[j] = v;
        }
        if (own) {
            // W_{k+1} = 2Q + sum_r th'_r c_r c_r' + sum_{pairs in a slack group} phi (a_r - a_r')(a_r - a_r')'
            double thp[MC];
#pragma unroll
            for (int r = 0; r < MC; ++r) {
                const int j = c.row_slack[r];
                thp[r] = j < 0 ? th[r] : 2.0 * c.Qs[j] * th[r] / Dsig[j];
            }
            const double* Ck = sC + k * MC * NX;
            for (int s = 0; s < NX; ++s)
                for (int u = 0; u < NX; ++u) {
                    double v = 2.0 * c.Q[s * NX + u];
#pragma unroll
                    for (int r = 0; r < MC; ++r) v = fma(thp[r] * Ck[r * NX + s], Ck[r * NX + u], v);
#pragma unroll
                    for (int r = 0; r < MC; ++r) {
                        const int j = c.row_slack[r];
                        if (j < 0) continue;
#pragma unroll
                        for (int r2 = r + 1; r2 < MC; ++r2) {
                            if (c.row_slack[r2] != j) continue;
                            const double s1 = c.row_sign[r], s2 = c.row_sign[r2];
                            const double phi = th[r] * th[r2] / Dsig[j];
                            const double ds = s1 * Ck[r * NX + s] - s2 * Ck[r2 * NX + s];
                            const double du = s1 * Ck[r * NX + u] - s2 * Ck[r2 * NX + u];
                            v = fma(phi * ds, du, v);
                        }
                    }
                    sW[(k * NX + s) * NX + u] = v;
                }
#pragma unroll
            for (int i = 0; i < NU; ++i) thin[k * NU + i] = th[MC + 2 * i] + th[MC + 2 * i + 1];
        }
        double* G0 = sm + L.G0;
        double* G1 = sm + L.G1;
        double* Y = sm + L.Y;
        for (int i = l; i < 3 * NXP * NP; i += 64) G0[i] = 0.0;  // G0, G1, Y contiguous
        bar();
#pragma unroll
        for (int q = 0; q < NT; ++q) acc[q] = v4d{0.0, 0.0, 0.0, 0.0};
        double* gc = G0;
        double* gn = G1;
        for (int kk = 0; kk < N; ++kk) {
            const int ncol = (kk + 1) * NU;
            const double* Ak = sA + kk * NX * NX;
            const double* Bk = sB + kk * NX * NU;
            for (int i = l; i < NX * ncol; i += 64) {
                const int s = i / ncol, col = i - s * ncol;
                double v = 0.0;
#pragma unroll
                for (int u = 0; u < NX; ++u) v = fma(Ak[s * NX + u], gc[u * NP + col], v);
                if (col >= kk * NU) v += Bk[s * NU + (col - kk * NU)];
                gn[s * NP + col] = v;
            }
            bar();
            const double* Wk = sW + kk * NX * NX;
            for (int i = l; i < NX * ncol; i += 64) {
                const int s = i / ncol, col = i - s * ncol;
                double v = 0.0;
#pragma unroll
                for (int u = 0; u < NX; ++u) v = fma(Wk[s * NX + u], gn[u * NP + col], v);
                Y[s * NP + col] = v;
            }
            bar();
#pragma unroll
            for (int q = 0; q < NXP; q += 4) {
                const int row = q + (l >> 4);
                double af[T], bf[T];
#pragma unroll
                for (int ti = 0; ti < T; ++ti) {
                    af[ti] = gn[row * NP + ti * 16 + (l & 15)];
                    bf[ti] = Y[row * NP + ti * 16 + (l & 15)];
                }
                // Branch-free on purpose: tiles beyond ncol multiply zeros.  A data-dependent skip here
                // let the compiler read the f64 MFMA result (v_accvgpr_read) on the skip path with too
                // few wait states (hazard padding sized for the fall-through path) -> stale high dwords.
#pragma unroll
                for (int ti = 0; ti < T; ++ti)
#pragma unroll
                    for (int tj = 0; tj <= ti; ++tj)
                        acc[ti * (ti + 1) / 2 + tj] =
                            __builtin_amdgcn_mfma_f64_16x16x4f64(af[ti], bf[tj], acc[ti * (ti + 1) / 2 + tj], 0, 0, 0);
            }
            double* tq = gc;
            gc = gn;
            gn = tq;
        }
        // + 2R + 2D'dR D (block tridiagonal) + input-row curvature; identity on the padding
#pragma unroll
        for (int ti = 0; ti < T; ++ti)
#pragma unroll
            for (int tj = 0; tj <= ti; ++tj)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = ti * 16 + (l >> 4) + 4 * r, col = tj * 16 + (l & 15);
                    double add = 0.0;
                    if (row < n && col < n) {
                        const int kr = row / NU, a = row - kr * NU, kc = col / NU, bq = col - kc * NU;
                        if (kr == kc)
                            add = 2.0 * c.R[a * NU + bq] + 2.0 * c.dR[a * NU + bq] * (kr + 1 < N ? 2.0 : 1.0) +
                                  (row == col ? thin[row] : 0.0);
                        else if (kr == kc + 1 || kc == kr + 1)
                            add = -2.0 * c.dR[a * NU + bq];
                    } else if (row == col) {
                        add = 1.0;
                    }
                    acc[ti * (ti + 1) / 2 + tj][r] += add;
                }
        STAMP(1);
        if (c.debug && it == 1 && P.stamps) {  // diagnostic: dump K (NP x NP, row-major) to the stamps buffer
            double* dk = reinterpret_cast<double*>(P.stamps) + (size_t)b * NP * NP;
#pragma unroll
            for (int ti = 0; ti < T; ++ti)
#pragma unroll
                for (int tj = 0; tj <= ti; ++tj)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        dk[(ti * 16 + (l >> 4) + 4 * r) * NP + tj * 16 + (l & 15)] = acc[ti * (ti + 1) / 2 + tj][r];
        }

        // ================= blocked Cholesky in the accumulator registers =================
        bool chol_ok = true;
#pragma unroll
        for (int J = 0; J < T; ++J) {
            const int JJ = J * (J + 1) / 2 + J;
#pragma unroll
            for (int r = 0; r < 4; ++r) S0[((l >> 4) + 4 * r) * 17 + (l & 15)] = acc[JJ][r];
            bar();
            double rw[16];
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) rw[cc] = S0[(l & 15) * 17 + cc];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const double djj = readlane_d(rw[j], j);
                if (!(djj > 0.0)) chol_ok = false;
                const double d = sqrt(djj);
                const double lj = (l > j) ? rw[j] / d : ((l == j) ? d : rw[j]);
                rw[j] = lj;
#pragma unroll
                for (int cc = j + 1; cc < 16; ++cc) rw[cc] = fma(-lj, readlane_d(lj, cc), rw[cc]);
            }
            bar();
            if (l < 16) {
#pragma unroll
                for (int cc = 0; cc < 16; ++cc) S0[l * 17 + cc] = (cc <= l) ? rw[cc] : 0.0;
            }
            bar();
            if ((l >> 4) == J) {
#pragma unroll
                for (int cc = 0; cc < 16; ++cc) {
                    Lrow[cc] = S0[(l & 15) * 17 + cc];
                    Lcol[cc] = S0[cc * 17 + (l & 15)];
                }
            }
            if (J + 1 < T) {
                // panel TRSM: L_IJ = K_IJ L_JJ^{-T}, one lane per stacked panel row
#pragma unroll
                for (int I = J + 1; I < T; ++I)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        SP[((I - J - 1) * 16 + (l >> 4) + 4 * r) * 17 + (l & 15)] = acc[I * (I + 1) / 2 + J][r];
                bar();
                if (l < 16 * (T - 1 - J)) {
                    double* yrow = SP + l * 17;  // this lane's stacked panel row, solved in place
#pragma unroll 1
                    for (int cc = 0; cc < 16; ++cc) {
                        double v = yrow[cc];
                        for (int p = 0; p < cc; ++p) v = fma(-S0[cc * 17 + p], yrow[p], v);
                        yrow[cc] = v / S0[cc * 17 + cc];
                    }
                }
                bar();
#pragma unroll
                for (int I = J + 1; I < T; ++I)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[I * (I + 1) / 2 + J][r] = SP[((I - J - 1) * 16 + (l >> 4) + 4 * r) * 17 + (l & 15)];
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
                bar();
            }
        }
        STAMP(2);
        if (!chol_ok) {
            stop = kStopBreakdown;
            break;
        }
        // inverse diagonal of the owning block row, for the in-block substitutions
        const double Ldinv = 1.0 / Lrow[l & 15];

        // ================= predictor / corrector =================
        double sig_c = 0.0, alpha = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
            for (int r = 0; r < RX; ++r) {
                if (!ACT(r)) {
                    rho[r] = 0.0;
                    continue;
                }
                double rc = -t[r] * lam[r];
                if (pass) rc += sig_c * mu - dtdl[r];
                rho[r] = (rc + lam[r] * rp[r]) / t[r];
            }
            // rho~ (stable slack-group form) enters only through C' rho~ and the input rows
            auto rtil = [&](int r) -> double {
                double v = rho[r];
                if (r < MC) {
                    const int j = c.row_slack[r];
                    if (j >= 0) {
                        v = 2.0 * c.Qs[j] * rho[r] - th[r] * c.row_sign[r] * rsig[j];
#pragma unroll
                        for (int r2 = 0; r2 < MC; ++r2) {
                            if (r2 == r || c.row_slack[r2] != j) continue;
                            v += th[r2] * rho[r] - th[r] * c.row_sign[r] * c.row_sign[r2] * rho[r2];
                        }
                        v /= Dsig[j];
                    }
                }
                return v;
            };
            if (own) {
                double ybv[NX];
#pragma unroll
                for (int s = 0; s < NX; ++s) ybv[s] = 0.0;
#pragma unroll
                for (int r = 0; r < MC; ++r) {
                    const double rr = rtil(r);
#pragma unroll
                    for (int s = 0; s < NX; ++s) ybv[s] = fma(rr, sC[(k * MC + r) * NX + s], ybv[s]);
                }
#pragma unroll
                for (int s = 0; s < NX; ++s) yb0[(k + 1) * NX + s] = ybv[s];
            }
            if (l < NX) yb0[l] = 0.0;
            bar();
            adj2<NX, NU>(N, sA, sB, yb0, yb0, vb, vb);
            bar();
            if (own) {
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    const int ci = k * NU + i;
                    vb[ci] = -rd[ci] - (vb[ci] + rho[MC + 2 * i] - rho[MC + 2 * i + 1]);
                }
            }
            bar();
            // ---- forward solve L y = vb (block rows; L_JI tiles in acc, L_JJ rows in Lrow) ----
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
                    bar();
                }
                double rv = 0.0;
                if ((l >> 4) == J) rv = vb[J * 16 + (l & 15)] - (J > 0 ? red[l & 15] : 0.0);
#pragma unroll
                for (int cc = 0; cc < 16; ++cc) {
                    if ((l & 15) == cc) rv *= Ldinv;
                    const double ycc = readlane_d(rv, 16 * J + cc);
                    if ((l & 15) > cc) rv = fma(-Lrow[cc], ycc, rv);
                }
                if ((l >> 4) == J) vb[J * 16 + (l & 15)] = rv;
                bar();
            }
            // ---- backward solve L' x = y ----
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
#pragma unroll
                for (int cc = 15; cc >= 0; --cc) {
                    if ((l & 15) == cc) rv *= Ldinv;
                    const double xcc = readlane_d(rv, 16 * J + cc);
                    if ((l & 15) < cc) rv = fma(-Lcol[cc], xcc, rv);
                }
                if ((l >> 4) == J) vb[J * 16 + (l & 15)] = rv;
                bar();
            }
            for (int i = l; i < NP; i += 64) dU[i] = (i < n) ? vb[i] : 0.0;
            bar();
            fwd2<NX, NU>(N, sA, sB, nullptr, dU, dX);
            bar();
            double dsg[NS];
#pragma unroll
            for (int r = 0; r < RX; ++r) gdu[r] = ACT(r) ? rowval(r, dX, dU, false) : 0.0;
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                double v = rsig[j];
#pragma unroll
                for (int r = 0; r < MC; ++r)
                    if (c.row_slack[r] == j) v += c.row_sign[r] * (rho[r] + th[r] * gdu[r]);
                dsg[j] = own ? -v / Dsig[j] : 0.0;
            }
            // dt_r = -rp - G dU - s dsig ;  dl_r = rho + th (G dU + s dsig)
            auto sdr = [&](int r) -> double {
                if (r < MC) {
                    const int j = c.row_slack[r];
                    if (j >= 0) return c.row_sign[r] * dsg[j];
                }
                return 0.0;
            };
            double amax_l = 1.0e300;
#pragma unroll
            for (int r = 0; r < RX; ++r) {
                if (!ACT(r)) continue;
                const double sd = sdr(r);
                const double dtv = -rp[r] - gdu[r] - sd;
                const double dlv = rho[r] + th[r] * (gdu[r] + sd);
                if (dtv < 0.0) amax_l = fmin(amax_l, -t[r] / dtv);
                if (dlv < 0.0) amax_l = fmin(amax_l, -lam[r] / dlv);
            }
            const double amax = wave_min(amax_l);
            if (!pass) {
                const double a = fmin(amax, 1.0);
                double mua_l = 0.0;
#pragma unroll
                for (int r = 0; r < RX; ++r) {
                    if (!ACT(r)) {
                        dtdl[r] = 0.0;
                        continue;
                    }
                    const double sd = sdr(r);
                    const double dtv = -rp[r] - gdu[r] - sd;
                    const double dlv = rho[r] + th[r] * (gdu[r] + sd);
                    mua_l += (t[r] + a * dtv) * (lam[r] + a * dlv);
                    dtdl[r] = dtv * dlv;
                }
                const double mu_aff = wave_sum(mua_l) / mact;
                const double ratio = mu > 0.0 ? mu_aff / mu : 0.0;
                sig_c = ratio * ratio * ratio;
                STAMP(3);
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
                STAMP(4);
            }
        }
        for (int i = l; i < n; i += 64) U[i] = fma(alpha, dU[i], U[i]);
        for (int i = l; i < (N + 1) * NX; i += 64) X[i] = fma(alpha, dX[i], X[i]);
        bar();
        STAMP(5);
    }
    if (it > c.max_iter) it = c.max_iter;
    bar();
    int status = CMPC_SOLVED;
    if (stop != kStopConverged) {
        if (best_it > 0) {  // restore the best iterate
            for (int i = l; i < NP; i += 64) U[i] = bU[i];
#pragma unroll
            for (int j = 0; j < NS; ++j) sg[j] = bsg[j];
            kkt = best_kkt;
        }
        status = stop_status(stop, best_m, c.tol);
    }
    bar();

    // ---- output in the reference layout ----
    fwd2<NX, NU>(N, sA, sB, sx0, U, X);
    bar();
    constexpr int NXE = NX + NS;
    const size_t nz = (size_t)NXE * (N + 1) + 2 * (size_t)n;
    double* z = P.z + (size_t)b * nz;
    for (int i = l; i < (N + 1) * NX; i += 64) {
        const int kk = i / NX, s = i - kk * NX;
        z[kk * NXE + s] = X[i];
    }
    if (l < NS) z[NX + l] = 0.0;
    if (own) {
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
        if (stamp) {
            unsigned long long* st = P.stamps + (size_t)b * 8;
            for (int i = 0; i < 6; ++i) st[i] = tsum[i];
            st[6] = it;
        }
    }
#undef STAMP
#undef ACT
}

template <int T, int NX, int NU, int MC>
static hipError_t launch2(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s) {
    const size_t lds = sizeof(double) * (size_t)lds2_layout<T, NX, NU, MC>(c.N).total;
    hipError_t e = hipFuncSetAttribute((const void*)mpc_ipm2_kernel<T, NX, NU, MC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((mpc_ipm2_kernel<T, NX, NU, MC>), dim3(batch), dim3(64), lds, s, c, p);
    return hipGetLastError();
}

template <int NX, int NU, int MC>
static hipError_t launch2_t(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s) {
    switch (c.npad / 16) {
        case 1: return launch2<1, NX, NU, MC>(c, p, batch, s);
        case 2: return launch2<2, NX, NU, MC>(c, p, batch, s);
        case 3: return launch2<3, NX, NU, MC>(c, p, batch, s);
        default: return launch2<4, NX, NU, MC>(c, p, batch, s);
    }
}

// Returns true (and launches) when a specialised instantiation covers the problem.
bool mpc2_try_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err) {
    if (c.ns != 3 || c.N > 64) return false;
#define CASE(NX_, NU_, MC_)                                 \
    if (c.nx == NX_ && c.nu == NU_ && c.mc == MC_) {        \
        *err = launch2_t<NX_, NU_, MC_>(c, p, batch, s);    \
        return true;                                        \
    }
    CASE(4, 2, 6)
#ifndef CMPC_V2_QUICK
    CASE(4, 2, 5)
    CASE(4, 2, 4)
    CASE(9, 2, 6)
    CASE(9, 2, 5)
    CASE(9, 2, 4)
    CASE(6, 3, 6)
#endif
#undef CASE
    return false;
}

}  // namespace cmpc
