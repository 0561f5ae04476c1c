// Batched condensed interior-point solver for the structured LTV agent-QP.
//
// One 64-lane wavefront (= one workgroup) solves one agent's QP — the QP that
// PlannerLPV.solve assembles (reference: planner/lib/plan_lib/distributedPlanner/
// LPV_Planner.py:279-475) and hands to OSQP (:192-249).  States are eliminated
// through the dynamics (X = xbar + Gamma U), the per-stage slacks through a
// diagonal Schur complement, and every interior-point iteration
//   1. forms  K = Gamma' W Gamma + 2R + 2D'dR D + diag(input rows)   (W = 2Q + M_k per stage)
//      by streaming Gamma_k stage by stage through LDS and accumulating the
//      16x16 output tiles with V_MFMA_F64_16X16X4_F64 (the only GEMM on the path);
//   2. factors K = L L' in LDS (one lane per row);
//   3. solves the Mehrotra predictor and corrector systems with the same factor,
//      using forward/adjoint recursions through the dynamics for G*v and G'*y.
//
// All arithmetic is fp64.  Control flow is wave-uniform: one wave == one agent,
// so agents that converge early simply retire their wave.
#include <cmath>

#include "internal.h"

namespace cmpc {

typedef double v4d __attribute__((ext_vector_type(4)));

struct Lds {
    int K, G0, G1, Y, W, X, dX, yb, psi, U, dU, rd, gU, sig, dsig, Dsig, rsig;
    int t, lam, th, rho, rt, rp, w, dta, dla, GdU, bU, bsig, red, total;
};

__host__ __device__ inline int lds_take(int& o, int cnt) {
    int r = o;
    o += (cnt + 1) & ~1;  // keep every region 16-byte aligned
    return r;
}

__host__ __device__ inline Lds lds_layout(const MpcConst& c) {
    Lds L;
    int o = 0;
    L.K = lds_take(o, c.n * c.ldk);
    L.G0 = lds_take(o, c.nxp * c.npad);
    L.G1 = lds_take(o, c.nxp * c.npad);
    L.Y = lds_take(o, c.nxp * c.npad);
    L.W = lds_take(o, c.nx * c.nx);
    L.X = lds_take(o, (c.N + 1) * c.nx);
    L.dX = lds_take(o, (c.N + 1) * c.nx);
    L.yb = lds_take(o, (c.N + 1) * c.nx);
    L.psi = lds_take(o, 2 * c.nx);
    L.U = lds_take(o, c.npad);
    L.dU = lds_take(o, c.npad);
    L.rd = lds_take(o, c.npad);
    L.gU = lds_take(o, c.npad);
    L.sig = lds_take(o, c.N * c.ns);
    L.dsig = lds_take(o, c.N * c.ns);
    L.Dsig = lds_take(o, c.N * c.ns);
    L.rsig = lds_take(o, c.N * c.ns);
    L.t = lds_take(o, c.m);
    L.lam = lds_take(o, c.m);
    L.th = lds_take(o, c.m);
    L.rho = lds_take(o, c.m);
    L.rt = lds_take(o, c.m);
    L.rp = lds_take(o, c.m);
    L.w = lds_take(o, c.m);
    L.dta = lds_take(o, c.m);
    L.dla = lds_take(o, c.m);
    L.GdU = lds_take(o, c.m);
    L.bU = lds_take(o, c.npad);
    L.bsig = lds_take(o, c.N * c.ns);
    L.red = lds_take(o, kWave);
    L.total = o;
    return L;
}

size_t mpc_lds_bytes(const MpcConst& c) { return sizeof(double) * (size_t)lds_layout(c).total; }

__device__ __forceinline__ void bar() { __syncthreads(); }

__device__ __forceinline__ double readlane_d(double v, int lane) {
    long long i = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(i & 0xffffffffll), lane);
    int hi = __builtin_amdgcn_readlane((int)(i >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// NaN-propagating max: a NaN residual must never look converged (fmax drops NaNs).
__device__ __forceinline__ double nmax(double a, double b) { return (a > b || a != a) ? a : b; }

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = nmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// X_0 = x0 (or 0), X_{k+1} = A_k X_k + B_k U_k
__device__ void fwd_sim(const MpcConst& c, const double* __restrict__ A, const double* __restrict__ B,
                        const double* __restrict__ x0, const double* U, double* X) {
    const int l = threadIdx.x, nx = c.nx, nu = c.nu;
    if (l < nx) X[l] = x0 ? x0[l] : 0.0;
    bar();
    for (int k = 0; k < c.N; ++k) {
        if (l < nx) {
            const double* Ak = A + ((size_t)k * nx + l) * nx;
            const double* Bk = B + ((size_t)k * nx + l) * nu;
            double v = 0.0;
            for (int t = 0; t < nx; ++t) v = fma(Ak[t], X[k * nx + t], v);
            for (int i = 0; i < nu; ++i) v = fma(Bk[i], U[k * nu + i], v);
            X[(k + 1) * nx + l] = v;
        }
        bar();
    }
}

// out_k = B_k' psi_{k+1}, psi_N = yb_N, psi_k = yb_k + A_k' psi_{k+1}   (out: n values)
__device__ void adjoint(const MpcConst& c, const double* __restrict__ A, const double* __restrict__ B,
                        const double* yb, double* out, double* psi2) {
    const int l = threadIdx.x, nx = c.nx, nu = c.nu, N = c.N;
    double* pa = psi2;
    double* pb = psi2 + nx;
    if (l < nx) pa[l] = yb[N * nx + l];
    bar();
    for (int k = N - 1; k >= 0; --k) {
        if (l < nu) {
            const double* Bk = B + (size_t)k * nx * nu;
            double v = 0.0;
            for (int s = 0; s < nx; ++s) v = fma(Bk[s * nu + l], pa[s], v);
            out[k * nu + l] = v;
        }
        if (k > 0 && l < nx) {
            const double* Ak = A + (size_t)k * nx * nx;
            double v = yb[k * nx + l];
            for (int s = 0; s < nx; ++s) v = fma(Ak[s * nx + l], pa[s], v);
            pb[l] = v;
        }
        bar();
        double* tq = pa;
        pa = pb;
        pb = tq;
    }
}

// Value of row r at (X, U, sig): state rows C_{k,r} . X_{k+1} (+ sign * sig), input rows +-U
__device__ __forceinline__ double row_value(const MpcConst& c, const double* __restrict__ C, int r,
                                            const double* X, const double* U, const double* sig) {
    if (r < c.ms) {
        const int k = r / c.mc, rr = r - k * c.mc;
        const double* cr = C + (size_t)r * c.nx;
        const double* xk = X + (k + 1) * c.nx;
        double v = 0.0;
        for (int s = 0; s < c.nx; ++s) v = fma(cr[s], xk[s], v);
        const int j = c.row_slack[rr];
        if (sig && j >= 0) v += c.row_sign[rr] * sig[k * c.ns + j];
        return v;
    }
    const int q = r - c.ms;
    const double u = U[q >> 1];
    return (q & 1) ? -u : u;
}

// 2R u_k + 2dR (du_k - du_{k+1}) for condensed variable index cidx (k*nu + i)
__device__ __forceinline__ double rdr_grad(const MpcConst& c, const double* U, const double* up, int cidx) {
    const int nu = c.nu, k = cidx / nu, i = cidx - k * nu;
    double v = 0.0;
    for (int j = 0; j < nu; ++j) {
        const double uk = U[k * nu + j];
        const double duk = uk - (k ? U[(k - 1) * nu + j] : up[j]);
        const double dun = (k + 1 < c.N) ? U[(k + 1) * nu + j] - uk : 0.0;
        v += 2.0 * c.R[i * nu + j] * uk + 2.0 * c.dR[i * nu + j] * (duk - dun);
    }
    return v;
}

// Entry (s,u) of the per-stage constraint curvature M_{k+1} (stable group Schur form):
//  no-slack rows:   th c c'
//  slack group j:   [q sum_r th_r c_r c_r' + sum_{r<r'} th_r th_r' (a_r - a_r')(a_r - a_r')'] / (q + sum th)
__device__ __forceinline__ double m_entry(const MpcConst& c, const double* __restrict__ Ck, const double* th_k,
                                          const double* Dsig_k, int s, int u) {
    const int nx = c.nx;
    double v = 0.0;
    for (int r = 0; r < c.mc; ++r) {
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
        for (int r2 = r + 1; r2 < c.mc; ++r2) {
            if (c.row_slack[r2] != j) continue;
            const double* c2 = Ck + r2 * nx;
            const double s2 = c.row_sign[r2];
            g += t1 * th_k[r2] * (s1 * c1[s] - s2 * c2[s]) * (s1 * c1[u] - s2 * c2[u]);
        }
        v = fma(g, inv, v);
    }
    return v;
}

template <int T>
__global__ __launch_bounds__(kWave) void mpc_ipm_kernel(const MpcConst c, const MpcPtrs P) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    constexpr int NT = T * (T + 1) / 2;
    const int b = blockIdx.x;
    const int l = threadIdx.x;
    const Lds L = lds_layout(c);
    const int nx = c.nx, nu = c.nu, N = c.N, ns = c.ns, mc = c.mc, n = c.n, ms = c.ms, m = c.m;
    const int npad = c.npad, ldk = c.ldk;

    const double* __restrict__ A = P.A + (size_t)b * N * nx * nx;
    const double* __restrict__ B = P.B + (size_t)b * N * nx * nu;
    const double* __restrict__ x0 = P.x0 + (size_t)b * nx;
    const double* __restrict__ up = P.up + (size_t)b * nu;
    const double* __restrict__ pl = P.p + (size_t)b * (N + 1) * nx;
    const double* __restrict__ C = P.C + (size_t)b * N * mc * nx;
    const double* __restrict__ h = P.h + (size_t)b * N * mc;

    double* K = sm + L.K;
    double* G0 = sm + L.G0;
    double* G1 = sm + L.G1;
    double* Y = sm + L.Y;
    double* W = sm + L.W;
    double* X = sm + L.X;
    double* dX = sm + L.dX;
    double* yb = sm + L.yb;
    double* psi = sm + L.psi;
    double* U = sm + L.U;
    double* dU = sm + L.dU;
    double* rd = sm + L.rd;
    double* gU = sm + L.gU;
    double* sig = sm + L.sig;
    double* dsig = sm + L.dsig;
    double* Dsig = sm + L.Dsig;
    double* rsig = sm + L.rsig;
    double* t = sm + L.t;
    double* lam = sm + L.lam;
    double* th = sm + L.th;
    double* rho = sm + L.rho;
    double* rt = sm + L.rt;
    double* rp = sm + L.rp;
    double* w = sm + L.w;
    double* dta = sm + L.dta;
    double* dla = sm + L.dla;
    double* GdU = sm + L.GdU;
    double* bU = sm + L.bU;
    double* bsig = sm + L.bsig;

    for (int i = l; i < L.total; i += kWave) sm[i] = 0.0;
    bar();

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
    bar();
    fwd_sim(c, A, B, x0, U, X);

    double mact_l = 0.0, sp_l = 1.0;
    for (int r = l; r < m; r += kWave) {
        if (isfinite(w[r])) {
            const double g = row_value(c, C, r, X, U, sig);
            t[r] = fmax(w[r] - g, kT0FloorCond);
            lam[r] = 1.0;
            mact_l += 1.0;
            sp_l = fmax(sp_l, fabs(w[r]));
        } else {
            t[r] = 1.0;
            lam[r] = 0.0;
        }
    }
    const double mact = fmax(wave_sum(mact_l), 1.0);
    const double scale_p = wave_max(sp_l);
    bar();

    // best iterate by merit max(res, 1e4 mu) (< tol <=> converged), returned when the method
    // stops short of convergence (iteration cap, factorisation breakdown, stagnation)
    double best_m = INFINITY, best_kkt = INFINITY;
    int best_it = 0, stop = kStopMaxIter, it;
    double kkt = INFINITY;
    double alpha_prev = 1;  // step of the previous iteration (kShortStep guard)
    for (it = 1; it <= c.max_iter; ++it) {
        // ================= residuals =================
        for (int i = l; i < (N + 1) * nx; i += kWave) {
            const int k = i / nx, s = i - k * nx;
            double v = 2.0 * pl[i];
            for (int u = 0; u < nx; ++u) v = fma(2.0 * c.Q[s * nx + u], X[k * nx + u], v);
            yb[i] = v;
        }
        bar();
        adjoint(c, A, B, yb, gU, psi);
        double gs_l = 1.0;
        for (int i = l; i < n; i += kWave) {
            gU[i] += rdr_grad(c, U, up, i);
            gs_l = nmax(gs_l, fabs(gU[i]));
        }
        const double gscale = wave_max(gs_l);
        for (int i = l; i < N * nx; i += kWave) {  // + C' lambda on stages 1..N
            const int k = i / nx, s = i - k * nx;
            double v = 0.0;
            for (int r = 0; r < mc; ++r) v = fma(lam[k * mc + r], C[((size_t)k * mc + r) * nx + s], v);
            yb[(k + 1) * nx + s] += v;
        }
        bar();
        adjoint(c, A, B, yb, rd, psi);
        double nrd_l = 0.0, nrs_l = 0.0, nrp_l = 0.0, mu_l = 0.0;
        for (int i = l; i < n; i += kWave) {
            const int r = ms + 2 * i;
            rd[i] += rdr_grad(c, U, up, i) + lam[r] - lam[r + 1];
            nrd_l = nmax(nrd_l, fabs(rd[i]));
        }
        for (int i = l; i < N * ns; i += kWave) {
            const int k = i / ns, j = i - k * ns;
            double v = 2.0 * c.Qs[j] * sig[i];
            for (int r = 0; r < mc; ++r)
                if (c.row_slack[r] == j) v += c.row_sign[r] * lam[k * mc + r];
            rsig[i] = v;
            nrs_l = nmax(nrs_l, fabs(v));
        }
        for (int r = l; r < m; r += kWave) {
            if (isfinite(w[r])) {
                const double v = row_value(c, C, r, X, U, sig) + t[r] - w[r];
                rp[r] = v;
                nrp_l = nmax(nrp_l, fabs(v));
                mu_l += t[r] * lam[r];
            } else {
                rp[r] = 0.0;
            }
        }
        const double mu = wave_sum(mu_l) / mact;
        // stationarity / feasibility relative; complementarity absolute and 1e4 tighter
        // (degenerate rows sit at t, lambda ~ sqrt(mu): primal accuracy needs tiny mu)
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
        if (merit < c.tol) {
            stop = kStopConverged;
            break;
        }
        if (best_m < 1e3 * c.tol && it - best_it >= kStallIters) {
            stop = kStopStalled;
            break;
        }
        bar();

        // ================= Newton matrix =================
        for (int r = l; r < m; r += kWave) th[r] = isfinite(w[r]) ? lam[r] / t[r] : 0.0;
        bar();
        for (int i = l; i < N * ns; i += kWave) {
            const int k = i / ns, j = i - k * ns;
            double v = 2.0 * c.Qs[j];
            for (int r = 0; r < mc; ++r)
                if (c.row_slack[r] == j) v += th[k * mc + r];
            Dsig[i] = v;
        }
        for (int i = l; i < 3 * c.nxp * npad; i += kWave) G0[i] = 0.0;  // G0,G1,Y contiguous
        bar();

        v4d acc[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) acc[q] = v4d{0.0, 0.0, 0.0, 0.0};
        double* gc = G0;
        double* gn = G1;
        for (int k = 0; k < N; ++k) {
            const int ncol = (k + 1) * nu;
            const double* Ak = A + (size_t)k * nx * nx;
            const double* Bk = B + (size_t)k * nx * nu;
            // Gamma_{k+1} = A_k Gamma_k + [0 .. B_k]
            for (int i = l; i < nx * ncol; i += kWave) {
                const int s = i / ncol, col = i - s * ncol;
                double v = 0.0;
                for (int u = 0; u < nx; ++u) v = fma(Ak[s * nx + u], gc[u * npad + col], v);
                if (col >= k * nu) v += Bk[s * nu + (col - k * nu)];
                gn[s * npad + col] = v;
            }
            // W = 2Q + M_{k+1}
            const double* Ck = C + (size_t)k * mc * nx;
            for (int i = l; i < nx * nx; i += kWave) {
                const int s = i / nx, u = i - s * nx;
                W[i] = 2.0 * c.Q[i] + m_entry(c, Ck, th + k * mc, Dsig + k * ns, s, u);
            }
            bar();
            // Y = W Gamma_{k+1}
            for (int i = l; i < nx * ncol; i += kWave) {
                const int s = i / ncol, col = i - s * ncol;
                double v = 0.0;
                for (int u = 0; u < nx; ++u) v = fma(W[s * nx + u], gn[u * npad + col], v);
                Y[s * npad + col] = v;
            }
            bar();
            // K += Gamma' Y  on f64 MFMA: A-frag = Gamma'[col][row] , B-frag = Y[row][col]
            for (int q = 0; q < c.nxp; q += 4) {
                const int row = q + (l >> 4);
                double af[T], bf[T];
#pragma unroll
                for (int ti = 0; ti < T; ++ti) {
                    af[ti] = gn[row * npad + ti * 16 + (l & 15)];
                    bf[ti] = Y[row * npad + ti * 16 + (l & 15)];
                }
#pragma unroll
                for (int ti = 0; ti < T; ++ti) {
                    if (ti * 16 < ncol) {
#pragma unroll
                        for (int tj = 0; tj <= ti; ++tj)
                            acc[ti * (ti + 1) / 2 + tj] =
                                __builtin_amdgcn_mfma_f64_16x16x4f64(af[ti], bf[tj], acc[ti * (ti + 1) / 2 + tj], 0, 0, 0);
                    }
                }
            }
            double* tq = gc;
            gc = gn;
            gn = tq;
        }
        // accumulator -> K (f64 16x16x4 C/D map: col = lane&15, row = (lane>>4) + 4*reg)
#pragma unroll
        for (int ti = 0; ti < T; ++ti)
#pragma unroll
            for (int tj = 0; tj <= ti; ++tj)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = ti * 16 + (l >> 4) + 4 * r, col = tj * 16 + (l & 15);
                    if (row < n && col < n) K[row * ldk + col] = acc[ti * (ti + 1) / 2 + tj][r];
                }
        bar();
        if (l < n) {
            const int k = l / nu, a = l - k * nu;
            for (int j = 0; j < nu; ++j) {
                const int col = k * nu + j;
                if (col <= l) K[l * ldk + col] += 2.0 * c.R[a * nu + j] + 2.0 * c.dR[a * nu + j] * (k + 1 < N ? 2.0 : 1.0);
                if (k > 0) K[l * ldk + (k - 1) * nu + j] -= 2.0 * c.dR[a * nu + j];
            }
            K[l * ldk + l] += th[ms + 2 * l] + th[ms + 2 * l + 1];
        }
        bar();

        // ================= Cholesky K = L L' (lane i owns row i) =================
        bool chol_ok = true;
        for (int j = 0; j < n; ++j) {
            double v = 0.0;
            if (l >= j && l < n) {
                v = K[l * ldk + j];
                const double* ri = K + l * ldk;
                const double* rj = K + j * ldk;
                for (int p = 0; p < j; ++p) v = fma(-ri[p], rj[p], v);
            }
            const double dj = readlane_d(v, j);
            if (!(dj > 0.0)) {
                chol_ok = false;
                break;
            }
            const double d = sqrt(dj);
            if (l == j) K[l * ldk + j] = d;
            else if (l > j && l < n) K[l * ldk + j] = v / d;
            bar();
        }
        if (!chol_ok) {
            stop = kStopBreakdown;
            if (c.rescue && P.ws) {  // hand the iterate to the Riccati rescue (hand_doubles)
                double* hd = P.ws + (size_t)b * c.ws_stride;
                const size_t ht = hand_t(c);
                if (l == 0) hd[1] = it - 1;
                for (int i = l; i < n; i += kWave) hd[2 + i] = U[i];
                for (int i = l; i < N * ns; i += kWave) hd[2 + n + i] = sig[i];
                for (int r = l; r < m; r += kWave) {
                    hd[ht + r] = t[r];
                    hd[ht + m + r] = lam[r];
                }
            }
            break;
        }

        // ================= predictor / corrector =================
        double sig_c = 0.0, alpha = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            for (int r = l; r < m; r += kWave) {
                if (!isfinite(w[r])) {
                    rho[r] = 0.0;
                    continue;
                }
                double rc = -t[r] * lam[r];
                if (pass) rc += sig_c * mu - dta[r] * dla[r];
                rho[r] = (rc + lam[r] * rp[r]) / t[r];
            }
            bar();
            for (int r = l; r < m; r += kWave) {
                double v = rho[r];
                if (r < ms) {
                    const int k = r / mc, rr = r - k * mc, j = c.row_slack[rr];
                    if (j >= 0) {
                        const double q = 2.0 * c.Qs[j];
                        v = q * rho[r] - th[r] * c.row_sign[rr] * rsig[k * ns + j];
                        for (int r2 = 0; r2 < mc; ++r2) {
                            if (r2 == rr || c.row_slack[r2] != j) continue;
                            const int R2 = k * mc + r2;
                            v += th[R2] * rho[r] - th[r] * c.row_sign[rr] * c.row_sign[r2] * rho[R2];
                        }
                        v /= Dsig[k * ns + j];
                    }
                }
                rt[r] = v;
            }
            bar();
            for (int i = l; i < (N + 1) * nx; i += kWave) {
                const int k = i / nx, s = i - k * nx;
                double v = 0.0;
                if (k > 0)
                    for (int r = 0; r < mc; ++r)
                        v = fma(rt[(k - 1) * mc + r], C[((size_t)(k - 1) * mc + r) * nx + s], v);
                yb[i] = v;
            }
            bar();
            adjoint(c, A, B, yb, dU, psi);
            // rhs = -rd - G' rt ; solve K dU = rhs with lane i holding entry i
            double bi = 0.0;
            if (l < n) bi = -rd[l] - (dU[l] + rt[ms + 2 * l] - rt[ms + 2 * l + 1]);
            for (int j = 0; j < n; ++j) {
                const double yj = readlane_d(bi, j) / K[j * ldk + j];
                if (l == j) bi = yj;
                else if (l > j && l < n) bi = fma(-K[l * ldk + j], yj, bi);
            }
            for (int j = n - 1; j >= 0; --j) {
                const double xj = readlane_d(bi, j) / K[j * ldk + j];
                if (l == j) bi = xj;
                else if (l < j) bi = fma(-K[j * ldk + l], xj, bi);
            }
            bar();
            if (l < n) dU[l] = bi;
            bar();
            fwd_sim(c, A, B, nullptr, dU, dX);
            for (int r = l; r < m; r += kWave) GdU[r] = row_value(c, C, r, dX, dU, nullptr);
            bar();
            for (int i = l; i < N * ns; i += kWave) {
                const int k = i / ns, j = i - k * ns;
                double v = rsig[i];
                for (int r = 0; r < mc; ++r)
                    if (c.row_slack[r] == j) {
                        const int R1 = k * mc + r;
                        v += c.row_sign[r] * (rho[R1] + th[R1] * GdU[R1]);
                    }
                dsig[i] = -v / Dsig[i];
            }
            bar();
            double amax_l = 1.0e300;
            double* dtp = pass ? rho : dta;  // corrector reuses rho/rt storage for (dt, dl)
            double* dlp = pass ? rt : dla;
            for (int r = l; r < m; r += kWave) {
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
            const double amax = fmin(wave_min(amax_l), 1.0e300);
            bar();
            if (!pass) {
                const double a = fmin(amax, 1.0);
                double mua_l = 0.0;
                for (int r = l; r < m; r += kWave)
                    if (isfinite(w[r])) mua_l += (t[r] + a * dta[r]) * (lam[r] + a * dla[r]);
                const double mu_aff = wave_sum(mua_l) / mact;
                const double ratio = mu > 0.0 ? mu_aff / mu : 0.0;
                sig_c = ratio * ratio;  // (the condensed kernels: e = 2, internal.h)
                if (alpha_prev < kShortStep) sig_c = fmax(sig_c, kSigmaMin);
            } else {
                alpha = fmin(1.0, 0.995 * amax);
                // stay in the wide neighbourhood t_r lam_r >= gamma mu(alpha) (see kNbhdGamma)
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
        }
        // ---- update (corrector direction: dU, dX, dsig, (rho, rt) = (dt, dl)) ----
        alpha_prev = alpha;
        for (int i = l; i < n; i += kWave) U[i] = fma(alpha, dU[i], U[i]);
        for (int i = l; i < N * ns; i += kWave) sig[i] = fma(alpha, dsig[i], sig[i]);
        for (int i = l; i < (N + 1) * nx; i += kWave) X[i] = fma(alpha, dX[i], X[i]);
        for (int r = l; r < m; r += kWave)
            if (isfinite(w[r])) {
                t[r] = fma(alpha, rho[r], t[r]);
                lam[r] = fma(alpha, rt[r], lam[r]);
            }
        bar();
    }
    if (it > c.max_iter) it = c.max_iter;
    bar();
    int status = CMPC_SOLVED;
    // a converged endpoint with a weakly active row (kPolishDegenerate) is polished as well
    bool degen = false;
    if (c.polish && P.ws && stop == kStopConverged) {
        double dg_l = 0.0;
        for (int r = l; r < m; r += kWave)
            if (isfinite(w[r])) dg_l = fmax(dg_l, fmin(t[r], lam[r]));
        degen = wave_max(dg_l) > kPolishDegenerate;
    }
    // polish (CMPC_FLAG_POLISH): a stall or max-iteration exit at the rounding floor leaves its last iterate
    // in the rescue image too (a breakdown wrote it above)
    if (c.polish && P.ws &&
        ((stop != kStopConverged && stop != kStopBreakdown && stop != kStopNonFinite &&
          (best_m < 1e3 * c.tol || stop == kStopMaxIter)) ||
         degen)) {
        double* hd = P.ws + (size_t)b * c.ws_stride;
        const size_t ht = hand_t(c);
        for (int i = l; i < n; i += kWave) hd[2 + i] = U[i];
        for (int i = l; i < N * ns; i += kWave) hd[2 + n + i] = sig[i];
        for (int r = l; r < m; r += kWave) {
            hd[ht + r] = t[r];
            hd[ht + m + r] = lam[r];
        }
    }
    if (stop != kStopConverged) {
        if (best_it > 0) {  // restore the best iterate
            for (int i = l; i < n; i += kWave) U[i] = bU[i];
            for (int i = l; i < N * ns; i += kWave) sig[i] = bsig[i];
            kkt = best_kkt;
        }
        status = stop_status(stop, best_m, c.tol);
    }
    bar();

    // ---- output in the reference layout ----
    fwd_sim(c, A, B, x0, U, X);
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
        if (P.iters) P.iters[b] = it;
        if (P.status) P.status[b] = status;
        // rescue hand-over flag: set only by a breakdown (the iterate was written there)
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
    }
}

int mpc_prepare(const cmpc_mpc_dims* d, const cmpc_mpc_weights* wt, const cmpc_opts* o, MpcConst* c,
                const char** msg) {
    if (!d || !wt || !c) {
        *msg = "null argument";
        return CMPC_ERR_ARG;
    }
    if (d->nx < 1 || d->nx > CMPC_MAX_NX || d->nu < 1 || d->nu > CMPC_MAX_NU || d->ns < 0 ||
        d->ns > CMPC_MAX_NS || d->mc < 0 || d->mc > CMPC_MAX_MC || d->N < 1 || d->batch < 0) {
        *msg = "dimension out of range (nx<=12, nu<=4, ns<=4, mc<=16)";
        return CMPC_ERR_UNSUPPORTED;
    }
    if (o && (o->flags & ~CMPC_FLAG_ALL)) {
        *msg = "unknown bits in opts.flags";
        return CMPC_ERR_ARG;
    }
    const bool fp32 = o && (o->flags & CMPC_FLAG_FP32);
    const bool lane_req = o && (o->flags & CMPC_FLAG_LANE);
    *c = MpcConst{};
    c->nx = d->nx;
    c->nu = d->nu;
    c->mc = d->mc;
    c->ns = d->ns;
    // the lane-per-agent kernel: CMPC_FLAG_LANE (fp64), or CMPC_FLAG_FP32 where it is instantiated
    const bool lane_ok = mpc_lane_supported(*c);
    if (lane_req && !lane_ok) {
        *msg = "CMPC_FLAG_LANE: no lane-per-agent kernel for these dimensions (nx,nu,mc,ns = 6,3,6,3 or 4,2,6,3)";
        return CMPC_ERR_UNSUPPORTED;
    }
    c->nx = d->nx;
    c->nu = d->nu;
    c->N = d->N;
    c->ns = d->ns;
    c->mc = d->mc;
    c->n = d->N * d->nu;
    c->ms = d->N * d->mc;
    c->m = c->ms + 2 * d->nu * d->N;
    c->nxp = (d->nx + 3) & ~3;
    c->npad = (c->n + 15) & ~15;
    c->ldk = (c->n & 1) ? c->n : c->n + 1;
    c->tol = (o && o->tol > 0) ? o->tol : 1e-9;
    c->max_iter = (o && o->max_iter > 0) ? o->max_iter : 60;
    // fp32: the stage-wise Riccati kernel's fp32 mode where it is instantiated (BASELINE cfg5), unless
    // CMPC_FLAG_LANE asks for the lane-per-agent kernel; else the lane kernel where it is instantiated;
    // other dimensions have no fp32 path (the round-1 workgroup-per-agent fp32 solver, which missed
    // the 1e-3 bar, is retired)
    c->f32 = (fp32 && !lane_req && mpc_riccati_f32_supported(*c)) ? 1 : 0;
    c->lane = (fp32 && lane_ok && !c->f32) ? 2 : (lane_req ? 1 : 0);
    if (fp32 && !c->f32 && !c->lane) {
        *msg = "CMPC_FLAG_FP32: no fp32 path for these dimensions (nx,nu,mc = 6,3,6 on the Riccati kernel; "
               "nx,nu,mc,ns = 6,3,6,3 or 4,2,6,3 on the lane kernel)";
        return CMPC_ERR_UNSUPPORTED;
    }
    c->riccati = (c->f32 || (!fp32 && !c->lane && (c->n > CMPC_MAX_NCOND || (o && (o->flags & CMPC_FLAG_RICCATI)))))
                     ? 1 : 0;
    double qs = 1.0;
    for (int i = 0; i < d->nx * d->nx; ++i) c->Q[i] = wt->Q[i];
    for (int i = 0; i < d->nu * d->nu; ++i) {
        c->R[i] = wt->R[i];
        c->dR[i] = wt->dR[i];
    }
    for (int j = 0; j < d->ns; ++j) {
        if (!(wt->Qs[j] > 0.0)) {
            *msg = "slack weights Qs must be > 0";
            return CMPC_ERR_ARG;
        }
        c->Qs[j] = wt->Qs[j];
        qs = fmax(qs, 2.0 * wt->Qs[j]);
    }
    c->qs_max = qs;
    if (c->riccati && mpc_riccati_lds_bytes(*c) > kMaxLdsBytes) {
        *msg = "the per-agent rows of this horizon do not fit the Riccati solver's 160 KB of LDS";
        return CMPC_ERR_UNSUPPORTED;
    }
    // rescue pass (CMPC_FLAG_RESCUE): only for condensed fp64 solves whose rows fit the Riccati kernel
    c->rescue = (!fp32 && !c->lane && !c->riccati && (o && (o->flags & CMPC_FLAG_RESCUE)) &&
                 mpc_riccati_lds_bytes(*c) <= kMaxLdsBytes)
                    ? 1 : 0;
    c->finish = (c->rescue && (o->flags & CMPC_FLAG_FINISH)) ? 1 : 0;
    if (o && (o->flags & CMPC_FLAG_TWO_WAVES) && (o->flags & CMPC_FLAG_ONE_WAVE)) {
        *msg = "CMPC_FLAG_ONE_WAVE and CMPC_FLAG_TWO_WAVES are exclusive";
        return CMPC_ERR_ARG;
    }
    c->waves = (o && (o->flags & CMPC_FLAG_TWO_WAVES)) ? 2 : ((o && (o->flags & CMPC_FLAG_ONE_WAVE)) ? 1 : 0);
    c->polish = 0;
    // (mpc_polish.hip: one lane per condensed variable in its H build, so n <= 64 — every condensed
    // solve, which is what carries the rescue image)
    c->polish = (c->rescue && (o->flags & CMPC_FLAG_POLISH) && c->n <= kWave &&
                 mpc_polish_lds_bytes(*c) <= kMaxLdsBytes)
                    ? 1 : 0;
    for (int i = 0; i < d->nu; ++i) {
        c->u_ub[i] = wt->u_ub[i];
        c->u_lb[i] = wt->u_lb[i];
    }
    for (int r = 0; r < d->mc; ++r) {
        if (wt->row_slack[r] >= d->ns || wt->row_slack[r] < -1) {
            *msg = "row_slack out of range";
            return CMPC_ERR_ARG;
        }
        c->row_slack[r] = wt->row_slack[r];
        c->row_sign[r] = wt->row_sign[r] >= 0 ? 1 : -1;
    }
    return CMPC_OK;
}

template <int T>
static hipError_t launch_t(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s) {
    const size_t lds = mpc_lds_bytes(c);
    hipError_t e = hipFuncSetAttribute((const void*)mpc_ipm_kernel<T>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(mpc_ipm_kernel<T>, dim3(batch), dim3(kWave), lds, s, c, p);
    return hipGetLastError();
}

hipError_t mpc_launch(const MpcConst& c_in, const MpcPtrs& p, int batch, hipStream_t s, int flags) {
    if (batch == 0) return hipSuccess;
    MpcConst c = c_in;
    c.ws_stride = p.ws ? mpc_ws_doubles(c) : 0;
    if (c.lane) return mpc_lane_launch(c, p, batch, s);
    if (c.riccati) {
        hipError_t er = mpc_riccati_launch(c, p, batch, s);
        if (er != hipSuccess || !c.f32 || !p.status || !p.ws) return er;
        // the fp32 path (Cfg::F32): an agent still short of tol after its in-launch fp64 restart gets the
        // fp64 kernel of the fp64 path at tol * 1e-3 (its floor the requested tol); every other workgroup
        // returns at once (rescue 3)
        MpcConst c64 = c;
        c64.f32 = 0;
        c64.tol = c.tol * 1e-3;
        c64.rescue = 3;
        return mpc_riccati_launch(c64, p, batch, s);
    }
    hipError_t e;
    if (flags & CMPC_FLAG_GENERIC || !mpc3_try_launch(c, p, batch, s, &e)) {
        switch (c.npad / 16) {
            case 1: e = launch_t<1>(c, p, batch, s); break;
            case 2: e = launch_t<2>(c, p, batch, s); break;
            case 3: e = launch_t<3>(c, p, batch, s); break;
            default: e = launch_t<4>(c, p, batch, s); break;
        }
    }
    if (e != hipSuccess || !c.rescue || !p.status || !p.ws) return e;
    // polish (CMPC_FLAG_POLISH) first: the condensed exits short of tol, and the breakdowns handed over to
    // the Riccati rescue (those it polishes to tol never reach it); the fused double-integrator round
    // keeps its rows in LDS only, so it has none to polish against
    const bool pol = c.polish && !p.fuse.on;
    if (pol && (e = mpc_polish_launch(c, p, batch, s)) != hipSuccess) return e;
    // rescue pass: the Riccati kernel re-solves, on the same problems, exactly the agents the
    // condensed solve left CMPC_UNSOLVED (its other workgroups return at once) — continuing from
    // the iterate a breakdown handed over (hand_doubles); a second pass restarts cold the rare
    // agent the continued solve leaves CMPC_UNSOLVED (the hand-over flag is consumed by then)
    MpcConst cr = c;
    cr.riccati = 1;
    if ((e = mpc_riccati_launch(cr, p, batch, s)) != hipSuccess) return e;
    cr.rescue = 2;  // the second (cold) pass: the last solve these agents get
    if ((e = mpc_riccati_launch(cr, p, batch, s)) != hipSuccess) return e;
    // ... and the Riccati rescue's own exits short of tol (rescue image flag 2)
    return pol ? mpc_polish_launch(c, p, batch, s) : hipSuccess;
}

// ---- f64 MFMA fragment-map self test: D(16x16) = A(16x4) * B(4x16) ----
__global__ void mfma_selftest_kernel(const double* A, const double* B, double* D) {
    const int l = threadIdx.x;
    v4d acc = {0.0, 0.0, 0.0, 0.0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

hipError_t selftest_mfma_launch(const double* A, const double* B, double* D, hipStream_t s) {
    hipLaunchKernelGGL(mfma_selftest_kernel, dim3(1), dim3(kWave), 0, s, A, B, D);
    return hipGetLastError();
}

}  // namespace cmpc
