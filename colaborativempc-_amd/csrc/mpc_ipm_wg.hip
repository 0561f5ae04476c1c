// Batched condensed IPM for long horizons (N*nu up to 256), one 256-thread workgroup per
// agent, in fp32 — the BASELINE cfg5 path (8192 agents, N=50, 3-D dynamics nx=6 nu=3, fp32
// with a tolerance check against the fp64 reference).  Same QP as the other solvers (the
// PlannerLPV form, planner/lib/plan_lib/distributedPlanner/LPV_Planner.py:279-475), same
// Mehrotra method, slack elimination in the stable group form, safeguards and termination
// structure (internal.h); tolerances are the caller's (fp32: ~1e-5).
//
// Layout: every per-agent array and the Newton matrix K live in LDS; K is stored packed
// lower-triangular (n(n+1)/2 floats: 45 KB at n = 150) and factored in place by a
// right-looking Cholesky with one thread per row.  K = sum_k Gamma_{k+1}' W_{k+1} Gamma_{k+1}
// is accumulated stage by stage with one thread per packed entry of the nonzero leading
// block.  The dynamics recursions run one thread per state component.
#include <cmath>

#include "internal.h"

namespace cmpc {

namespace {

constexpr int kWgThreads = 256;

struct LdsWg {
    int K, A, B, C, h, p, x0, up, W, G0, G1, Y, X, dX, yb, psi, U, dU, rd, gU, rhs, sig, dsig, Dsig, rsig;
    int t, lam, th, rho, rt, rp, w, dta, dla, GdU, bU, bsig, red, total;
};

template <class R>
__host__ __device__ inline LdsWg wg_layout(const MpcConst& c) {
    LdsWg L;
    int o = 0;
    auto take = [&](int cnt) {
        int r = o;
        o += (cnt + 3) & ~3;
        return r;
    };
    const int n = c.n, N = c.N, nx = c.nx, nu = c.nu, mc = c.mc, ns = c.ns, m = c.m;
    L.K = take(n * (n + 1) / 2);
    L.A = take(N * nx * nx);
    L.B = take(N * nx * nu);
    L.C = take(N * mc * nx);
    L.h = take(N * mc);
    L.p = take((N + 1) * nx);
    L.x0 = take(nx);
    L.up = take(nu);
    L.W = take(nx * nx);
    L.G0 = take(nx * n);
    L.G1 = take(nx * n);
    L.Y = take(nx * n);
    L.X = take((N + 1) * nx);
    L.dX = take((N + 1) * nx);
    L.yb = take((N + 1) * nx);
    L.psi = take(2 * nx);
    L.U = take(n);
    L.dU = take(n);
    L.rd = take(n);
    L.gU = take(n);
    L.rhs = take(n);
    L.sig = take(N * ns);
    L.dsig = take(N * ns);
    L.Dsig = take(N * ns);
    L.rsig = take(N * ns);
    L.t = take(m);
    L.lam = take(m);
    L.th = take(m);
    L.rho = take(m);
    L.rt = take(m);
    L.rp = take(m);
    L.w = take(m);
    L.dta = take(m);
    L.dla = take(m);
    L.GdU = take(m);
    L.bU = take(n);
    L.bsig = take(N * ns);
    L.red = take(kWgThreads);
    L.total = o;
    return L;
}

__device__ __forceinline__ int pk(int i, int j) { return i * (i + 1) / 2 + j; }  // packed lower, j <= i

template <class R>
struct WgRed {
    R* s;
    __device__ R sum(R v) {
        const int t = threadIdx.x;
        __syncthreads();
        s[t] = v;
        __syncthreads();
        for (int o = kWgThreads / 2; o > 0; o >>= 1) {
            if (t < o) s[t] += s[t + o];
            __syncthreads();
        }
        const R r = s[0];
        __syncthreads();
        return r;
    }
    __device__ R max(R v) {  // NaN-propagating
        const int t = threadIdx.x;
        __syncthreads();
        s[t] = v;
        __syncthreads();
        for (int o = kWgThreads / 2; o > 0; o >>= 1) {
            if (t < o) {
                const R a = s[t], b = s[t + o];
                s[t] = (a > b || a != a) ? a : b;
            }
            __syncthreads();
        }
        const R r = s[0];
        __syncthreads();
        return r;
    }
    __device__ R min(R v) {
        const int t = threadIdx.x;
        __syncthreads();
        s[t] = v;
        __syncthreads();
        for (int o = kWgThreads / 2; o > 0; o >>= 1) {
            if (t < o) s[t] = fmin(s[t], s[t + o]);
            __syncthreads();
        }
        const R r = s[0];
        __syncthreads();
        return r;
    }
};

template <class R>
__device__ __forceinline__ R rmax(R a, R b) { return (a > b || a != a) ? a : b; }

}  // namespace

template <class R>
__global__ __launch_bounds__(kWgThreads) void mpc_ipm_wg_kernel(const MpcConst c, const MpcPtrs P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    R* sm = reinterpret_cast<R*>(smem_raw);
    const LdsWg L = wg_layout<R>(c);
    const int tid = threadIdx.x, b = blockIdx.x;
    const int nx = c.nx, nu = c.nu, N = c.N, ns = c.ns, mc = c.mc, n = c.n, ms = c.ms, m = c.m;
    R *K = sm + L.K, *A = sm + L.A, *B = sm + L.B, *C = sm + L.C, *hh = sm + L.h, *pl = sm + L.p;
    R *x0 = sm + L.x0, *up = sm + L.up, *W = sm + L.W, *G0 = sm + L.G0, *G1 = sm + L.G1, *Y = sm + L.Y;
    R *X = sm + L.X, *dX = sm + L.dX, *yb = sm + L.yb, *psi = sm + L.psi, *U = sm + L.U, *dU = sm + L.dU;
    R *rd = sm + L.rd, *gU = sm + L.gU, *rhs = sm + L.rhs, *sig = sm + L.sig, *dsig = sm + L.dsig;
    R *Dsig = sm + L.Dsig, *rsig = sm + L.rsig, *t = sm + L.t, *lam = sm + L.lam, *th = sm + L.th;
    R *rho = sm + L.rho, *rt = sm + L.rt, *rp = sm + L.rp, *w = sm + L.w, *dta = sm + L.dta, *dla = sm + L.dla;
    R *GdU = sm + L.GdU, *bU = sm + L.bU, *bsig = sm + L.bsig;
    WgRed<R> red{sm + L.red};

    // ---- stage inputs (fp64 in HBM -> R in LDS) ----
    {
        const double* gA = P.A + (size_t)b * N * nx * nx;
        const double* gB = P.B + (size_t)b * N * nx * nu;
        const double* gC = P.C + (size_t)b * N * mc * nx;
        const double* gh = P.h + (size_t)b * ms;
        const double* gp = P.p + (size_t)b * (N + 1) * nx;
        for (int i = tid; i < N * nx * nx; i += kWgThreads) A[i] = (R)gA[i];
        for (int i = tid; i < N * nx * nu; i += kWgThreads) B[i] = (R)gB[i];
        for (int i = tid; i < N * mc * nx; i += kWgThreads) C[i] = (R)gC[i];
        for (int i = tid; i < ms; i += kWgThreads) hh[i] = (R)gh[i];
        for (int i = tid; i < (N + 1) * nx; i += kWgThreads) pl[i] = (R)gp[i];
        if (tid < nx) x0[tid] = (R)P.x0[(size_t)b * nx + tid];
        if (tid < nu) up[tid] = (R)P.up[(size_t)b * nu + tid];
        for (int i = tid; i < n; i += kWgThreads) U[i] = bU[i] = 0;
        for (int i = tid; i < N * ns; i += kWgThreads) sig[i] = bsig[i] = 0;
    }
    __syncthreads();
    auto fwd = [&](const R* xin, const R* Uv, R* Xo) {
        if (tid < nx) Xo[tid] = xin ? xin[tid] : R(0);
        __syncthreads();
        for (int k = 0; k < N; ++k) {
            if (tid < nx) {
                R v = 0;
                for (int s2 = 0; s2 < nx; ++s2) v = fma(A[(k * nx + tid) * nx + s2], Xo[k * nx + s2], v);
                for (int i = 0; i < nu; ++i) v = fma(B[(k * nx + tid) * nu + i], Uv[k * nu + i], v);
                Xo[(k + 1) * nx + tid] = v;
            }
            __syncthreads();
        }
    };
    auto adj = [&](const R* y, R* out) {  // out_k = B_k' psi_{k+1}, psi_N = y_N, psi_k = y_k + A_k' psi_{k+1}
        R* pa = psi;
        R* pb = psi + nx;
        if (tid < nx) pa[tid] = y[N * nx + tid];
        __syncthreads();
        for (int k = N - 1; k >= 0; --k) {
            if (tid < nu) {
                R v = 0;
                for (int s2 = 0; s2 < nx; ++s2) v = fma(B[(k * nx + s2) * nu + tid], pa[s2], v);
                out[k * nu + tid] = v;
            }
            if (k > 0 && tid >= 64 && tid < 64 + nx) {
                const int s = tid - 64;
                R v = y[k * nx + s];
                for (int s2 = 0; s2 < nx; ++s2) v = fma(A[(k * nx + s2) * nx + s], pa[s2], v);
                pb[s] = v;
            }
            __syncthreads();
            R* tq = pa;
            pa = pb;
            pb = tq;
        }
    };
    auto rowval = [&](int r, const R* Xv, const R* Uv, const R* sg) -> R {
        if (r < ms) {
            const int k = r / mc, rr = r - k * mc;
            const R* cr = C + r * nx;
            R v = 0;
            for (int s2 = 0; s2 < nx; ++s2) v = fma(cr[s2], Xv[(k + 1) * nx + s2], v);
            const int j = c.row_slack[rr];
            if (sg && j >= 0) v += (R)c.row_sign[rr] * sg[k * ns + j];
            return v;
        }
        const int q = r - ms;
        const R u = Uv[q >> 1];
        return (q & 1) ? -u : u;
    };
    auto rdr = [&](int ci) -> R {  // 2R u_k + 2dR (du_k - du_{k+1})
        const int k = ci / nu, i = ci - k * nu;
        R v = 0;
        for (int j = 0; j < nu; ++j) {
            const R uk = U[k * nu + j];
            const R duk = uk - (k ? U[(k - 1) * nu + j] : up[j]);
            const R dun = (k + 1 < N) ? U[(k + 1) * nu + j] - uk : R(0);
            v += (R)(2.0 * c.R[i * nu + j]) * uk + (R)(2.0 * c.dR[i * nu + j]) * (duk - dun);
        }
        return v;
    };

    for (int r = tid; r < m; r += kWgThreads) {
        double v;
        if (r < ms) v = P.h[(size_t)b * ms + r];
        else {
            const int q = r - ms, i = (q >> 1) % nu;
            v = (q & 1) ? -c.u_lb[i] : c.u_ub[i];
        }
        w[r] = isfinite(v) ? (R)v : R(INFINITY);
    }
    __syncthreads();
    fwd(x0, U, X);
    R mact_l = 0, sp_l = 1;
    for (int r = tid; r < m; r += kWgThreads) {
        if (isfinite(w[r])) {
            t[r] = fmax(w[r] - rowval(r, X, U, sig), R(1));
            lam[r] = 1;
            mact_l += 1;
            sp_l = fmax(sp_l, fabs(w[r]));
        } else {
            t[r] = 1;
            lam[r] = 0;
        }
    }
    const R mact = fmax(red.sum(mact_l), R(1));
    const R scale_p = red.max(sp_l);
    const R tol = (R)c.tol, qs_max = (R)c.qs_max;

    R best_m = R(INFINITY), best_kkt = R(INFINITY), kkt = R(INFINITY);
    int best_it = 0, stop = kStopMaxIter, it;
    R alpha_prev = 1;  // step of the previous iteration (kShortStep guard)
    for (it = 1; it <= c.max_iter; ++it) {
        // ================= residuals =================
        for (int i = tid; i < (N + 1) * nx; i += kWgThreads) {
            const int k = i / nx, s = i - k * nx;
            R v = 2 * pl[i];
            for (int u = 0; u < nx; ++u) v = fma((R)(2.0 * c.Q[s * nx + u]), X[k * nx + u], v);
            yb[i] = v;
        }
        __syncthreads();
        adj(yb, gU);
        R gs_l = 1;
        for (int i = tid; i < n; i += kWgThreads) {
            gU[i] += rdr(i);
            gs_l = rmax(gs_l, fabs(gU[i]));
        }
        for (int i = tid; i < N * nx; i += kWgThreads) {
            const int k = i / nx, s = i - k * nx;
            R v = 0;
            for (int r = 0; r < mc; ++r) v = fma(lam[k * mc + r], C[(k * mc + r) * nx + s], v);
            yb[(k + 1) * nx + s] += v;
        }
        __syncthreads();
        adj(yb, rd);
        R nrd_l = 0, nrs_l = 0, nrp_l = 0, mu_l = 0;
        for (int i = tid; i < n; i += kWgThreads) {
            const int r = ms + 2 * i;
            rd[i] += rdr(i) + lam[r] - lam[r + 1];
            nrd_l = rmax(nrd_l, fabs(rd[i]));
        }
        for (int i = tid; i < N * ns; i += kWgThreads) {
            const int k = i / ns, j = i - k * ns;
            R v = (R)(2.0 * c.Qs[j]) * sig[i];
            for (int r = 0; r < mc; ++r)
                if (c.row_slack[r] == j) v += (R)c.row_sign[r] * lam[k * mc + r];
            rsig[i] = v;
            nrs_l = rmax(nrs_l, fabs(v));
        }
        for (int r = tid; r < m; r += kWgThreads) {
            if (isfinite(w[r])) {
                rp[r] = rowval(r, X, U, sig) + t[r] - w[r];
                nrp_l = rmax(nrp_l, fabs(rp[r]));
                mu_l += t[r] * lam[r];
            } else {
                rp[r] = 0;
            }
        }
        const R mu = red.sum(mu_l) / mact;
        const R res = rmax(rmax(red.max(nrd_l) / red.max(gs_l), red.max(nrs_l) / qs_max), red.max(nrp_l) / scale_p);
        kkt = rmax(res, mu);
        // fp64: complementarity 1e4 tighter than the residuals (degenerate rows sit at sqrt(mu));
        // fp32 cannot resolve mu below ~1e-7 under Theta ~ 1e7 — there the factor is 10
        const R merit = rmax(res, (sizeof(R) == 4 ? R(10) : R(1e4)) * mu);
        if (!isfinite(merit)) {
            stop = kStopNonFinite;
            break;
        }
        if (merit < best_m) {
            best_m = merit;
            best_kkt = kkt;
            best_it = it;
            for (int i = tid; i < n; i += kWgThreads) bU[i] = U[i];
            for (int i = tid; i < N * ns; i += kWgThreads) bsig[i] = sig[i];
        }
        if (merit < tol) {
            stop = kStopConverged;
            break;
        }
        if (best_m < R(1e3) * tol && it - best_it >= kStallIters) {
            stop = kStopStalled;
            break;
        }
        __syncthreads();

        // ================= Newton matrix (packed lower) =================
        for (int r = tid; r < m; r += kWgThreads) th[r] = isfinite(w[r]) ? lam[r] / t[r] : R(0);
        __syncthreads();
        for (int i = tid; i < N * ns; i += kWgThreads) {
            const int k = i / ns, j = i - k * ns;
            R v = (R)(2.0 * c.Qs[j]);
            for (int r = 0; r < mc; ++r)
                if (c.row_slack[r] == j) v += th[k * mc + r];
            Dsig[i] = v;
        }
        for (int i = tid; i < n * (n + 1) / 2; i += kWgThreads) K[i] = 0;
        // both Gamma buffers: stage k reads the columns of Gamma_k that stage k-1 did not write
        for (int i = tid; i < nx * n; i += kWgThreads) G0[i] = G1[i] = 0;
        __syncthreads();
        R* gc = G0;
        R* gn = G1;
        for (int k = 0; k < N; ++k) {
            const int ncol = (k + 1) * nu;
            for (int i = tid; i < nx * ncol; i += kWgThreads) {  // Gamma_{k+1} = A_k Gamma_k + [0 .. B_k]
                const int s = i / ncol, col = i - s * ncol;
                R v = 0;
                for (int u = 0; u < nx; ++u) v = fma(A[(k * nx + s) * nx + u], gc[u * n + col], v);
                if (col >= k * nu) v += B[(k * nx + s) * nu + (col - k * nu)];
                gn[s * n + col] = v;
            }
            const R* Ck = C + k * mc * nx;
            const R* thk = th + k * mc;
            const R* Dk = Dsig + k * ns;
            for (int i = tid; i < nx * nx; i += kWgThreads) {  // W = 2Q + M_{k+1} (stable group Schur form)
                const int s = i / nx, u = i - s * nx;
                R v = (R)(2.0 * c.Q[i]);
                for (int r = 0; r < mc; ++r) {
                    const R* c1 = Ck + r * nx;
                    const R t1 = thk[r];
                    const int j = c.row_slack[r];
                    if (j < 0) {
                        v = fma(t1 * c1[s], c1[u], v);
                        continue;
                    }
                    R g = (R)(2.0 * c.Qs[j]) * t1 * c1[s] * c1[u];
                    const R s1 = (R)c.row_sign[r];
                    for (int r2 = r + 1; r2 < mc; ++r2) {
                        if (c.row_slack[r2] != j) continue;
                        const R* c2 = Ck + r2 * nx;
                        const R s2 = (R)c.row_sign[r2];
                        g += t1 * thk[r2] * (s1 * c1[s] - s2 * c2[s]) * (s1 * c1[u] - s2 * c2[u]);
                    }
                    v = fma(g, R(1) / Dk[j], v);
                }
                W[i] = v;
            }
            __syncthreads();
            for (int i = tid; i < nx * ncol; i += kWgThreads) {  // Y = W Gamma_{k+1}
                const int s = i / ncol, col = i - s * ncol;
                R v = 0;
                for (int u = 0; u < nx; ++u) v = fma(W[s * nx + u], gn[u * n + col], v);
                Y[s * n + col] = v;
            }
            __syncthreads();
            const int np = ncol * (ncol + 1) / 2;
            for (int e = tid; e < np; e += kWgThreads) {  // K[i][j] += Gamma' Y on the nonzero leading block
                const int i = (int)((sqrtf(8.0f * e + 1.0f) - 1.0f) * 0.5f);
                int ii = i;
                while (pk(ii + 1, 0) <= e) ++ii;
                while (pk(ii, 0) > e) --ii;
                const int j = e - pk(ii, 0);
                R v = 0;
                for (int s = 0; s < nx; ++s) v = fma(gn[s * n + ii], Y[s * n + j], v);
                K[e] += v;
            }
            __syncthreads();
            R* tq = gc;
            gc = gn;
            gn = tq;
        }
        for (int i = tid; i < n; i += kWgThreads) {  // + 2R + 2D'dR D + input-row curvature
            const int k = i / nu, a = i - k * nu;
            for (int j = 0; j < nu; ++j) {
                const int col = k * nu + j;
                if (col <= i) K[pk(i, col)] += (R)(2.0 * c.R[a * nu + j] + 2.0 * c.dR[a * nu + j] * (k + 1 < N ? 2.0 : 1.0));
                if (k > 0) K[pk(i, (k - 1) * nu + j)] -= (R)(2.0 * c.dR[a * nu + j]);
            }
            K[pk(i, i)] += th[ms + 2 * i] + th[ms + 2 * i + 1];
        }
        __syncthreads();
        // ================= Cholesky (packed, right-looking, thread per row) =================
        bool chol_ok = true;
        for (int j = 0; j < n; ++j) {
            const R djj = K[pk(j, j)];
            if (!(djj > R(0))) {
                chol_ok = false;
                break;
            }
            const R d = sqrt(djj);
            const R dinv = R(1) / d;
            __syncthreads();
            if (tid == 0) K[pk(j, j)] = d;
            for (int i = j + 1 + tid; i < n; i += kWgThreads) K[pk(i, j)] *= dinv;
            __syncthreads();
            for (int i = j + 1 + tid; i < n; i += kWgThreads) {
                const R lij = K[pk(i, j)];
                R* row = K + pk(i, 0);
                for (int cc = j + 1; cc <= i; ++cc) row[cc] = fma(-lij, K[pk(cc, j)], row[cc]);
            }
            __syncthreads();
        }
        if (!chol_ok) {
            stop = kStopBreakdown;
            break;
        }

        // ================= predictor / corrector =================
        R sig_c = 0, alpha = 0;
        for (int pass = 0; pass < 2; ++pass) {
            for (int r = tid; r < m; r += kWgThreads) {
                if (!isfinite(w[r])) {
                    rho[r] = 0;
                    continue;
                }
                R rc = -t[r] * lam[r];
                if (pass) rc += sig_c * mu - dta[r] * dla[r];
                rho[r] = (rc + lam[r] * rp[r]) / t[r];
            }
            __syncthreads();
            for (int r = tid; r < m; r += kWgThreads) {
                R v = rho[r];
                if (r < ms) {
                    const int k = r / mc, rr = r - k * mc, j = c.row_slack[rr];
                    if (j >= 0) {
                        v = (R)(2.0 * c.Qs[j]) * rho[r] - th[r] * (R)c.row_sign[rr] * rsig[k * ns + j];
                        for (int r2 = 0; r2 < mc; ++r2) {
                            if (r2 == rr || c.row_slack[r2] != j) continue;
                            const int R2 = k * mc + r2;
                            v += th[R2] * rho[r] - th[r] * (R)(c.row_sign[rr] * c.row_sign[r2]) * rho[R2];
                        }
                        v /= Dsig[k * ns + j];
                    }
                }
                rt[r] = v;
            }
            __syncthreads();
            for (int i = tid; i < (N + 1) * nx; i += kWgThreads) {
                const int k = i / nx, s = i - k * nx;
                R v = 0;
                if (k > 0)
                    for (int r = 0; r < mc; ++r) v = fma(rt[(k - 1) * mc + r], C[((k - 1) * mc + r) * nx + s], v);
                yb[i] = v;
            }
            __syncthreads();
            adj(yb, dU);
            for (int i = tid; i < n; i += kWgThreads) rhs[i] = -rd[i] - (dU[i] + rt[ms + 2 * i] - rt[ms + 2 * i + 1]);
            __syncthreads();
            // forward L z = rhs (column sweep), backward L' x = z (row sweep)
            for (int j = 0; j < n; ++j) {
                const R zj = rhs[j] / K[pk(j, j)];
                __syncthreads();
                if (tid == 0) rhs[j] = zj;
                for (int i = j + 1 + tid; i < n; i += kWgThreads) rhs[i] = fma(-K[pk(i, j)], zj, rhs[i]);
                __syncthreads();
            }
            for (int j = n - 1; j >= 0; --j) {
                const R xj = rhs[j] / K[pk(j, j)];
                __syncthreads();
                if (tid == 0) rhs[j] = xj;
                for (int i = tid; i < j; i += kWgThreads) rhs[i] = fma(-K[pk(j, i)], xj, rhs[i]);
                __syncthreads();
            }
            for (int i = tid; i < n; i += kWgThreads) dU[i] = rhs[i];
            __syncthreads();
            fwd(nullptr, dU, dX);
            for (int r = tid; r < m; r += kWgThreads) GdU[r] = rowval(r, dX, dU, nullptr);
            __syncthreads();
            for (int i = tid; i < N * ns; i += kWgThreads) {
                const int k = i / ns, j = i - k * ns;
                R v = rsig[i];
                for (int r = 0; r < mc; ++r)
                    if (c.row_slack[r] == j) {
                        const int R1 = k * mc + r;
                        v += (R)c.row_sign[r] * (rho[R1] + th[R1] * GdU[R1]);
                    }
                dsig[i] = -v / Dsig[i];
            }
            __syncthreads();
            R amax_l = R(1e30);
            R* dtp = pass ? rho : dta;  // corrector reuses rho / rt for (dt, dl)
            R* dlp = pass ? rt : dla;
            for (int r = tid; r < m; r += kWgThreads) {
                if (!isfinite(w[r])) {
                    dtp[r] = 0;
                    dlp[r] = 0;
                    continue;
                }
                R sd = 0;
                if (r < ms) {
                    const int k = r / mc, rr = r - k * mc, j = c.row_slack[rr];
                    if (j >= 0) sd = (R)c.row_sign[rr] * dsig[k * ns + j];
                }
                const R rho_r = rho[r];
                const R dtv = -rp[r] - GdU[r] - sd;
                const R dlv = rho_r + th[r] * (GdU[r] + sd);
                dtp[r] = dtv;
                dlp[r] = dlv;
                if (dtv < 0) amax_l = fmin(amax_l, -t[r] / dtv);
                if (dlv < 0) amax_l = fmin(amax_l, -lam[r] / dlv);
            }
            const R amax = red.min(amax_l);
            if (!pass) {
                const R a = fmin(amax, R(1));
                R mua_l = 0;
                for (int r = tid; r < m; r += kWgThreads)
                    if (isfinite(w[r])) mua_l += (t[r] + a * dta[r]) * (lam[r] + a * dla[r]);
                const R mu_aff = red.sum(mua_l) / mact;
                const R ratio = mu > 0 ? mu_aff / mu : R(0);
                sig_c = ratio * ratio * ratio;
                if (alpha_prev < R(kShortStep)) sig_c = fmax(sig_c, R(kSigmaMin));
            } else {
                alpha = fmin(R(1), R(0.995) * amax);
                for (int bt = 0; bt < kMaxBacktrack; ++bt) {
                    R mn_l = 0, pm_l = R(INFINITY);
                    for (int r = tid; r < m; r += kWgThreads)
                        if (isfinite(w[r])) {
                            const R pr = (t[r] + alpha * rho[r]) * (lam[r] + alpha * rt[r]);
                            mn_l += pr;
                            pm_l = fmin(pm_l, pr);
                        }
                    const R pmin = red.min(pm_l), mn = red.sum(mn_l);
                    if (pmin >= (R)kNbhdGamma * (mn / mact)) break;
                    alpha *= R(0.8);
                }
            }
        }
        alpha_prev = alpha;
        for (int i = tid; i < n; i += kWgThreads) U[i] = fma(alpha, dU[i], U[i]);
        for (int i = tid; i < N * ns; i += kWgThreads) sig[i] = fma(alpha, dsig[i], sig[i]);
        for (int i = tid; i < (N + 1) * nx; i += kWgThreads) X[i] = fma(alpha, dX[i], X[i]);
        for (int r = tid; r < m; r += kWgThreads)
            if (isfinite(w[r])) {
                t[r] = fma(alpha, rho[r], t[r]);
                lam[r] = fma(alpha, rt[r], lam[r]);
            }
        __syncthreads();
    }
    if (it > c.max_iter) it = c.max_iter;
    __syncthreads();
    int status = CMPC_SOLVED;
    if (stop != kStopConverged) {
        if (best_it > 0) {
            for (int i = tid; i < n; i += kWgThreads) U[i] = bU[i];
            for (int i = tid; i < N * ns; i += kWgThreads) sig[i] = bsig[i];
            kkt = best_kkt;
        }
        status = stop_status(stop, (double)best_m, c.tol);
    }
    __syncthreads();
    fwd(x0, U, X);
    const int nxe = nx + ns;
    const size_t nz = (size_t)nxe * (N + 1) + 2 * (size_t)n;
    double* z = P.z + (size_t)b * nz;
    for (int i = tid; i < (N + 1) * nxe; i += kWgThreads) {
        const int k = i / nxe, s = i - k * nxe;
        z[i] = (s < nx) ? (double)X[k * nx + s] : (k ? (double)sig[(k - 1) * ns + (s - nx)] : 0.0);
    }
    for (int i = tid; i < n; i += kWgThreads) {
        const int k = i / nu, j = i - k * nu;
        z[(size_t)(N + 1) * nxe + i] = (double)U[i];
        z[(size_t)(N + 1) * nxe + n + i] = (double)(U[i] - (k ? U[(k - 1) * nu + j] : up[j]));
    }
    if (tid == 0) {
        if (P.kkt) P.kkt[b] = (double)kkt;
        if (P.iters) P.iters[b] = it;
        if (P.status) P.status[b] = status;
    }
}

size_t mpc_wg_lds_bytes(const MpcConst& c, bool fp32) {
    return fp32 ? sizeof(float) * (size_t)wg_layout<float>(c).total : sizeof(double) * (size_t)wg_layout<double>(c).total;
}

hipError_t mpc_wg_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, bool fp32) {
    if (batch == 0) return hipSuccess;
    const size_t lds = mpc_wg_lds_bytes(c, fp32);
    const void* fn = fp32 ? (const void*)mpc_ipm_wg_kernel<float> : (const void*)mpc_ipm_wg_kernel<double>;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (fp32) hipLaunchKernelGGL(mpc_ipm_wg_kernel<float>, dim3(batch), dim3(kWgThreads), lds, s, c, p);
    else hipLaunchKernelGGL(mpc_ipm_wg_kernel<double>, dim3(batch), dim3(kWgThreads), lds, s, c, p);
    return hipGetLastError();
}

}  // namespace cmpc
