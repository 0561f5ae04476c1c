// Batched dense convex QP with quadprog semantics — the drop-in for the MATLAB path's
// quadprog(H, f, A, b, Aeq, beq, lb, ub) reached through YALMIP
// (Matlab-tests/yalmip/yalmip/YALMIP-master/solvers/callquadprog.m:63-69) and for the Python
// path's generic osqp_solve_qp(P, q, G, h, A, b) (planner/lib/plan_lib/distributedPlanner/
// LPV_Planner.py:192-249) on problems that do not have the structured agent-QP form.
//
//   min 1/2 x'Hx + f'x   s.t.  A x <= b,  Aeq x = beq,  lb <= x <= ub
//
// One 256-thread workgroup per problem.  Mehrotra primal-dual interior point with the same
// safeguards as the structured solver (wide neighbourhood, best iterate, stagnation exit).
// Each Newton system is the regularised quasi-definite KKT matrix
//   [H + A'Theta A + Theta_bounds + rho I , Aeq' ; Aeq , -delta I]
// factored by a dense LDL' without pivoting (quasi-definite => factorisable in any order)
// in a per-problem global-memory workspace (column-major, coalesced over rows), followed by
// iterative refinement against the unregularised system.  Rows of Aeq / A that are entirely
// zero are dropped (0 = 0 rows of the reference's QP, LPV_Planner.py:445-447), or flag the
// problem infeasible when their right-hand side cannot hold.
#include <cmath>

#include "internal.h"

namespace cmpc {

namespace {

constexpr int kQpThreads = 256;

struct QpWs {  // offsets (doubles) into one problem's workspace
    int K, x, y, t, lam, act, rd, re, rp, th, rho, dx, dy, gdx, rhs, sol, res, tmp, bx, by, dsc, rsa, rse, total;
};

__host__ __device__ inline int mi_of(int m, int n) { return m - 2 * n; }

__host__ __device__ inline QpWs qp_ws_layout(int n, int me, int m) {
    QpWs w;
    int o = 0;
    auto take = [&](int cnt) {
        int r = o;
        o += (cnt + 1) & ~1;
        return r;
    };
    const int nk = n + me;
    w.K = take(nk * nk);
    w.x = take(n);
    w.y = take(me);
    w.t = take(m);
    w.lam = take(m);
    w.act = take(m + me);  // 1.0 active, 0.0 inactive (rows of A/bounds, then Aeq rows)
    w.rd = take(n);
    w.re = take(me);
    w.rp = take(m);
    w.th = take(m);
    w.rho = take(m);
    w.dx = take(n);
    w.dy = take(me);
    w.gdx = take(m);
    w.rhs = take(nk);
    w.sol = take(nk);
    w.res = take(nk);
    w.tmp = take(nk > m ? nk : m);
    w.bx = take(n);
    w.by = take(me);
    w.dsc = take(n);
    w.rsa = take(mi_of(m, n));
    w.rse = take(me);
    w.total = o;
    return w;
}

struct BlockRed {
    double* s;
    __device__ double sum(double v) {
        const int t = threadIdx.x;
        __syncthreads();
        s[t] = v;
        __syncthreads();
        for (int o = kQpThreads / 2; o > 0; o >>= 1) {
            if (t < o) s[t] += s[t + o];
            __syncthreads();
        }
        const double r = s[0];
        __syncthreads();
        return r;
    }
    __device__ double max(double v) {  // NaN-propagating
        const int t = threadIdx.x;
        __syncthreads();
        s[t] = v;
        __syncthreads();
        for (int o = kQpThreads / 2; o > 0; o >>= 1) {
            if (t < o) {
                const double a = s[t], b2 = s[t + o];
                s[t] = (a > b2 || a != a) ? a : b2;
            }
            __syncthreads();
        }
        const double r = s[0];
        __syncthreads();
        return r;
    }
    __device__ double min(double v) {
        const int t = threadIdx.x;
        __syncthreads();
        s[t] = v;
        __syncthreads();
        for (int o = kQpThreads / 2; o > 0; o >>= 1) {
            if (t < o) s[t] = fmin(s[t], s[t + o]);
            __syncthreads();
        }
        const double r = s[0];
        __syncthreads();
        return r;
    }
};

__device__ __forceinline__ double qmax(double a, double b) { return (a > b || a != a) ? a : b; }

}  // namespace

__global__ __launch_bounds__(kQpThreads) void qp_dense_kernel(const QpConst c, const QpPtrs P) {
    __shared__ double red_s[kQpThreads];
    BlockRed R{red_s};
    const int tid = threadIdx.x, pb = blockIdx.x;
    const int n = c.n, mi = c.mi, me = c.me, nk = n + me, m = mi + 2 * n;
    const QpWs L = qp_ws_layout(n, me, m);
    double* ws = P.ws + (size_t)pb * L.total;
    double* K = ws + L.K;
    double *x = ws + L.x, *y = ws + L.y, *t = ws + L.t, *lam = ws + L.lam, *act = ws + L.act;
    double *rd = ws + L.rd, *re = ws + L.re, *rp = ws + L.rp, *th = ws + L.th, *rho = ws + L.rho;
    double *dx = ws + L.dx, *dy = ws + L.dy, *gdx = ws + L.gdx, *rhs = ws + L.rhs, *sol = ws + L.sol;
    double *res = ws + L.res, *tmp = ws + L.tmp, *bx = ws + L.bx, *by = ws + L.by;
    double *dsc = ws + L.dsc, *rsa = ws + L.rsa, *rse = ws + L.rse;
    const double* H = P.H + (size_t)pb * n * n;
    const double* f = P.f + (size_t)pb * n;
    const double* A = P.A ? P.A + (size_t)pb * mi * n : nullptr;
    const double* b = P.b ? P.b + (size_t)pb * mi : nullptr;
    const double* Aeq = P.Aeq ? P.Aeq + (size_t)pb * me * n : nullptr;
    const double* beq = P.beq ? P.beq + (size_t)pb * me : nullptr;
    const double* lb = P.lb ? P.lb + (size_t)pb * n : nullptr;
    const double* ub = P.ub ? P.ub + (size_t)pb * n : nullptr;
    const bool cm = c.col_major != 0;
    // raw element accessors (row-major, or MATLAB column-major)
    auto Araw = [&](int i, int j) { return cm ? A[(size_t)j * mi + i] : A[(size_t)i * n + j]; };
    auto Eraw = [&](int i, int j) { return cm ? Aeq[(size_t)j * me + i] : Aeq[(size_t)i * n + j]; };
    // The IPM runs on the scaled problem x = D xs (D_jj = 1/sqrt(max(|H_jj|, 1)): the reference's
    // Qs = 1e7 slack curvature becomes O(1)) with rows of A and Aeq equilibrated to unit max-norm.
    auto Hel = [&](int i, int j) { return dsc[i] * (0.5 * (H[i * n + j] + H[j * n + i])) * dsc[j]; };
    auto Ael = [&](int i, int j) { return rsa[i] * Araw(i, j) * dsc[j]; };
    auto Eel = [&](int i, int j) { return rse[i] * Eraw(i, j) * dsc[j]; };
    auto fel = [&](int i) { return dsc[i] * f[i]; };
    // inequality row r: r < mi general row, mi <= r < mi+n upper bound of x_{r-mi}, else lower bound
    auto hval = [&](int r) -> double {
        if (r < mi) return rsa[r] * b[r];
        if (r < mi + n) return ub ? ub[r - mi] / dsc[r - mi] : INFINITY;
        return lb ? -lb[r - mi - n] / dsc[r - mi - n] : INFINITY;
    };
    auto gval = [&](int r, const double* v) -> double {  // row value G_r v
        if (r < mi) {
            double s = 0.0;
            for (int j = 0; j < n; ++j) s = fma(Ael(r, j), v[j], s);
            return s;
        }
        if (r < mi + n) return v[r - mi];
        return -v[r - mi - n];
    };

    // ---- scaling ----
    for (int i = tid; i < n; i += kQpThreads) dsc[i] = 1.0 / sqrt(fmax(fabs(H[i * n + i]), 1.0));
    __syncthreads();
    for (int r = tid; r < mi; r += kQpThreads) {
        double mx = 0.0;
        for (int j = 0; j < n; ++j) mx = fmax(mx, fabs(Araw(r, j) * dsc[j]));
        rsa[r] = mx > 0.0 ? 1.0 / mx : 1.0;
    }
    for (int r = tid; r < me; r += kQpThreads) {
        double mx = 0.0;
        for (int j = 0; j < n; ++j) mx = fmax(mx, fabs(Eraw(r, j) * dsc[j]));
        rse[r] = mx > 0.0 ? 1.0 / mx : 1.0;
    }
    __syncthreads();
    // ---- activity: drop all-zero rows (flag infeasible when the rhs cannot hold) ----
    int bad_l = 0;
    for (int r = tid; r < m; r += kQpThreads) {
        const double h = hval(r);
        double a = isfinite(h) ? 1.0 : 0.0;
        if (r < mi && a != 0.0) {
            double nz = 0.0;
            for (int j = 0; j < n; ++j) nz = fmax(nz, fabs(Ael(r, j)));
            if (nz == 0.0) {
                a = 0.0;
                if (h < 0.0) bad_l = 1;
            }
        }
        if (!(h == h)) bad_l = 1;  // NaN bound
        act[r] = a;
    }
    for (int r = tid; r < me; r += kQpThreads) {
        double nz = 0.0;
        for (int j = 0; j < n; ++j) nz = fmax(nz, fabs(Eel(r, j)));
        act[m + r] = nz > 0.0 ? 1.0 : 0.0;
        if (nz == 0.0 && beq[r] != 0.0) bad_l = 1;
        if (!(beq[r] == beq[r])) bad_l = 1;
    }
    for (int i = tid; i < n; i += kQpThreads) {
        x[i] = 0.0;
        // start inside finite boxes
        const double lo = lb ? lb[i] / dsc[i] : -INFINITY, hi = ub ? ub[i] / dsc[i] : INFINITY;
        if (isfinite(lo) && isfinite(hi)) x[i] = 0.5 * (lo + hi);
        else if (isfinite(lo)) x[i] = fmax(0.0, lo + 1.0);
        else if (isfinite(hi)) x[i] = fmin(0.0, hi - 1.0);
    }
    for (int i = tid; i < me; i += kQpThreads) y[i] = 0.0;
    __syncthreads();
    const bool bad = R.max((double)bad_l) > 0.0;
    // scales
    double sf_l = 1.0, sh_l = 1.0, mact_l = 0.0;
    for (int i = tid; i < n; i += kQpThreads) sf_l = qmax(sf_l, fabs(fel(i)));
    for (int r = tid; r < m; r += kQpThreads)
        if (act[r] != 0.0) {
            sh_l = qmax(sh_l, fabs(hval(r)));
            mact_l += 1.0;
        }
    for (int r = tid; r < me; r += kQpThreads)
        if (act[m + r] != 0.0) sh_l = qmax(sh_l, fabs(rse[r] * beq[r]));
    const double scale_f = R.max(sf_l), scale_p = R.max(sh_l), mact = fmax(R.sum(mact_l), 1.0);
    // nonconvexity screen: a negative diagonal of H
    double hneg_l = 0.0;
    for (int i = tid; i < n; i += kQpThreads) hneg_l = qmax(hneg_l, -H[i * n + i] * dsc[i] * dsc[i]);
    const bool nonconvex_diag = R.max(hneg_l) > 1e-9 * scale_f;
    for (int r = tid; r < m; r += kQpThreads) {
        if (act[r] != 0.0) {
            t[r] = fmax(hval(r) - gval(r, x), 1.0);
            lam[r] = 1.0;
        } else {
            t[r] = 1.0;
            lam[r] = 0.0;
        }
    }
    __syncthreads();

    const double rho_reg = c.reg;
    double best_m = INFINITY, fval = 0.0;
    int best_it = 0, stop = kStopMaxIter, it = 0;
    bool factor_fail = false, indefinite = false;
    double res_d_best = INFINITY, res_p_best = INFINITY;
    if (bad || nonconvex_diag) stop = kStopNonFinite;
    for (it = 1; it <= c.max_iter && stop == kStopMaxIter; ++it) {
        // ================= residuals =================
        // rd = Hx + f + Aeq'y + A'lam_A + lam_u - lam_l
        double hx_l = 0.0;
        for (int i = tid; i < n; i += kQpThreads) {
            double v = 0.0;
            for (int j = 0; j < n; ++j) v = fma(Hel(i, j), x[j], v);
            hx_l = qmax(hx_l, fabs(v));
            v += fel(i);
            for (int r = 0; r < me; ++r)
                if (act[m + r] != 0.0) v = fma(Eel(r, i), y[r], v);
            for (int r = 0; r < mi; ++r) v = fma(Ael(r, i), lam[r], v);
            v += lam[mi + i] - lam[mi + n + i];
            rd[i] = v;
        }
        double nre_l = 0.0, nrp_l = 0.0, mu_l = 0.0, nrd_l = 0.0;
        for (int r = tid; r < me; r += kQpThreads) {
            double v = 0.0;
            if (act[m + r] != 0.0) {
                for (int j = 0; j < n; ++j) v = fma(Eel(r, j), x[j], v);
                v -= rse[r] * beq[r];
            }
            re[r] = v;
            nre_l = qmax(nre_l, fabs(v));
        }
        for (int r = tid; r < m; r += kQpThreads) {
            if (act[r] != 0.0) {
                const double v = gval(r, x) + t[r] - hval(r);
                rp[r] = v;
                nrp_l = qmax(nrp_l, fabs(v));
                mu_l += t[r] * lam[r];
            } else {
                rp[r] = 0.0;
            }
        }
        __syncthreads();
        for (int i = tid; i < n; i += kQpThreads) nrd_l = qmax(nrd_l, fabs(rd[i]));
        const double res_d = R.max(nrd_l) / fmax(scale_f, R.max(hx_l));
        const double res_p = qmax(R.max(nre_l), R.max(nrp_l)) / scale_p;
        const double mu = R.sum(mu_l) / mact;
        const double merit = qmax(qmax(res_d, res_p), mu);
        if (!isfinite(merit)) {
            stop = kStopNonFinite;
            break;
        }
        if (merit < best_m) {
            best_m = merit;
            best_it = it;
            res_d_best = res_d;
            res_p_best = res_p;
            for (int i = tid; i < n; i += kQpThreads) bx[i] = x[i];
            for (int i = tid; i < me; i += kQpThreads) by[i] = y[i];
        }
        if (merit < c.tol) {
            stop = kStopConverged;
            break;
        }
        if (best_m < 1e3 * c.tol && it - best_it >= kStallIters) {
            stop = kStopStalled;
            break;
        }

        // ================= KKT matrix (column-major lower triangle) + LDL' =================
        for (int r = tid; r < m; r += kQpThreads) th[r] = act[r] != 0.0 ? lam[r] / t[r] : 0.0;
        __syncthreads();
        double rr = rho_reg;  // quasi-definite regularisation; raised x100 after a breakdown
        for (int attempt = 0; attempt < 4; ++attempt, rr *= 100.0) {
            factor_fail = false;
            for (int cidx = 0; cidx < n; ++cidx) {  // column cidx of the (1,1) block, rows i >= cidx
                for (int i = cidx + tid; i < n; i += kQpThreads) {
                    double v = Hel(i, cidx);
                    for (int r = 0; r < mi; ++r) v = fma(th[r] * Ael(r, i), Ael(r, cidx), v);
                    if (i == cidx) v += th[mi + i] + th[mi + n + i] + rr;
                    K[(size_t)cidx * nk + i] = v;
                }
                for (int r = tid; r < me; r += kQpThreads)
                    K[(size_t)cidx * nk + n + r] = act[m + r] != 0.0 ? Eel(r, cidx) : 0.0;
            }
            // (2,2) block: -delta I (its lower part is fill-in of the previous factorisation)
            for (int r = 0; r < me; ++r)
                for (int i = n + r + tid; i < nk; i += kQpThreads) K[(size_t)(n + r) * nk + i] = (i == n + r) ? -rr : 0.0;
            __syncthreads();
            // LDL' without pivoting (quasi-definite)
            for (int j = 0; j < nk; ++j) {
                const double d = K[(size_t)j * nk + j];
                if (j < n ? !(d > 0.0) : !(d < 0.0)) {
                    // at the first iterate Theta is moderate: a non-positive pivot of the (1,1) block
                    // means H is not positive semidefinite on the problem
                    factor_fail = true;
                    indefinite = (j < n) && it == 1 && attempt == 0;
                    break;
                }
                for (int i = j + 1 + tid; i < nk; i += kQpThreads) K[(size_t)j * nk + i] /= d;
                __syncthreads();
                for (int i = j + 1 + tid; i < nk; i += kQpThreads) {
                    const double lij = K[(size_t)j * nk + i] * d;
                    for (int cc = j + 1; cc <= i; ++cc) K[(size_t)cc * nk + i] = fma(-lij, K[(size_t)j * nk + cc], K[(size_t)cc * nk + i]);
                }
                __syncthreads();
            }
            __syncthreads();
            if (!factor_fail || indefinite) break;
        }
        if (factor_fail) {
            stop = kStopBreakdown;
            break;
        }

        // solve K s = rhs (in place in sol) with the LDL' factor
        auto ldl_solve = [&]() {
            for (int j = 0; j < nk; ++j) {
                const double zj = sol[j];
                __syncthreads();
                for (int i = j + 1 + tid; i < nk; i += kQpThreads) sol[i] = fma(-K[(size_t)j * nk + i], zj, sol[i]);
                __syncthreads();
            }
            for (int i = tid; i < nk; i += kQpThreads) sol[i] /= K[(size_t)i * nk + i];
            __syncthreads();
            for (int j = nk - 1; j >= 0; --j) {
                const double wj = sol[j];
                __syncthreads();
                for (int i = tid; i < j; i += kQpThreads) sol[i] = fma(-K[(size_t)i * nk + j], wj, sol[i]);
                __syncthreads();
            }
        };
        // unregularised KKT operator: out = [ (H + A'Th A + Th_b) v1 + Aeq' v2 ; Aeq v1 ]
        auto kkt_apply = [&](const double* v, double* out) {
            for (int r = tid; r < mi; r += kQpThreads) tmp[r] = th[r] * gval(r, v);
            __syncthreads();
            for (int i = tid; i < n; i += kQpThreads) {
                double s = 0.0;
                for (int j = 0; j < n; ++j) s = fma(Hel(i, j), v[j], s);
                for (int r = 0; r < mi; ++r) s = fma(Ael(r, i), tmp[r], s);
                s += (th[mi + i] + th[mi + n + i]) * v[i];
                for (int r = 0; r < me; ++r)
                    if (act[m + r] != 0.0) s = fma(Eel(r, i), v[n + r], s);
                out[i] = s;
            }
            for (int r = tid; r < me; r += kQpThreads) {
                double s = 0.0;
                if (act[m + r] != 0.0)
                    for (int j = 0; j < n; ++j) s = fma(Eel(r, j), v[j], s);
                out[n + r] = act[m + r] != 0.0 ? s : -rr * v[n + r];
            }
            __syncthreads();
        };

        // ================= predictor / corrector =================
        double sig_c = 0.0, alpha = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            // rho_r = (rc_r + lam_r rp_r) / t_r ; corrector: rc += sig mu - dt_aff dl_aff (predictor
            // direction still in rho, gdx)
            for (int r = tid; r < m; r += kQpThreads) {
                if (act[r] == 0.0) {
                    rho[r] = 0.0;
                    continue;
                }
                double rc = -t[r] * lam[r];
                if (pass) {
                    const double dta = -rp[r] - gdx[r];
                    const double dla = rho[r] + th[r] * gdx[r];
                    rc += sig_c * mu - dta * dla;
                }
                rho[r] = (rc + lam[r] * rp[r]) / t[r];
            }
            __syncthreads();
            // rhs = [-rd - G' rho ; -re]
            for (int i = tid; i < n; i += kQpThreads) {
                double s = -rd[i];
                for (int r = 0; r < mi; ++r) s = fma(-Ael(r, i), rho[r], s);
                s -= rho[mi + i] - rho[mi + n + i];
                rhs[i] = s;
            }
            for (int r = tid; r < me; r += kQpThreads) rhs[n + r] = act[m + r] != 0.0 ? -re[r] : 0.0;
            __syncthreads();
            for (int i = tid; i < nk; i += kQpThreads) sol[i] = rhs[i];
            __syncthreads();
            ldl_solve();
            // iterative refinement against the unregularised system
            double nrhs_l = 0.0;
            for (int i = tid; i < nk; i += kQpThreads) nrhs_l = qmax(nrhs_l, fabs(rhs[i]));
            const double nrhs = R.max(nrhs_l);
            for (int rf = 0; rf < c.refine; ++rf) {
                kkt_apply(sol, res);
                double nres_l = 0.0;
                for (int i = tid; i < nk; i += kQpThreads) nres_l = qmax(nres_l, fabs(rhs[i] - res[i]));
                if (R.max(nres_l) <= 1e-13 * nrhs) break;  // converged refinement
                for (int i = tid; i < nk; i += kQpThreads) {
                    tmp[i] = sol[i];  // keep the current solution (tmp reused after kkt_apply)
                    res[i] = rhs[i] - res[i];
                }
                __syncthreads();
                for (int i = tid; i < nk; i += kQpThreads) {
                    const double keep = tmp[i];
                    sol[i] = res[i];
                    res[i] = keep;
                }
                __syncthreads();
                ldl_solve();
                for (int i = tid; i < nk; i += kQpThreads) sol[i] += res[i];
                __syncthreads();
            }
            for (int i = tid; i < n; i += kQpThreads) dx[i] = sol[i];
            for (int r = tid; r < me; r += kQpThreads) dy[r] = sol[n + r];
            __syncthreads();
            for (int r = tid; r < m; r += kQpThreads) gdx[r] = act[r] != 0.0 ? gval(r, dx) : 0.0;
            __syncthreads();
            double amax_l = 1.0e300;
            for (int r = tid; r < m; r += kQpThreads) {
                if (act[r] == 0.0) continue;
                const double dtv = -rp[r] - gdx[r];
                const double dlv = rho[r] + th[r] * gdx[r];
                if (dtv < 0.0) amax_l = fmin(amax_l, -t[r] / dtv);
                if (dlv < 0.0) amax_l = fmin(amax_l, -lam[r] / dlv);
            }
            const double amax = R.min(amax_l);
            if (!pass) {
                const double a = fmin(amax, 1.0);
                double mua_l = 0.0;
                for (int r = tid; r < m; r += kQpThreads)
                    if (act[r] != 0.0)
                        mua_l += (t[r] + a * (-rp[r] - gdx[r])) * (lam[r] + a * (rho[r] + th[r] * gdx[r]));
                const double mu_aff = R.sum(mua_l) / mact;
                const double ratio = mu > 0.0 ? mu_aff / mu : 0.0;
                sig_c = ratio * ratio * ratio;
            } else {
                alpha = fmin(1.0, 0.995 * amax);
                for (int bt = 0; bt < kMaxBacktrack; ++bt) {
                    double mn_l = 0.0, pm_l = INFINITY;
                    for (int r = tid; r < m; r += kQpThreads)
                        if (act[r] != 0.0) {
                            const double pr = (t[r] + alpha * (-rp[r] - gdx[r])) * (lam[r] + alpha * (rho[r] + th[r] * gdx[r]));
                            mn_l += pr;
                            pm_l = fmin(pm_l, pr);
                        }
                    const double pmin = R.min(pm_l), mn = R.sum(mn_l);
                    if (pmin >= kNbhdGamma * (mn / mact)) break;
                    alpha *= 0.8;
                }
                for (int r = tid; r < m; r += kQpThreads)
                    if (act[r] != 0.0) {
                        t[r] = fma(alpha, -rp[r] - gdx[r], t[r]);
                        lam[r] = fma(alpha, rho[r] + th[r] * gdx[r], lam[r]);
                    }
                for (int i = tid; i < n; i += kQpThreads) x[i] = fma(alpha, dx[i], x[i]);
                for (int r = tid; r < me; r += kQpThreads) y[r] = fma(alpha, dy[r], y[r]);
                __syncthreads();
            }
        }
    }
    if (it > c.max_iter) it = c.max_iter;
    __syncthreads();
    int flag = 1;
    if (stop != kStopConverged) {
        if (best_it > 0) {
            for (int i = tid; i < n; i += kQpThreads) x[i] = bx[i];
            for (int i = tid; i < me; i += kQpThreads) y[i] = by[i];
            __syncthreads();
        }
        // quadprog exit flags: 1 converged, 0 iteration cap, -2 infeasible, -3 unbounded, -6 nonconvex
        if (bad) flag = -2;
        else if (nonconvex_diag || indefinite) flag = -6;
        else if (best_m < 1e3 * c.tol) flag = 1;  // converged to the attainable accuracy (reported in output)
        else if (res_p_best > 1e3 * c.tol) flag = -2;
        else if (res_d_best > 1e3 * c.tol) flag = -3;
        else flag = 0;
    }
    // back to the unscaled problem: x = D xs, lambda_A = ra lambda_s, y = re y_s, bound
    // multipliers / D; fval = 1/2 x'Hx + f'x (scaling-invariant)
    double fv_l = 0.0;
    for (int i = tid; i < n; i += kQpThreads) {
        double v = 0.0;
        for (int j = 0; j < n; ++j) v = fma(Hel(i, j), x[j], v);
        fv_l += x[i] * (0.5 * v + fel(i));
    }
    fval = R.sum(fv_l);
    for (int i = tid; i < n; i += kQpThreads) {
        P.x[(size_t)pb * n + i] = dsc[i] * x[i];
        if (P.lam_lo) P.lam_lo[(size_t)pb * n + i] = lam[mi + n + i] / dsc[i];
        if (P.lam_up) P.lam_up[(size_t)pb * n + i] = lam[mi + i] / dsc[i];
    }
    if (P.lam_ineq)
        for (int r = tid; r < mi; r += kQpThreads) P.lam_ineq[(size_t)pb * mi + r] = rsa[r] * lam[r];
    if (P.lam_eq)
        for (int r = tid; r < me; r += kQpThreads) P.lam_eq[(size_t)pb * me + r] = rse[r] * y[r];
    if (tid == 0) {
        if (P.fval) P.fval[pb] = fval;
        if (P.exitflag) P.exitflag[pb] = flag;
        if (P.iters) P.iters[pb] = it;
        if (P.merit) P.merit[pb] = best_m;
    }
}

size_t qp_ws_doubles(int n, int mi, int me) { return (size_t)qp_ws_layout(n, me, mi + 2 * n).total; }

hipError_t qp_launch(const QpConst& c, const QpPtrs& p, int batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(qp_dense_kernel, dim3(batch), dim3(kQpThreads), 0, s, c, p);
    return hipGetLastError();
}

}  // namespace cmpc
