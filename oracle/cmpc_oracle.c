/* ORACLE — test infrastructure only (never linked into the product).
 *
 * Plain-C fp64 restatement of the per-agent LPV-MPC QP solve the reference
 * performs in PlannerLPV.solve (planner/lib/plan_lib/distributedPlanner/
 * LPV_Planner.py:115-182): the same reference-form QP
 *   z = [xi_0..xi_N | u_0..u_{N-1} | du_0..du_{N-1}],  xi_k = [x_k | sigma_k]
 *   min 1/2 z'Pz + q'z,  P = 2 blkdiag(Q (+) Qs, R, dR)  (:382-427)
 *   dynamics / du equalities (:429-475), stage rows c'x_k + s*sigma <= h
 *   (:279-380), input boxes,
 * solved in condensed form (x eliminated through the dynamics) by a Mehrotra
 * primal-dual interior-point method with the per-stage slacks eliminated by
 * a diagonal Schur complement.  Dense Gamma, dense Cholesky: written for
 * clarity, not speed.  OpenMP over agents — this is bench.py's cpu_baseline
 * ("kind": "port") and the at-scale checker of the HIP path.
 *
 * Pinned by tests/test_oracle_c.py against the reference-form IPM
 * (oracle/qp_ipm.py) on QPs captured from the reference (tests/golden).
 */
#include <math.h>
#ifdef ORACLE_TRACE
#include <stdio.h>
#endif
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int nx, nu, N, ns, mc;
    const double *Q, *R, *dR, *Qs, *u_ub, *u_lb;
    const int *row_slack, *row_sign;
} shared_t;

typedef struct {
    const double *A, *B, *x0, *up, *p, *C, *h;
} agent_t;

#define IDX2(i, j, ld) ((size_t)(i) * (ld) + (j))

static void fwd_sim(const shared_t* S, const agent_t* a, const double* x0, const double* U, double* X) {
    int nx = S->nx, nu = S->nu, N = S->N;
    for (int s = 0; s < nx; ++s) X[s] = x0 ? x0[s] : 0.0;
    for (int k = 0; k < N; ++k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        for (int s = 0; s < nx; ++s) {
            double v = 0.0;
            for (int t = 0; t < nx; ++t) v += Ak[s * nx + t] * X[k * nx + t];
            for (int i = 0; i < nu; ++i) v += Bk[s * nu + i] * U[k * nu + i];
            X[(k + 1) * nx + s] = v;
        }
    }
}

/* out_k (k=0..N-1, nu each) = B_k' psi_{k+1},  psi_N = y_N, psi_k = y_k + A_k' psi_{k+1} */
static void adjoint(const shared_t* S, const agent_t* a, const double* ybar, double* out, double* psi, double* tmp) {
    int nx = S->nx, nu = S->nu, N = S->N;
    memcpy(psi, ybar + (size_t)N * nx, sizeof(double) * nx);
    for (int k = N - 1; k >= 0; --k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        for (int i = 0; i < nu; ++i) {
            double v = 0.0;
            for (int s = 0; s < nx; ++s) v += Bk[s * nu + i] * psi[s];
            out[k * nu + i] = v;
        }
        if (k > 0) {
            for (int t = 0; t < nx; ++t) {
                double v = ybar[(size_t)k * nx + t];
                for (int s = 0; s < nx; ++s) v += Ak[s * nx + t] * psi[s];
                tmp[t] = v;
            }
            memcpy(psi, tmp, sizeof(double) * nx);
        }
    }
}

/* NaN-propagating max (fmax would drop a NaN residual and report convergence) */
static double nmax(double a, double b) { return (a > b || a != a) ? a : b; }

#ifndef NBHD_GAMMA
#define NBHD_GAMMA 0.01 /* wide-neighbourhood floor: t_r lambda_r >= gamma mu after a step */
#endif
#define STALL_ITERS 3   /* near-converged iterations without merit progress before stopping */

static int chol(double* K, int n) {
    for (int j = 0; j < n; ++j) {
        double d = K[IDX2(j, j, n)];
        for (int p = 0; p < j; ++p) d -= K[IDX2(j, p, n)] * K[IDX2(j, p, n)];
        if (!(d > 0.0)) return -1;
        d = sqrt(d);
        K[IDX2(j, j, n)] = d;
        for (int i = j + 1; i < n; ++i) {
            double v = K[IDX2(i, j, n)];
            for (int p = 0; p < j; ++p) v -= K[IDX2(i, p, n)] * K[IDX2(j, p, n)];
            K[IDX2(i, j, n)] = v / d;
        }
    }
    return 0;
}

static void chol_solve(const double* L, int n, double* b) {
    for (int i = 0; i < n; ++i) {
        double v = b[i];
        for (int p = 0; p < i; ++p) v -= L[IDX2(i, p, n)] * b[p];
        b[i] = v / L[IDX2(i, i, n)];
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = b[i];
        for (int p = i + 1; p < n; ++p) v -= L[IDX2(p, i, n)] * b[p];
        b[i] = v / L[IDX2(i, i, n)];
    }
}

/* largest step keeping v + a dv >= 0 (unbounded: +inf; callers clip) */
static double max_step(const double* v, const double* dv, const unsigned char* act, int m) {
    double a = INFINITY;
    for (int r = 0; r < m; ++r)
        if (act[r] && dv[r] < 0.0) {
            double c = -v[r] / dv[r];
            if (c < a) a = c;
        }
    return a;
}

typedef struct {
    double *bU, *bsig, *Gam, *K, *X, *dX, *U, *dU, *sig, *dsig, *Dsig, *rsig, *t, *lam, *th, *rho, *rt, *rp, *w,
        *dt_a, *dl_a, *dtv, *dlv, *GdU, *ybar, *gU, *rd, *rhs, *psi, *tmp, *W, *Yk;
    unsigned char* act;
} work_t;

/* Solve one agent.  Returns OSQP-style status: 1 solved, 2 solved inaccurate, -2 max_iter, -10 unsolved. */
static int solve_one(const shared_t* S, const agent_t* a, double tol, int max_iter, work_t* wk,
                     double* z, double* kkt_out, int* iters_out) {
    const int nx = S->nx, nu = S->nu, N = S->N, ns = S->ns, mc = S->mc;
    const int n = N * nu, ms = N * mc, m = ms + 2 * nu * N;
    double* Gam = wk->Gam; /* (N+1) x nx x n */
    memset(Gam, 0, sizeof(double) * (size_t)(N + 1) * nx * n);
    for (int k = 0; k < N; ++k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        double* Gn = Gam + (size_t)(k + 1) * nx * n;
        const double* Gc = Gam + (size_t)k * nx * n;
        for (int s = 0; s < nx; ++s)
            for (int c = 0; c < n; ++c) {
                double v = 0.0;
                for (int t = 0; t < nx; ++t) v += Ak[s * nx + t] * Gc[t * n + c];
                if (c >= k * nu && c < (k + 1) * nu) v += Bk[s * nu + (c - k * nu)];
                Gn[s * n + c] = v;
            }
    }
    /* rhs of rows; inactive rows (infinite bound) are skipped */
    for (int k = 0; k < N; ++k)
        for (int r = 0; r < mc; ++r) {
            double h = a->h[k * mc + r];
            wk->w[k * mc + r] = h;
            wk->act[k * mc + r] = isfinite(h) ? 1 : 0;
        }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            int r = ms + (k * nu + i) * 2;
            wk->w[r] = S->u_ub[i];
            wk->w[r + 1] = -S->u_lb[i];
            wk->act[r] = isfinite(S->u_ub[i]) ? 1 : 0;
            wk->act[r + 1] = isfinite(S->u_lb[i]) ? 1 : 0;
        }
    int mact = 0;
    for (int r = 0; r < m; ++r) mact += wk->act[r];

    double *U = wk->U, *sig = wk->sig, *X = wk->X, *t = wk->t, *lam = wk->lam;
    memset(U, 0, sizeof(double) * n);
    memset(sig, 0, sizeof(double) * N * ns);
    fwd_sim(S, a, a->x0, U, X);

#define ROWVAL(Xv, Uv, sg, r, out)                                                      \
    do {                                                                                \
        if ((r) < ms) {                                                                 \
            int k_ = (r) / mc, rr_ = (r) % mc;                                          \
            const double* c_ = a->C + ((size_t)k_ * mc + rr_) * nx;                     \
            double v_ = 0.0;                                                            \
            for (int s_ = 0; s_ < nx; ++s_) v_ += c_[s_] * (Xv)[(k_ + 1) * nx + s_];   \
            int j_ = S->row_slack[rr_];                                                 \
            if (j_ >= 0 && (sg)) v_ += S->row_sign[rr_] * (sg)[k_ * ns + j_];           \
            out = v_;                                                                   \
        } else {                                                                        \
            int q_ = (r) - ms, ki_ = q_ / 2;                                            \
            out = (q_ & 1) ? -(Uv)[ki_] : (Uv)[ki_];                                    \
        }                                                                               \
    } while (0)

    for (int r = 0; r < m; ++r) {
        if (!wk->act[r]) { t[r] = 1.0; lam[r] = 0.0; continue; }
        double g; ROWVAL(X, U, sig, r, g);
        double s0 = wk->w[r] - g;
        t[r] = s0 > 1.0 ? s0 : 1.0;
        lam[r] = 1.0;
    }
    double scale_p = 1.0;
    for (int r = 0; r < m; ++r) if (wk->act[r] && fabs(wk->w[r]) > scale_p) scale_p = fabs(wk->w[r]);
    double qs_max = 1.0;
    for (int j = 0; j < ns; ++j) if (2 * S->Qs[j] > qs_max) qs_max = 2 * S->Qs[j];

    /* best iterate by merit max(res, 1e4 mu) (< tol <=> converged): returned when the
       method stops short of convergence (max_iter, factorisation breakdown, stagnation) */
    double best_m = INFINITY, best_kkt = INFINITY;
    int best_it = 0, stop = 0; /* stop: 0 max_iter, 1 converged, 2 breakdown, 3 stagnation, 4 non-finite */
    double *bU = wk->bU, *bsig = wk->bsig;
    int it;
    double kkt = INFINITY;
#ifdef SHORT_STEP
    double alpha_prev = 1.0;
#endif
    for (it = 1; it <= max_iter; ++it) {
        /* ---- residuals ---- */
        double* ybar = wk->ybar;
        double gscale = 1.0;
        for (int k = 0; k <= N; ++k)
            for (int s = 0; s < nx; ++s) {
                double v = 2.0 * a->p[k * nx + s];
                for (int t2 = 0; t2 < nx; ++t2) v += 2.0 * S->Q[s * nx + t2] * X[k * nx + t2];
                ybar[k * nx + s] = v;
            }
        /* gradient of f alone (for scaling) */
        adjoint(S, a, ybar, wk->gU, wk->psi, wk->tmp);
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nu; ++i) {
                double v = 0.0;
                for (int j = 0; j < nu; ++j) {
                    double du_k = U[k * nu + j] - (k ? U[(k - 1) * nu + j] : a->up[j]);
                    double du_n = (k + 1 < N) ? U[(k + 1) * nu + j] - U[k * nu + j] : 0.0;
                    v += 2.0 * S->R[i * nu + j] * U[k * nu + j] + 2.0 * S->dR[i * nu + j] * (du_k - du_n);
                }
                wk->gU[k * nu + i] += v;
            }
        for (int c = 0; c < n; ++c) gscale = nmax(gscale, fabs(wk->gU[c]));
        for (int k = 0; k < N; ++k)
            for (int r = 0; r < mc; ++r) {
                const double* c_ = a->C + ((size_t)k * mc + r) * nx;
                for (int s = 0; s < nx; ++s) ybar[(k + 1) * nx + s] += lam[k * mc + r] * c_[s];
            }
        adjoint(S, a, ybar, wk->rd, wk->psi, wk->tmp);
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nu; ++i) {
                double v = 0.0;
                for (int j = 0; j < nu; ++j) {
                    double du_k = U[k * nu + j] - (k ? U[(k - 1) * nu + j] : a->up[j]);
                    double du_n = (k + 1 < N) ? U[(k + 1) * nu + j] - U[k * nu + j] : 0.0;
                    v += 2.0 * S->R[i * nu + j] * U[k * nu + j] + 2.0 * S->dR[i * nu + j] * (du_k - du_n);
                }
                int r = ms + (k * nu + i) * 2;
                wk->rd[k * nu + i] += v + lam[r] - lam[r + 1];
            }
        for (int k = 0; k < N; ++k)
            for (int j = 0; j < ns; ++j) {
                double v = 2.0 * S->Qs[j] * sig[k * ns + j];
                for (int r = 0; r < mc; ++r)
                    if (S->row_slack[r] == j) v += S->row_sign[r] * lam[k * mc + r];
                wk->rsig[k * ns + j] = v;
            }
        double mu = 0.0, nrp = 0.0, nrd = 0.0, nrs = 0.0;
        for (int r = 0; r < m; ++r) {
            if (!wk->act[r]) { wk->rp[r] = 0.0; continue; }
            double g; ROWVAL(X, U, sig, r, g);
            wk->rp[r] = g + t[r] - wk->w[r];
            nrp = nmax(nrp, fabs(wk->rp[r]));
            mu += t[r] * lam[r];
        }
        mu = mact ? mu / mact : 0.0;
        for (int c = 0; c < n; ++c) nrd = nmax(nrd, fabs(wk->rd[c]));
        for (int q = 0; q < N * ns; ++q) nrs = nmax(nrs, fabs(wk->rsig[q]));
        /* stationarity / feasibility relative; complementarity absolute and 1e4 tighter
           (degenerate rows sit at t, lambda ~ sqrt(mu): primal accuracy needs tiny mu) */
        double res = nmax(nmax(nrd / gscale, nrs / qs_max), nrp / scale_p);
        kkt = nmax(res, mu);
        const double merit = nmax(res, 1e4 * mu);
        if (!isfinite(merit)) { stop = 4; break; }
        if (merit < best_m) {
            best_m = merit;
            best_kkt = kkt;
            best_it = it;
            memcpy(bU, U, sizeof(double) * n);
            memcpy(bsig, sig, sizeof(double) * N * ns);
        }
#ifdef ORACLE_TRACE
        fprintf(stderr, "it %2d mu %.3e res %.3e (rd %.2e rs %.2e rp %.2e) merit %.3e\n", it, mu, res,
                nrd / gscale, nrs / qs_max, nrp / scale_p, merit);
#endif
        if (merit < tol) { stop = 1; break; }
        /* near-converged but no progress for STALL_ITERS iterations: rounding floor reached */
        if (best_m < 1e3 * tol && it - best_it >= STALL_ITERS) { stop = 3; break; }

        /* ---- Newton matrix ---- */
        for (int r = 0; r < m; ++r) wk->th[r] = wk->act[r] ? lam[r] / t[r] : 0.0;
        for (int k = 0; k < N; ++k)
            for (int j = 0; j < ns; ++j) {
                double v = 2.0 * S->Qs[j];
                for (int r = 0; r < mc; ++r) if (S->row_slack[r] == j) v += wk->th[k * mc + r];
                wk->Dsig[k * ns + j] = v;
            }
        double* K = wk->K;
        memset(K, 0, sizeof(double) * n * n);
        double* W = wk->W;
        for (int k = 0; k < N; ++k) {
            /* W = 2Q + M_{k+1} (stable group Schur forms) */
            for (int s = 0; s < nx * nx; ++s) W[s] = 2.0 * S->Q[s];
            for (int r = 0; r < mc; ++r) {
                const double* c1 = a->C + ((size_t)k * mc + r) * nx;
                double th1 = wk->th[k * mc + r];
                int j = S->row_slack[r];
                if (j < 0) {
                    for (int s = 0; s < nx; ++s) for (int u = 0; u < nx; ++u) W[s * nx + u] += th1 * c1[s] * c1[u];
                    continue;
                }
                double inv = 1.0 / wk->Dsig[k * ns + j], q = 2.0 * S->Qs[j];
                for (int s = 0; s < nx; ++s) for (int u = 0; u < nx; ++u) W[s * nx + u] += q * th1 * c1[s] * c1[u] * inv;
                for (int r2 = r + 1; r2 < mc; ++r2) {
                    if (S->row_slack[r2] != j) continue;
                    const double* c2 = a->C + ((size_t)k * mc + r2) * nx;
                    double th2 = wk->th[k * mc + r2];
                    double s1 = S->row_sign[r], s2 = S->row_sign[r2];
                    for (int s = 0; s < nx; ++s)
                        for (int u = 0; u < nx; ++u)
                            W[s * nx + u] += th1 * th2 * (s1 * c1[s] - s2 * c2[s]) * (s1 * c1[u] - s2 * c2[u]) * inv;
                }
            }
            const double* G = Gam + (size_t)(k + 1) * nx * n;
            const int ncol = (k + 1) * nu; /* Gamma_{k+1} is zero beyond column (k+1)nu */
            double* Yk = wk->Yk;
            for (int s = 0; s < nx; ++s)
                for (int c2 = 0; c2 < ncol; ++c2) {
                    double v = 0.0;
                    for (int u = 0; u < nx; ++u) v += W[s * nx + u] * G[u * n + c2];
                    Yk[s * n + c2] = v;
                }
            for (int c1 = 0; c1 < ncol; ++c1)
                for (int c2 = 0; c2 <= c1; ++c2) {
                    double v = 0.0;
                    for (int s = 0; s < nx; ++s) v += G[s * n + c1] * Yk[s * n + c2];
                    K[IDX2(c1, c2, n)] += v;
                }
        }
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nu; ++i)
                for (int j = 0; j < nu; ++j) {
                    int ci = k * nu + i, cj = k * nu + j;
                    double v = 2.0 * S->R[i * nu + j] + 2.0 * S->dR[i * nu + j] * (k + 1 < N ? 2.0 : 1.0);
                    if (cj <= ci) K[IDX2(ci, cj, n)] += v;
                    if (k > 0 && 1) K[IDX2(ci, (k - 1) * nu + j, n)] += -2.0 * S->dR[i * nu + j];
                }
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nu; ++i) {
                int r = ms + (k * nu + i) * 2;
                K[IDX2(k * nu + i, k * nu + i, n)] += wk->th[r] + wk->th[r + 1];
            }
        if (chol(K, n)) { stop = 2; break; }

        /* ---- predictor / corrector ---- */
        double sig_c = 0.0, mu_aff = 0.0;
#ifdef RETRY_SIGMA
        int retried = 0;
#endif
        for (int pass = 0; pass < 2; ++pass) {
            for (int r = 0; r < m; ++r) {
                if (!wk->act[r]) { wk->rho[r] = 0.0; continue; }
                double rc = -t[r] * lam[r];
                if (pass) rc += sig_c * mu - wk->dt_a[r] * wk->dl_a[r];
                wk->rho[r] = (rc + lam[r] * wk->rp[r]) / t[r];
            }
            /* rho~ (stable form) */
            for (int r = 0; r < m; ++r) wk->rt[r] = wk->rho[r];
            for (int k = 0; k < N; ++k)
                for (int r = 0; r < mc; ++r) {
                    int j = S->row_slack[r];
                    if (j < 0) continue;
                    int R1 = k * mc + r;
                    double v = 2.0 * S->Qs[j] * wk->rho[R1] - wk->th[R1] * S->row_sign[r] * wk->rsig[k * ns + j];
                    for (int r2 = 0; r2 < mc; ++r2) {
                        if (r2 == r || S->row_slack[r2] != j) continue;
                        int R2 = k * mc + r2;
                        v += wk->th[R2] * wk->rho[R1] - wk->th[R1] * S->row_sign[r] * S->row_sign[r2] * wk->rho[R2];
                    }
                    wk->rt[R1] = v / wk->Dsig[k * ns + j];
                }
            memset(ybar, 0, sizeof(double) * (N + 1) * nx);
            for (int k = 0; k < N; ++k)
                for (int r = 0; r < mc; ++r) {
                    const double* c_ = a->C + ((size_t)k * mc + r) * nx;
                    for (int s = 0; s < nx; ++s) ybar[(k + 1) * nx + s] += wk->rt[k * mc + r] * c_[s];
                }
            adjoint(S, a, ybar, wk->rhs, wk->psi, wk->tmp);
            for (int c = 0; c < n; ++c) {
                int r = ms + c * 2;
                wk->rhs[c] = -wk->rd[c] - (wk->rhs[c] + wk->rt[r] - wk->rt[r + 1]);
            }
            memcpy(wk->dU, wk->rhs, sizeof(double) * n);
            chol_solve(K, n, wk->dU);
            fwd_sim(S, a, NULL, wk->dU, wk->dX);
            for (int r = 0; r < m; ++r) {
                double g; ROWVAL(wk->dX, wk->dU, (const double*)NULL, r, g);
                wk->GdU[r] = g;
            }
            for (int k = 0; k < N; ++k)
                for (int j = 0; j < ns; ++j) {
                    double v = wk->rsig[k * ns + j];
                    for (int r = 0; r < mc; ++r)
                        if (S->row_slack[r] == j) {
                            int R1 = k * mc + r;
                            v += S->row_sign[r] * (wk->rho[R1] + wk->th[R1] * wk->GdU[R1]);
                        }
                    wk->dsig[k * ns + j] = -v / wk->Dsig[k * ns + j];
                }
            double* dt = pass ? wk->dtv : wk->dt_a;
            double* dl = pass ? wk->dlv : wk->dl_a;
            for (int r = 0; r < m; ++r) {
                if (!wk->act[r]) { dt[r] = 0.0; dl[r] = 0.0; continue; }
                double sd = 0.0;
                if (r < ms) {
                    int j = S->row_slack[r % mc];
                    if (j >= 0) sd = S->row_sign[r % mc] * wk->dsig[(r / mc) * ns + j];
                }
                dt[r] = -wk->rp[r] - wk->GdU[r] - sd;
                dl[r] = wk->rho[r] + wk->th[r] * (wk->GdU[r] + sd);
            }
            double ap = max_step(t, dt, wk->act, m), ad = max_step(lam, dl, wk->act, m);
            double al = ap < ad ? ap : ad;
            if (!pass) {
                if (al > 1.0) al = 1.0;
                mu_aff = 0.0;
                for (int r = 0; r < m; ++r)
                    if (wk->act[r]) mu_aff += (t[r] + al * dt[r]) * (lam[r] + al * dl[r]);
                mu_aff /= mact ? mact : 1;
                sig_c = mu > 0 ? pow(mu_aff / mu, 3.0) : 0.0;
#ifdef SHORT_STEP
                if (alpha_prev < SHORT_STEP) sig_c = fmax(sig_c, SIGMA_MIN);
#endif
            } else {
                al = 0.995 * al;
#ifdef RETRY_SIGMA
                const double al_free = al > 1.0 ? 1.0 : al;
#endif
                if (al > 1.0) al = 1.0;
                /* keep the iterate in the wide neighbourhood t_r lambda_r >= gamma mu(al):
                   without it Mehrotra's corrector can cycle on degenerate collision rows
                   (two rows alternately blocking the step, mu stalled near 1e-5) */
                for (int bt = 0; bt < 30 && mact; ++bt) {
                    double mn = 0.0, pmin = INFINITY;
                    for (int r = 0; r < m; ++r)
                        if (wk->act[r]) {
                            double pr = (t[r] + al * dt[r]) * (lam[r] + al * dl[r]);
                            mn += pr;
                            if (pr < pmin) pmin = pr;
                        }
                    if (pmin >= NBHD_GAMMA * (mn / mact)) break;
                    al *= 0.8;
#ifdef ORACLE_TRACE
                    fprintf(stderr, "      backtrack %d al %.3e\n", bt, al);
#endif
                }
#ifdef ORACLE_TRACE
                {
                    int blk = -1; double amin = INFINITY;
                    for (int r = 0; r < m; ++r) if (wk->act[r]) {
                        if (dt[r] < 0 && -t[r] / dt[r] < amin) { amin = -t[r] / dt[r]; blk = r; }
                        if (dl[r] < 0 && -lam[r] / dl[r] < amin) { amin = -lam[r] / dl[r]; blk = 10000 + r; }
                    }
                    if (blk >= 0)
                        fprintf(stderr, "      step al %.3e sigma %.2e mu_aff/mu %.2e blocking %d (t %.2e lam %.2e)\n",
                                al, sig_c, mu > 0 ? mu_aff / mu : 0.0, blk, t[blk % 10000], lam[blk % 10000]);
                }
#endif
#ifdef RETRY_SIGMA
                /* the neighbourhood cut the corrector step hard: recompute it once with more centring */
                if (!retried && al < RETRY_FRAC * al_free) {
                    retried = 1;
                    sig_c = fmax(sig_c, RETRY_SIGMA);
                    pass = 0;
                    continue;
                }
#endif
#ifdef SHORT_STEP
                alpha_prev = al;
#endif
                for (int c = 0; c < n; ++c) U[c] += al * wk->dU[c];
                for (int q = 0; q < N * ns; ++q) sig[q] += al * wk->dsig[q];
                for (int r = 0; r < m; ++r)
                    if (wk->act[r]) { t[r] += al * dt[r]; lam[r] += al * dl[r]; }
                for (int q = 0; q < (N + 1) * nx; ++q) X[q] += al * wk->dX[q];
            }
        }
    }
    if (it > max_iter) it = max_iter;
    int status;
    if (stop == 1) {
        status = 1;
    } else {
        if (best_it > 0) { /* restore the best iterate */
            memcpy(U, bU, sizeof(double) * n);
            memcpy(sig, bsig, sizeof(double) * N * ns);
            kkt = best_kkt;
        }
        status = best_m < 1e3 * tol ? 2 : (stop == 0 ? -2 : -10);
    }
    /* exact re-simulation for the output trajectory */
    fwd_sim(S, a, a->x0, U, X);
    const int nxe = nx + ns;
    for (int k = 0; k <= N; ++k) {
        for (int s = 0; s < nx; ++s) z[k * nxe + s] = X[k * nx + s];
        for (int j = 0; j < ns; ++j) z[k * nxe + nx + j] = k ? sig[(k - 1) * ns + j] : 0.0;
    }
    double* zu = z + (size_t)(N + 1) * nxe;
    double* zd = zu + n;
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            zu[k * nu + i] = U[k * nu + i];
            zd[k * nu + i] = U[k * nu + i] - (k ? U[(k - 1) * nu + i] : a->up[i]);
        }
    *kkt_out = kkt;
    *iters_out = it;
    return status;
}

int cmpc_oracle_solve(int nx, int nu, int N, int ns, int mc, int batch,
                      const double* Q, const double* R, const double* dR, const double* Qs,
                      const double* u_ub, const double* u_lb, const int* row_slack, const int* row_sign,
                      const double* A, const double* Bm, const double* x0, const double* u_prev,
                      const double* qlin, const double* Crow, const double* hrow,
                      double tol, int max_iter, int nthreads,
                      double* z, double* kkt, int* iters, int* status) {
    shared_t S = {nx, nu, N, ns, mc, Q, R, dR, Qs, u_ub, u_lb, row_slack, row_sign};
    const int n = N * nu, m = N * mc + 2 * nu * N;
    const size_t nz = (size_t)(nx + ns) * (N + 1) + 2 * (size_t)nu * N;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int err = 0;
#pragma omp parallel
    {
        work_t wk;
        size_t need = (size_t)n + (size_t)N * ns + (size_t)(N + 1) * nx * n + (size_t)n * n + 4 * (size_t)(N + 1) * nx + 4 * (size_t)n +
                      4 * (size_t)N * ns + 12 * (size_t)m + 2 * (size_t)nx + (size_t)nx * nx + (size_t)n * 3 + (size_t)nx * n;
        double* buf = (double*)calloc(need, sizeof(double));
        unsigned char* act = (unsigned char*)calloc(m, 1);
        if (!buf || !act) {
#pragma omp atomic write
            err = 1;
        } else {
            double* p = buf;
#define TAKE(f, cnt) do { wk.f = p; p += (cnt); } while (0)
            TAKE(bU, n); TAKE(bsig, N * ns);
            TAKE(Gam, (size_t)(N + 1) * nx * n); TAKE(K, (size_t)n * n);
            TAKE(X, (N + 1) * nx); TAKE(dX, (N + 1) * nx); TAKE(ybar, (N + 1) * nx); TAKE(W, nx * nx);
            TAKE(U, n); TAKE(dU, n); TAKE(gU, n); TAKE(rd, n); TAKE(rhs, n);
            TAKE(sig, N * ns); TAKE(dsig, N * ns); TAKE(Dsig, N * ns); TAKE(rsig, N * ns);
            TAKE(t, m); TAKE(lam, m); TAKE(th, m); TAKE(rho, m); TAKE(rt, m); TAKE(rp, m); TAKE(w, m);
            TAKE(dt_a, m); TAKE(dl_a, m); TAKE(dtv, m); TAKE(dlv, m); TAKE(GdU, m);
            TAKE(psi, nx); TAKE(tmp, nx); TAKE(Yk, (size_t)nx * n);
#undef TAKE
            wk.act = act;
#pragma omp for schedule(dynamic, 4)
            for (int b = 0; b < batch; ++b) {
                agent_t ag = {A + (size_t)b * N * nx * nx, Bm + (size_t)b * N * nx * nu, x0 + (size_t)b * nx,
                              u_prev + (size_t)b * nu, qlin + (size_t)b * (N + 1) * nx,
                              Crow + (size_t)b * N * mc * nx, hrow + (size_t)b * N * mc};
                status[b] = solve_one(&S, &ag, tol, max_iter, &wk, z + b * nz, kkt + b, iters + b);
            }
        }
        free(buf);
        free(act);
    }
    return err ? -1 : 0;
}
