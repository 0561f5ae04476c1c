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
#if defined(ORACLE_TRACE) || defined(POLISH_DEBUG) || defined(RIC_DEBUG) || defined(LAB_THDUMP) || defined(DIRCHECK) || defined(LAB_STOPDUMP) || defined(LAB_DEGEN)
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
    int newton, refine; /* refine: iterative-refinement steps of the Riccati solve */
    int refine_dd;      /* refinement steps of a double-double iteration (RIC_REFINE_MAX; continued
                           rescue solves RIC_REFINE_WARM, the kernels' kRefineMaxWarm) */
    int polish;         /* CMPC_FLAG_POLISH: active-set polish of a breakdown at the rounding floor */
    int polish_amax;    /* largest polished active set (0: POLISH_MAX_ACTIVE) */
    /* newton: 0 condensed Cholesky; 1 Riccati (P = Qyy + A'PA + Hvy'K); 2 Riccati, Joseph form */
} shared_t;

typedef struct {
    const double *A, *B, *x0, *up, *p, *C, *h;
    const double* U0; /* optional starting inputs (warm start), NULL: U = 0 */
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

#ifdef DD_COUNT
long cmpc_dd_iters = 0; /* lab: double-double iterations */
#endif
#ifdef POLISH_AT
long lab_pol_tried = 0, lab_pol_ok = 0; /* lab: polish attempts at iteration POLISH_AT, successes */
#endif
#ifdef GONDZIO
long cmpc_gz_solves = 0; /* lab: corrector solves performed */
#endif
#ifdef LAB_DEGEN_COUNT
/* lab: converged solves flagged for the polish by the degenerate-row test, and those whose polished point
   replaced the endpoint (tools/degen_lab.py: the threshold's reach at a loose tol) */
long cmpc_degen_flagged = 0, cmpc_degen_taken = 0;
#endif
/* after a step shorter than SHORT_STEP the next corrector centres with sigma >= SIGMA_MIN
   (kernels: kShortStep, kSigmaMin in internal.h) */
#ifndef SHORT_STEP
#define SHORT_STEP 0.02
#endif
#ifndef SIGMA_MIN
#define SIGMA_MIN 0.5
#endif
#ifndef NBHD_GAMMA
#define NBHD_GAMMA 0.01 /* wide-neighbourhood floor: t_r lambda_r >= gamma mu after a step */
#endif
#define STALL_ITERS 3   /* near-converged iterations without merit progress before stopping */
#ifndef REF_TOL
#define REF_TOL 1e-13 /* refinement stops once |correction| <= REF_TOL |dU| (kernel: kRefineTol) */
#endif

#ifndef WARM_STALL
#define WARM_STALL 3 /* kWarmStall (internal.h) */
#endif
#ifndef LR_MAX
#define LR_MAX 4
#endif
#ifndef CREF_TH
#define CREF_TH 1e10
#endif
#ifndef MU_FACTOR
#define MU_FACTOR 1e4   /* merit max(res, MU_FACTOR mu); lab: the fp32 kernels use 10 */
#endif
#ifndef T0_FLOOR
#define T0_FLOOR 0.5    /* starting slacks t_r = max(w_r - g_r, T0_FLOOR) (internal.h kT0Floor): stage-wise methods */
#endif
#ifndef T0_FLOOR_COND
#define T0_FLOOR_COND 0.1 /* ... the condensed method (newton 0; kT0FloorCond) */
#endif

static int chol(double* K, int n) {
    for (int j = 0; j < n; ++j) {
        double d = K[IDX2(j, j, n)];
        for (int p = 0; p < j; ++p) d -= K[IDX2(j, p, n)] * K[IDX2(j, p, n)];
#ifdef WRIGHT_PIVOT
        /* lab: Wright's modified Cholesky — a pivot lost to cancellation (<= WRIGHT_PIVOT times the
           original diagonal) is replaced by a huge one, which drops that component of the step */
        if (!(d > WRIGHT_PIVOT * K[IDX2(j, j, n)])) d = 1e128;
#else
        if (!(d > 0.0)) return -1;
#endif
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


#ifdef RIC_DEBUG
#define NEWTON_C 0
#else
#define NEWTON_C (S->newton)
#endif
/* ---- stage-wise Riccati Newton solve (mirrors colaborativempc-_amd/csrc/mpc_riccati.hip) ----
 * The condensed Newton system K dU = rhs is the LQ problem
 *   min sum_{k>=1} 1/2 dX_k'W_k dX_k + sum_k 1/2 v_k'(2R + th_k) v_k + 1/2 (v_k - v_{k-1})'2dR(.) - rhs'v
 *   s.t. dX_{k+1} = A_k dX_k + B_k v_k, dX_0 = 0, v_{-1} = 0,
 * solved on the augmented state y_k = [dX_k; v_{k-1}] (na = nx + nu). */
#define NA_MAX 16
#define NU_MAX 4

/* W = 2Q + M (stable group Schur form) for the stage rows of block k (rows of X_{k+1}) */
static void stage_w(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, int k, double* W) {
    const int nx = S->nx, mc = S->mc, ns = S->ns;
    for (int s = 0; s < nx * nx; ++s) W[s] = 2.0 * S->Q[s];
    for (int r = 0; r < mc; ++r) {
        const double* c1 = a->C + ((size_t)k * mc + r) * nx;
        double th1 = th[k * mc + r];
        int j = S->row_slack[r];
        if (j < 0) {
            for (int s = 0; s < nx; ++s) for (int u = 0; u < nx; ++u) W[s * nx + u] += th1 * c1[s] * c1[u];
            continue;
        }
        double inv = 1.0 / Dsig[k * ns + j], q = 2.0 * S->Qs[j];
        for (int s = 0; s < nx; ++s) for (int u = 0; u < nx; ++u) W[s * nx + u] += q * th1 * c1[s] * c1[u] * inv;
        for (int r2 = r + 1; r2 < mc; ++r2) {
            if (S->row_slack[r2] != j) continue;
            const double* c2 = a->C + ((size_t)k * mc + r2) * nx;
            double th2 = th[k * mc + r2], s1 = S->row_sign[r], s2 = S->row_sign[r2];
            for (int s = 0; s < nx; ++s)
                for (int u = 0; u < nx; ++u)
                    W[s * nx + u] += th1 * th2 * (s1 * c1[s] - s2 * c2[s]) * (s1 * c1[u] - s2 * c2[u]) * inv;
        }
    }
}

/* gains F_k = [K_k (nu x na) | Hinv_k (nu x nu)];  returns -1 on a non-positive pivot */
static int ric_factor(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, double* F) {
    const int nx = S->nx, nu = S->nu, N = S->N, na = nx + nu, ms = N * S->mc, sF = nu * na + nu * nu;
    double P[NA_MAX * NA_MAX], Pn[NA_MAX * NA_MAX], W[NA_MAX * NA_MAX], H[NU_MAX * NU_MAX], Hy[NU_MAX * NA_MAX];
    double Lf[NU_MAX * NU_MAX], Hi[NU_MAX * NU_MAX], Acl[NA_MAX * NA_MAX], T[NA_MAX * NA_MAX];
    memset(P, 0, sizeof P);
    stage_w(S, a, th, Dsig, N - 1, W);
    for (int i = 0; i < nx; ++i) for (int j = 0; j < nx; ++j) P[i * na + j] = W[i * nx + j];
    for (int k = N - 1; k >= 0; --k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        /* Bb = [B_k; I] (na x nu), Ab = [[A_k, 0], [0, 0]];  PB = P Bb */
        double PB[NA_MAX * NU_MAX];
        for (int i = 0; i < na; ++i)
            for (int c = 0; c < nu; ++c) {
                double v = P[i * na + nx + c];
                for (int s = 0; s < nx; ++s) v += P[i * na + s] * Bk[s * nu + c];
                PB[i * nu + c] = v;
            }
        /* Hvv = 2R + 2dR + diag(th_u) + Bb'P Bb */
        for (int c = 0; c < nu; ++c)
            for (int e = 0; e < nu; ++e) {
                double v = 2.0 * S->R[c * nu + e] + 2.0 * S->dR[c * nu + e] + PB[(nx + c) * nu + e];
                for (int s = 0; s < nx; ++s) v += Bk[s * nu + c] * PB[s * nu + e];
                if (c == e) { int r = ms + 2 * (k * nu + c); v += th[r] + th[r + 1]; }
                H[c * nu + e] = v;
            }
        /* Hvy = [Bb'P[:, :nx] A_k | -2dR] */
        for (int c = 0; c < nu; ++c)
            for (int j = 0; j < na; ++j) {
                double v = 0.0;
                if (j < nx)
                    for (int s = 0; s < nx; ++s) v += PB[s * nu + c] * Ak[s * nx + j];
                else
                    v = -2.0 * S->dR[c * nu + (j - nx)];
                Hy[c * na + j] = v;
            }
        /* Cholesky of Hvv and its inverse */
        for (int j = 0; j < nu; ++j) {
            double d = H[j * nu + j];
            for (int p = 0; p < j; ++p) d -= Lf[j * nu + p] * Lf[j * nu + p];
            if (!(d > 0.0)) return -1;
            d = sqrt(d);
            Lf[j * nu + j] = d;
            for (int i = j + 1; i < nu; ++i) {
                double v = H[i * nu + j];
                for (int p = 0; p < j; ++p) v -= Lf[i * nu + p] * Lf[j * nu + p];
                Lf[i * nu + j] = v / d;
            }
        }
        for (int c = 0; c < nu; ++c) {
            double e[NU_MAX];
            for (int i = 0; i < nu; ++i) e[i] = (i == c) ? 1.0 : 0.0;
            for (int i = 0; i < nu; ++i) {
                double v = e[i];
                for (int p = 0; p < i; ++p) v -= Lf[i * nu + p] * e[p];
                e[i] = v / Lf[i * nu + i];
            }
            for (int i = nu - 1; i >= 0; --i) {
                double v = e[i];
                for (int p = i + 1; p < nu; ++p) v -= Lf[p * nu + i] * e[p];
                e[i] = v / Lf[i * nu + i];
            }
            for (int i = 0; i < nu; ++i) Hi[i * nu + c] = e[i];
        }
        double* Fk = F + (size_t)k * sF;
        for (int c = 0; c < nu; ++c)
            for (int j = 0; j < na; ++j) {
                double v = 0.0;
                for (int e = 0; e < nu; ++e) v -= Hi[c * nu + e] * Hy[e * na + j];
                Fk[c * na + j] = v;
            }
        for (int c = 0; c < nu * nu; ++c) Fk[nu * na + c] = Hi[c];
        if (k == 0) break;
        stage_w(S, a, th, Dsig, k - 1, W);
        const double* Kk = Fk;
        if (S->newton == 2) {
            /* Joseph form: P_k = blkdiag(W_k, 0) + K'(2R + th)K + (K - E)'2dR(K - E) + Acl'P Acl,
               Acl = Ab + Bb K, E = [0 | I]: a sum of PSD terms */
            for (int i = 0; i < na; ++i)
                for (int j = 0; j < na; ++j) {
                    double v;
                    if (i < nx) {
                        v = (j < nx) ? Ak[i * nx + j] : 0.0;
                        for (int c = 0; c < nu; ++c) v += Bk[i * nu + c] * Kk[c * na + j];
                    } else {
                        v = Kk[(i - nx) * na + j];
                    }
                    Acl[i * na + j] = v;
                }
            for (int i = 0; i < na; ++i)
                for (int j = 0; j < na; ++j) {
                    double v = 0.0;
                    for (int s = 0; s < na; ++s) v += P[i * na + s] * Acl[s * na + j];
                    T[i * na + j] = v;
                }
            for (int i = 0; i < na; ++i)
                for (int j = 0; j <= i; ++j) {
                    double v = (i < nx && j < nx) ? W[i * nx + j] : 0.0;
                    for (int s = 0; s < na; ++s) v += Acl[s * na + i] * T[s * na + j];
                    for (int c = 0; c < nu; ++c) {
                        const double kc_i = Kk[c * na + i], kc_j = Kk[c * na + j];
                        double ru = 0.0;
                        for (int e = 0; e < nu; ++e) {
                            const double ke_j = Kk[e * na + j];
                            ru += 2.0 * S->R[c * nu + e] * ke_j;
                            const double d_i = kc_i - ((i >= nx && i - nx == c) ? 1.0 : 0.0);
                            const double d_j = ke_j - ((j >= nx && j - nx == e) ? 1.0 : 0.0);
                            v += d_i * 2.0 * S->dR[c * nu + e] * d_j;
                        }
                        const int r = ms + 2 * (k * nu + c);
                        v += kc_i * (ru + (th[r] + th[r + 1]) * kc_j);
                    }
                    Pn[i * na + j] = v;
                    Pn[j * na + i] = v;
                }
        } else {
            /* P_k = blkdiag(W_k + A'Pxx A, 2dR) + Hvy'K */
            for (int i = 0; i < na; ++i)
                for (int j = 0; j <= i; ++j) {
                    double v;
                    if (i < nx) {
                        v = W[i * nx + j];
                        for (int s = 0; s < nx; ++s) {
                            double pa = 0.0;
                            for (int t2 = 0; t2 < nx; ++t2) pa += P[s * na + t2] * Ak[t2 * nx + j];
                            v += Ak[s * nx + i] * pa;
                        }
                    } else {
                        v = (j >= nx) ? 2.0 * S->dR[(i - nx) * nu + (j - nx)] : 0.0;
                    }
                    for (int c = 0; c < nu; ++c) v += Hy[c * na + i] * Kk[c * na + j];
                    Pn[i * na + j] = v;
                    Pn[j * na + i] = v;
                }
        }
        memcpy(P, Pn, sizeof(double) * na * na);
    }
    return 0;
}

#ifdef RIC_QUAD
#include <quadmath.h>
typedef __float128 RQ;
/* gains F_k = [K_k (nu x na) | Hinv_k (nu x nu)];  returns -1 on a non-positive pivot */
static int ric_factor_q(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, double* F) {
    const int nx = S->nx, nu = S->nu, N = S->N, na = nx + nu, ms = N * S->mc, sF = nu * na + nu * nu;
    RQ P[NA_MAX * NA_MAX], Pn[NA_MAX * NA_MAX], H[NU_MAX * NU_MAX], Hy[NU_MAX * NA_MAX]; double W[NA_MAX * NA_MAX];
    RQ Lf[NU_MAX * NU_MAX], Hi[NU_MAX * NU_MAX], Acl[NA_MAX * NA_MAX], T[NA_MAX * NA_MAX], Kq[NU_MAX * NA_MAX];
    memset(P, 0, sizeof P);
    stage_w(S, a, th, Dsig, N - 1, W);
    for (int i = 0; i < nx; ++i) for (int j = 0; j < nx; ++j) P[i * na + j] = W[i * nx + j];
    for (int k = N - 1; k >= 0; --k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        /* Bb = [B_k; I] (na x nu), Ab = [[A_k, 0], [0, 0]];  PB = P Bb */
        RQ PB[NA_MAX * NU_MAX];
        for (int i = 0; i < na; ++i)
            for (int c = 0; c < nu; ++c) {
                RQ v = P[i * na + nx + c];
                for (int s = 0; s < nx; ++s) v += P[i * na + s] * Bk[s * nu + c];
                PB[i * nu + c] = v;
            }
        /* Hvv = 2R + 2dR + diag(th_u) + Bb'P Bb */
        for (int c = 0; c < nu; ++c)
            for (int e = 0; e < nu; ++e) {
                RQ v = (RQ)(2.0 * S->R[c * nu + e] + 2.0 * S->dR[c * nu + e]) + PB[(nx + c) * nu + e];
                for (int s = 0; s < nx; ++s) v += Bk[s * nu + c] * PB[s * nu + e];
                if (c == e) { int r = ms + 2 * (k * nu + c); v += th[r] + th[r + 1]; }
                H[c * nu + e] = v;
            }
        /* Hvy = [Bb'P[:, :nx] A_k | -2dR] */
        for (int c = 0; c < nu; ++c)
            for (int j = 0; j < na; ++j) {
                RQ v = 0.0;
                if (j < nx)
                    for (int s = 0; s < nx; ++s) v += PB[s * nu + c] * Ak[s * nx + j];
                else
                    v = -2.0 * S->dR[c * nu + (j - nx)];
                Hy[c * na + j] = v;
            }
        /* Cholesky of Hvv and its inverse */
        for (int j = 0; j < nu; ++j) {
            RQ d = H[j * nu + j];
            for (int p = 0; p < j; ++p) d -= Lf[j * nu + p] * Lf[j * nu + p];
            if (!(d > 0.0)) return -1;
            d = sqrtq(d);
            Lf[j * nu + j] = d;
            for (int i = j + 1; i < nu; ++i) {
                RQ v = H[i * nu + j];
                for (int p = 0; p < j; ++p) v -= Lf[i * nu + p] * Lf[j * nu + p];
                Lf[i * nu + j] = v / d;
            }
        }
        for (int c = 0; c < nu; ++c) {
            RQ e[NU_MAX];
            for (int i = 0; i < nu; ++i) e[i] = (i == c) ? 1.0 : 0.0;
            for (int i = 0; i < nu; ++i) {
                RQ v = e[i];
                for (int p = 0; p < i; ++p) v -= Lf[i * nu + p] * e[p];
                e[i] = v / Lf[i * nu + i];
            }
            for (int i = nu - 1; i >= 0; --i) {
                RQ v = e[i];
                for (int p = i + 1; p < nu; ++p) v -= Lf[p * nu + i] * e[p];
                e[i] = v / Lf[i * nu + i];
            }
            for (int i = 0; i < nu; ++i) Hi[i * nu + c] = e[i];
        }
        double* Fk = F + (size_t)k * sF;
        for (int c = 0; c < nu; ++c)
            for (int j = 0; j < na; ++j) {
                RQ v = 0.0;
                for (int e = 0; e < nu; ++e) v -= Hi[c * nu + e] * Hy[e * na + j];
                Fk[c * na + j] = (double)v;
                Kq[c * na + j] = v;
            }
        for (int c = 0; c < nu * nu; ++c) Fk[nu * na + c] = (double)Hi[c];
        if (k == 0) break;
        stage_w(S, a, th, Dsig, k - 1, W);
        const RQ* Kk = Kq;
        if (S->newton == 2) {
            /* Joseph form: P_k = blkdiag(W_k, 0) + K'(2R + th)K + (K - E)'2dR(K - E) + Acl'P Acl,
               Acl = Ab + Bb K, E = [0 | I]: a sum of PSD terms */
            for (int i = 0; i < na; ++i)
                for (int j = 0; j < na; ++j) {
                    RQ v;
                    if (i < nx) {
                        v = (j < nx) ? Ak[i * nx + j] : 0.0;
                        for (int c = 0; c < nu; ++c) v += Bk[i * nu + c] * Kk[c * na + j];
                    } else {
                        v = Kk[(i - nx) * na + j];
                    }
                    Acl[i * na + j] = v;
                }
            for (int i = 0; i < na; ++i)
                for (int j = 0; j < na; ++j) {
                    RQ v = 0.0;
                    for (int s = 0; s < na; ++s) v += P[i * na + s] * Acl[s * na + j];
                    T[i * na + j] = v;
                }
            for (int i = 0; i < na; ++i)
                for (int j = 0; j <= i; ++j) {
                    RQ v = (i < nx && j < nx) ? W[i * nx + j] : 0.0;
                    for (int s = 0; s < na; ++s) v += Acl[s * na + i] * T[s * na + j];
                    for (int c = 0; c < nu; ++c) {
                        const RQ kc_i = Kk[c * na + i], kc_j = Kk[c * na + j];
                        RQ ru = 0.0;
                        for (int e = 0; e < nu; ++e) {
                            const RQ ke_j = Kk[e * na + j];
                            ru += 2.0 * S->R[c * nu + e] * ke_j;
                            const RQ d_i = kc_i - ((i >= nx && i - nx == c) ? 1.0 : 0.0);
                            const RQ d_j = ke_j - ((j >= nx && j - nx == e) ? 1.0 : 0.0);
                            v += d_i * 2.0 * S->dR[c * nu + e] * d_j;
                        }
                        const int r = ms + 2 * (k * nu + c);
                        v += kc_i * (ru + (th[r] + th[r + 1]) * kc_j);
                    }
                    Pn[i * na + j] = v;
                    Pn[j * na + i] = v;
                }
        } else {
            /* P_k = blkdiag(W_k + A'Pxx A, 2dR) + Hvy'K */
            for (int i = 0; i < na; ++i)
                for (int j = 0; j <= i; ++j) {
                    RQ v;
                    if (i < nx) {
                        v = W[i * nx + j];
                        for (int s = 0; s < nx; ++s) {
                            RQ pa = 0.0;
                            for (int t2 = 0; t2 < nx; ++t2) pa += P[s * na + t2] * Ak[t2 * nx + j];
                            v += Ak[s * nx + i] * pa;
                        }
                    } else {
                        v = (j >= nx) ? 2.0 * S->dR[(i - nx) * nu + (j - nx)] : 0.0;
                    }
                    for (int c = 0; c < nu; ++c) v += Hy[c * na + i] * Kk[c * na + j];
                    Pn[i * na + j] = v;
                    Pn[j * na + i] = v;
                }
        }
        memcpy(P, Pn, sizeof(RQ) * na * na);
    }
    return 0;
}

#endif
/* dU, dX for the right-hand side rhs with the gains F */
static void ric_solve(const shared_t* S, const agent_t* a, const double* F, const double* rhs, double* dU, double* dX) {
    const int nx = S->nx, nu = S->nu, N = S->N, na = nx + nu, sF = nu * na + nu * nu;
    double p[NA_MAX], pn[NA_MAX], g[NA_MAX];
    memset(p, 0, sizeof p);
    for (int k = N - 1; k >= 0; --k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        const double* Kg = F + (size_t)k * sF;
        const double* Hg = Kg + nu * na;
        for (int c = 0; c < nu; ++c) {
            double v = p[nx + c] - rhs[k * nu + c];
            for (int s = 0; s < nx; ++s) v += Bk[s * nu + c] * p[s];
            g[c] = v;
        }
        for (int c = 0; c < nu; ++c) {
            double v = 0.0;
            for (int e = 0; e < nu; ++e) v -= Hg[c * nu + e] * g[e];
            dU[k * nu + c] = v;
        }
        for (int j = 0; j < na; ++j) {
            double v = 0.0;
            if (j < nx)
                for (int s = 0; s < nx; ++s) v += Ak[s * nx + j] * p[s];
            for (int c = 0; c < nu; ++c) v += Kg[c * na + j] * g[c];
            pn[j] = v;
        }
        memcpy(p, pn, sizeof(double) * na);
    }
    for (int s = 0; s < nx; ++s) dX[s] = 0.0;
    for (int k = 0; k < N; ++k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        const double* Kg = F + (size_t)k * sF;
        for (int c = 0; c < nu; ++c) {
            double v = dU[k * nu + c];
            for (int j = 0; j < nx; ++j) v += Kg[c * na + j] * dX[k * nx + j];
            if (k > 0)
                for (int e = 0; e < nu; ++e) v += Kg[c * na + nx + e] * dU[(k - 1) * nu + e];
            dU[k * nu + c] = v;
        }
        for (int s = 0; s < nx; ++s) {
            double v = 0.0;
            for (int t2 = 0; t2 < nx; ++t2) v += Ak[s * nx + t2] * dX[k * nx + t2];
            for (int c = 0; c < nu; ++c) v += Bk[s * nu + c] * dU[k * nu + c];
            dX[(k + 1) * nx + s] = v;
        }
    }
}


#ifdef RIC_F32
/* lab: the Riccati factorisation and Newton solves in single precision (gains, cost-to-go and every
   operation of ric_factor / ric_solve in float), iterates and residuals in double — the mixed
   scheme of an fp32 stage-wise kernel (tools/f32_lab.py) */
static int ric_factor_f32(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, double* F) {
    const int nx = S->nx, nu = S->nu, N = S->N, na = nx + nu, ms = N * S->mc, sF = nu * na + nu * nu;
    float P[NA_MAX * NA_MAX], Pn[NA_MAX * NA_MAX], H[NU_MAX * NU_MAX], Hy[NU_MAX * NA_MAX];
    float Lf[NU_MAX * NU_MAX], Hi[NU_MAX * NU_MAX], Ak[NA_MAX * NA_MAX], Bk[NA_MAX * NU_MAX], PB[NA_MAX * NU_MAX];
    double W[NA_MAX * NA_MAX];
    memset(P, 0, sizeof P);
    stage_w(S, a, th, Dsig, N - 1, W);
    for (int i = 0; i < nx; ++i) for (int j = 0; j < nx; ++j) P[i * na + j] = (float)W[i * nx + j];
    for (int k = N - 1; k >= 0; --k) {
        for (int i = 0; i < nx * nx; ++i) Ak[i] = (float)a->A[(size_t)k * nx * nx + i];
        for (int i = 0; i < nx * nu; ++i) Bk[i] = (float)a->B[(size_t)k * nx * nu + i];
        for (int i = 0; i < na; ++i)
            for (int c = 0; c < nu; ++c) {
                float v = P[i * na + nx + c];
                for (int s2 = 0; s2 < nx; ++s2) v += P[i * na + s2] * Bk[s2 * nu + c];
                PB[i * nu + c] = v;
            }
        for (int c = 0; c < nu; ++c)
            for (int e = 0; e < nu; ++e) {
                float v = (float)(2.0 * S->R[c * nu + e] + 2.0 * S->dR[c * nu + e]) + PB[(nx + c) * nu + e];
                for (int s2 = 0; s2 < nx; ++s2) v += Bk[s2 * nu + c] * PB[s2 * nu + e];
                if (c == e) { int r = ms + 2 * (k * nu + c); v += (float)(th[r] + th[r + 1]); }
                H[c * nu + e] = v;
            }
        for (int c = 0; c < nu; ++c)
            for (int j = 0; j < na; ++j) {
                float v = 0.0f;
                if (j < nx)
                    for (int s2 = 0; s2 < nx; ++s2) v += PB[s2 * nu + c] * Ak[s2 * nx + j];
                else
                    v = (float)(-2.0 * S->dR[c * nu + (j - nx)]);
                Hy[c * na + j] = v;
            }
        for (int j = 0; j < nu; ++j) {
            float d = H[j * nu + j];
            for (int q = 0; q < j; ++q) d -= Lf[j * nu + q] * Lf[j * nu + q];
            if (!(d > 0.0f)) return -1;
            d = sqrtf(d);
            Lf[j * nu + j] = d;
            for (int i = j + 1; i < nu; ++i) {
                float v = H[i * nu + j];
                for (int q = 0; q < j; ++q) v -= Lf[i * nu + q] * Lf[j * nu + q];
                Lf[i * nu + j] = v / d;
            }
        }
        for (int c = 0; c < nu; ++c) {
            float e[NU_MAX];
            for (int i = 0; i < nu; ++i) e[i] = (i == c) ? 1.0f : 0.0f;
            for (int i = 0; i < nu; ++i) {
                float v = e[i];
                for (int q = 0; q < i; ++q) v -= Lf[i * nu + q] * e[q];
                e[i] = v / Lf[i * nu + i];
            }
            for (int i = nu - 1; i >= 0; --i) {
                float v = e[i];
                for (int q = i + 1; q < nu; ++q) v -= Lf[q * nu + i] * e[q];
                e[i] = v / Lf[i * nu + i];
            }
            for (int i = 0; i < nu; ++i) Hi[i * nu + c] = e[i];
        }
        double* Fk = F + (size_t)k * sF;
        float Kk[NU_MAX * NA_MAX];
        for (int c = 0; c < nu; ++c)
            for (int j = 0; j < na; ++j) {
                float v = 0.0f;
                for (int e = 0; e < nu; ++e) v -= Hi[c * nu + e] * Hy[e * na + j];
                Kk[c * na + j] = v;
                Fk[c * na + j] = v;
            }
        for (int c = 0; c < nu * nu; ++c) Fk[nu * na + c] = Hi[c];
        if (k == 0) break;
        stage_w(S, a, th, Dsig, k - 1, W);
#ifdef RIC_F32_JOSEPH
        {   /* Joseph form in float: P_k = blkdiag(W_k, 0) + K'(2R + th)K + (K - E)'2dR(K - E) + Acl'P Acl */
            float Acl[NA_MAX * NA_MAX], T[NA_MAX * NA_MAX];
            for (int i = 0; i < na; ++i)
                for (int j = 0; j < na; ++j) {
                    float v;
                    if (i < nx) {
                        v = (j < nx) ? Ak[i * nx + j] : 0.0f;
                        for (int c = 0; c < nu; ++c) v += Bk[i * nu + c] * Kk[c * na + j];
                    } else {
                        v = Kk[(i - nx) * na + j];
                    }
                    Acl[i * na + j] = v;
                }
            for (int i = 0; i < na; ++i)
                for (int j = 0; j < na; ++j) {
                    float v = 0.0f;
                    for (int s2 = 0; s2 < na; ++s2) v += P[i * na + s2] * Acl[s2 * na + j];
                    T[i * na + j] = v;
                }
            for (int i = 0; i < na; ++i)
                for (int j = 0; j <= i; ++j) {
                    float v = (i < nx && j < nx) ? (float)W[i * nx + j] : 0.0f;
                    for (int s2 = 0; s2 < na; ++s2) v += Acl[s2 * na + i] * T[s2 * na + j];
                    for (int c = 0; c < nu; ++c) {
                        const float kc_i = Kk[c * na + i], kc_j = Kk[c * na + j];
                        float ru = 0.0f;
                        for (int e = 0; e < nu; ++e) {
                            const float ke_j = Kk[e * na + j];
                            ru += (float)(2.0 * S->R[c * nu + e]) * ke_j;
                            const float d_i = kc_i - ((i >= nx && i - nx == c) ? 1.0f : 0.0f);
                            const float d_j = ke_j - ((j >= nx && j - nx == e) ? 1.0f : 0.0f);
                            v += d_i * (float)(2.0 * S->dR[c * nu + e]) * d_j;
                        }
                        const int r = ms + 2 * (k * nu + c);
                        v += kc_i * (ru + (float)(th[r] + th[r + 1]) * kc_j);
                    }
                    Pn[i * na + j] = v;
                    Pn[j * na + i] = v;
                }
            memcpy(P, Pn, sizeof(float) * na * na);
            continue;
        }
#endif
        for (int i = 0; i < na; ++i)
            for (int j = 0; j <= i; ++j) {
                float v;
                if (i < nx) {
                    v = (float)W[i * nx + j];
                    for (int s2 = 0; s2 < nx; ++s2) {
                        float pa = 0.0f;
                        for (int t2 = 0; t2 < nx; ++t2) pa += P[s2 * na + t2] * Ak[t2 * nx + j];
                        v += Ak[s2 * nx + i] * pa;
                    }
                } else {
                    v = (j >= nx) ? (float)(2.0 * S->dR[(i - nx) * nu + (j - nx)]) : 0.0f;
                }
                for (int c = 0; c < nu; ++c) v += Hy[c * na + i] * Kk[c * na + j];
                Pn[i * na + j] = v;
                Pn[j * na + i] = v;
            }
        memcpy(P, Pn, sizeof(float) * na * na);
    }
    return 0;
}

static void ric_solve_f32(const shared_t* S, const agent_t* a, const double* F, const double* rhs, double* dU, double* dX) {
    const int nx = S->nx, nu = S->nu, N = S->N, na = nx + nu, sF = nu * na + nu * nu;
    float p[NA_MAX], pn[NA_MAX], g[NA_MAX];
    float* dUf = (float*)malloc(sizeof(float) * (size_t)N * nu);
    float* dXf = (float*)malloc(sizeof(float) * (size_t)(N + 1) * nx);
    memset(p, 0, sizeof p);
    for (int k = N - 1; k >= 0; --k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        const double* Kg = F + (size_t)k * sF;
        const double* Hg = Kg + nu * na;
        for (int c = 0; c < nu; ++c) {
            float v = p[nx + c] - (float)rhs[k * nu + c];
            for (int s2 = 0; s2 < nx; ++s2) v += (float)Bk[s2 * nu + c] * p[s2];
            g[c] = v;
        }
        for (int c = 0; c < nu; ++c) {
            float v = 0.0f;
            for (int e = 0; e < nu; ++e) v -= (float)Hg[c * nu + e] * g[e];
            dUf[k * nu + c] = v;
        }
        for (int j = 0; j < na; ++j) {
            float v = 0.0f;
            if (j < nx)
                for (int s2 = 0; s2 < nx; ++s2) v += (float)Ak[s2 * nx + j] * p[s2];
            for (int c = 0; c < nu; ++c) v += (float)Kg[c * na + j] * g[c];
            pn[j] = v;
        }
        memcpy(p, pn, sizeof(float) * na);
    }
    /* forward: the feedback in float, the state recursion dX_{k+1} = A dX_k + B dU_k in double (the
       iterate's X stays the simulation of its U) */
    for (int s2 = 0; s2 < nx; ++s2) dX[s2] = 0.0;
    for (int k = 0; k < N; ++k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        const double* Kg = F + (size_t)k * sF;
        for (int c = 0; c < nu; ++c) {
            float v = dUf[k * nu + c];
            for (int j = 0; j < nx; ++j) v += (float)Kg[c * na + j] * (float)dX[k * nx + j];
            if (k > 0)
                for (int e = 0; e < nu; ++e) v += (float)Kg[c * na + nx + e] * dUf[(k - 1) * nu + e];
            dUf[k * nu + c] = v;
            dU[k * nu + c] = v;
        }
        for (int s2 = 0; s2 < nx; ++s2) {
            double v = 0.0;
            for (int t2 = 0; t2 < nx; ++t2) v += Ak[s2 * nx + t2] * dX[k * nx + t2];
            for (int c = 0; c < nu; ++c) v += Bk[s2 * nu + c] * dU[k * nu + c];
            dX[(k + 1) * nx + s2] = v;
        }
    }
    (void)dXf;
    free(dUf);
    free(dXf);
}
long cmpc_f32_iters = 0, cmpc_f64_iters = 0, cmpc_f64_agents = 0; /* lab counters */
#ifndef F32_STALL
#define F32_STALL 2      /* lab: fp32 iterations without a new best before the agent switches to fp64 */
#endif
#ifndef F32_SWITCH_M
#define F32_SWITCH_M 0.0 /* lab: best merit below which the agent switches to fp64 (0: off) */
#endif
#endif

/* y = K v for the condensed Newton matrix K = sum_k Gamma_k'W_k Gamma_k + 2R + 2D'dR D + diag(th_u),
   matrix-free through the stage recursions (dX = Gamma v, then the adjoint) */
static void kmul(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, const double* v, double* y,
                 double* dX, double* yb, double* psi, double* tmp) {
    const int nx = S->nx, nu = S->nu, N = S->N, ms = N * S->mc;
    double W[NA_MAX * NA_MAX];
    fwd_sim(S, a, NULL, v, dX);
    for (int s = 0; s < nx; ++s) yb[s] = 0.0;
    for (int k = 1; k <= N; ++k) {
        stage_w(S, a, th, Dsig, k - 1, W);
        for (int s = 0; s < nx; ++s) {
            double acc = 0.0;
            for (int u = 0; u < nx; ++u) acc += W[s * nx + u] * dX[k * nx + u];
            yb[k * nx + s] = acc;
        }
    }
    adjoint(S, a, yb, y, psi, tmp);
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            double acc = 0.0;
            for (int j = 0; j < nu; ++j) {
                const double vk = v[k * nu + j];
                const double dk = vk - (k ? v[(k - 1) * nu + j] : 0.0);
                const double dn = (k + 1 < N) ? v[(k + 1) * nu + j] - vk : 0.0;
                acc += 2.0 * S->R[i * nu + j] * vk + 2.0 * S->dR[i * nu + j] * (dk - dn);
            }
            const int r = ms + 2 * (k * nu + i);
            y[k * nu + i] += acc + (th[r] + th[r + 1]) * v[k * nu + i];
        }
}


#ifdef RIC_QREF
#include <quadmath.h>
/* debug: the condensed Newton solve in quad precision (reference direction) */
static void condensed_q(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, const double* rhs,
                        double* out) {
    const int nx = S->nx, nu = S->nu, N = S->N, n = N * nu, mc = S->mc, ns = S->ns, ms = N * mc;
    __float128* G = calloc((size_t)(N + 1) * nx * n, sizeof(__float128));
    __float128* K = calloc((size_t)n * n, sizeof(__float128));
    __float128 W[NA_MAX * NA_MAX];
    for (int k = 0; k < N; ++k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        for (int s = 0; s < nx; ++s)
            for (int c = 0; c < n; ++c) {
                __float128 v = 0;
                for (int t = 0; t < nx; ++t) v += (__float128)Ak[s * nx + t] * G[((size_t)k * nx + t) * n + c];
                if (c >= k * nu && c < (k + 1) * nu) v += Bk[s * nu + (c - k * nu)];
                G[((size_t)(k + 1) * nx + s) * n + c] = v;
            }
    }
    for (int k = 0; k < N; ++k) {
        for (int s = 0; s < nx * nx; ++s) W[s] = 2.0 * S->Q[s];
        for (int r = 0; r < mc; ++r) {
            const double* c1 = a->C + ((size_t)k * mc + r) * nx;
            __float128 th1 = th[k * mc + r];
            int j = S->row_slack[r];
            if (j < 0) { for (int s = 0; s < nx; ++s) for (int u = 0; u < nx; ++u) W[s * nx + u] += th1 * c1[s] * c1[u]; continue; }
            __float128 D = 2.0 * S->Qs[j];
            for (int r2 = 0; r2 < mc; ++r2) if (S->row_slack[r2] == j) D += th[k * mc + r2];
            __float128 q = 2.0 * S->Qs[j];
            for (int s = 0; s < nx; ++s) for (int u = 0; u < nx; ++u) W[s * nx + u] += q * th1 * c1[s] * c1[u] / D;
            for (int r2 = r + 1; r2 < mc; ++r2) {
                if (S->row_slack[r2] != j) continue;
                const double* c2 = a->C + ((size_t)k * mc + r2) * nx;
                __float128 th2 = th[k * mc + r2], s1 = S->row_sign[r], s2 = S->row_sign[r2];
                for (int s = 0; s < nx; ++s) for (int u = 0; u < nx; ++u)
                    W[s * nx + u] += th1 * th2 * (s1 * c1[s] - s2 * c2[s]) * (s1 * c1[u] - s2 * c2[u]) / D;
            }
        }
        const __float128* Gk = G + (size_t)(k + 1) * nx * n;
        const int ncol = (k + 1) * nu;
        __float128* Y = calloc((size_t)nx * ncol, sizeof(__float128));
        for (int s = 0; s < nx; ++s) for (int c2 = 0; c2 < ncol; ++c2) { __float128 y = 0; for (int u = 0; u < nx; ++u) y += W[s * nx + u] * Gk[u * n + c2]; Y[s * ncol + c2] = y; }
        for (int c1 = 0; c1 < ncol; ++c1)
            for (int c2 = 0; c2 <= c1; ++c2) {
                __float128 v = 0;
                for (int s = 0; s < nx; ++s) v += Gk[s * n + c1] * Y[s * ncol + c2];
                K[(size_t)c1 * n + c2] += v;
            }
        free(Y);
    }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i)
            for (int j = 0; j < nu; ++j) {
                int ci = k * nu + i, cj = k * nu + j;
                __float128 v = 2.0 * S->R[i * nu + j] + 2.0 * S->dR[i * nu + j] * (k + 1 < N ? 2.0 : 1.0);
                if (cj <= ci) K[(size_t)ci * n + cj] += v;
                if (k > 0) K[(size_t)ci * n + (k - 1) * nu + j] += -2.0 * S->dR[i * nu + j];
            }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) { int r = ms + (k * nu + i) * 2; K[(size_t)(k * nu + i) * n + k * nu + i] += (__float128)th[r] + th[r + 1]; }
    for (int j = 0; j < n; ++j) {
        __float128 d = K[(size_t)j * n + j];
        for (int p = 0; p < j; ++p) d -= K[(size_t)j * n + p] * K[(size_t)j * n + p];
        d = sqrtq(d); K[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; ++i) { __float128 v = K[(size_t)i * n + j]; for (int p = 0; p < j; ++p) v -= K[(size_t)i * n + p] * K[(size_t)j * n + p]; K[(size_t)i * n + j] = v / d; }
    }
    __float128* b = calloc(n, sizeof(__float128));
    for (int i = 0; i < n; ++i) { __float128 v = rhs[i]; for (int p = 0; p < i; ++p) v -= K[(size_t)i * n + p] * b[p]; b[i] = v / K[(size_t)i * n + i]; }
    for (int i = n - 1; i >= 0; --i) { __float128 v = b[i]; for (int p = i + 1; p < n; ++p) v -= K[(size_t)p * n + i] * b[p]; b[i] = v / K[(size_t)i * n + i]; }
    for (int i = 0; i < n; ++i) out[i] = (double)b[i];
    free(G); free(K); free(b); (void)Dsig; (void)ns;
}
#endif


#ifdef KMUL_QUAD
#include <quadmath.h>
/* r = rhs - K v with the product in quad precision (residual for iterative refinement) */
static void kres_q(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, const double* v,
                   const double* rhs, double* out) {
    const int nx = S->nx, nu = S->nu, N = S->N, ms = N * S->mc;
    double W[NA_MAX * NA_MAX];
    __float128 X[(NA_MAX) * 256], Y[NA_MAX * 256], psi[NA_MAX], tmp[NA_MAX];
    for (int s = 0; s < nx; ++s) X[s] = 0;
    for (int k = 0; k < N; ++k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        for (int s = 0; s < nx; ++s) {
            __float128 acc = 0;
            for (int t = 0; t < nx; ++t) acc += (__float128)Ak[s * nx + t] * X[k * nx + t];
            for (int i = 0; i < nu; ++i) acc += (__float128)Bk[s * nu + i] * v[k * nu + i];
            X[(k + 1) * nx + s] = acc;
        }
    }
    for (int k = 1; k <= N; ++k) {
        stage_w(S, a, th, Dsig, k - 1, W);
        for (int s = 0; s < nx; ++s) {
            __float128 acc = 0;
            for (int u = 0; u < nx; ++u) acc += (__float128)W[s * nx + u] * X[k * nx + u];
            Y[k * nx + s] = acc;
        }
    }
    for (int s = 0; s < nx; ++s) psi[s] = Y[N * nx + s];
    for (int k = N - 1; k >= 0; --k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        for (int i = 0; i < nu; ++i) {
            __float128 acc = 0;
            for (int s = 0; s < nx; ++s) acc += (__float128)Bk[s * nu + i] * psi[s];
            for (int j = 0; j < nu; ++j) {
                const __float128 vk = v[k * nu + j];
                const __float128 dk = vk - (k ? (__float128)v[(k - 1) * nu + j] : 0);
                const __float128 dn = (k + 1 < N) ? (__float128)v[(k + 1) * nu + j] - vk : 0;
                acc += 2.0 * S->R[i * nu + j] * vk + 2.0 * S->dR[i * nu + j] * (dk - dn);
            }
            const int r = ms + 2 * (k * nu + i);
            acc += ((__float128)th[r] + th[r + 1]) * v[k * nu + i];
            out[k * nu + i] = (double)((__float128)rhs[k * nu + i] - acc);
        }
        if (k > 0) {
            for (int t = 0; t < nx; ++t) {
                __float128 acc = Y[k * nx + t];
                for (int s = 0; s < nx; ++s) acc += (__float128)Ak[s * nx + t] * psi[s];
                tmp[t] = acc;
            }
            for (int t = 0; t < nx; ++t) psi[t] = tmp[t];
        }
    }
}
#endif


/* ---- double-double arithmetic (hi + lo, |lo| <= ulp(hi)/2; fma-based, as the kernel's) ----
 * The Riccati factor and the refinement residual switch to it once max th exceeds RIC_DD_TH:
 * there the double recursion's error grows past what Newton can absorb (near the solution
 * th -> 1e18..1e21 on saturated inputs and collision rows; SURVEY M4's 1e8 conditioning). */
typedef struct { double hi, lo; } dd_t;
static inline dd_t dd_qts(double a, double b) { double s = a + b; dd_t r = {s, b - (s - a)}; return r; }
static inline dd_t dd_ts(double a, double b) {
    double s = a + b, bb = s - a;
    dd_t r = {s, (a - (s - bb)) + (b - bb)};
    return r;
}
static inline dd_t dd_add(dd_t x, dd_t y) {
    dd_t s = dd_ts(x.hi, y.hi);
    return dd_qts(s.hi, s.lo + x.lo + y.lo);
}
static inline dd_t dd_mul(dd_t x, dd_t y) {
    double p = x.hi * y.hi, e = fma(x.hi, y.hi, -p);
    e = fma(x.hi, y.lo, fma(x.lo, y.hi, e));
    return dd_qts(p, e);
}
static inline dd_t dd_muld(dd_t x, double y) {
    double p = x.hi * y, e = fma(x.hi, y, -p);
    e = fma(x.lo, y, e);
    return dd_qts(p, e);
}
static inline dd_t dd_fma(dd_t acc, dd_t x, dd_t y) { return dd_add(acc, dd_mul(x, y)); }
static inline dd_t dd_fmad(dd_t acc, dd_t x, double y) { return dd_add(acc, dd_muld(x, y)); }
static inline dd_t dd_d(double a) { dd_t r = {a, 0.0}; return r; }
static inline dd_t dd_neg(dd_t x) { dd_t r = {-x.hi, -x.lo}; return r; }
static inline dd_t dd_div(dd_t x, dd_t y) {
    double q1 = x.hi / y.hi;
    dd_t r = dd_add(x, dd_neg(dd_muld(y, q1)));
    double q2 = r.hi / y.hi;
    r = dd_add(r, dd_neg(dd_muld(y, q2)));
    double q3 = r.hi / y.hi;
    dd_t q = dd_qts(q1, q2);
    return dd_add(q, dd_d(q3));
}
static inline dd_t dd_sqrt(dd_t x) {
    double s = sqrt(x.hi);
    dd_t r = dd_add(x, dd_neg(dd_mul(dd_d(s), dd_d(s))));
    return dd_qts(s, r.hi / (2.0 * s));
}

#ifndef RIC_DD_TH
#define RIC_DD_TH 1e10
#endif
#ifndef RIC_REFINE_MAX
#define RIC_REFINE_MAX 6
#endif
#ifndef RIC_REFINE_WARM
#define RIC_REFINE_WARM 2
#endif

/* ric_factor in double-double (standard form); gains rounded to double */
static int ric_factor_dd(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, double* F) {
    const int nx = S->nx, nu = S->nu, N = S->N, na = nx + nu, ms = N * S->mc, sF = nu * na + nu * nu;
    dd_t P[NA_MAX * NA_MAX], Pn[NA_MAX * NA_MAX], H[NU_MAX * NU_MAX], Hy[NU_MAX * NA_MAX], Lf[NU_MAX * NU_MAX],
        Hi[NU_MAX * NU_MAX], Kk[NU_MAX * NA_MAX], PB[NA_MAX * NU_MAX], PA[NA_MAX * NA_MAX];
    double W[NA_MAX * NA_MAX];
    for (int e = 0; e < na * na; ++e) P[e] = dd_d(0.0);
    stage_w(S, a, th, Dsig, N - 1, W);
    for (int i = 0; i < nx; ++i) for (int j = 0; j < nx; ++j) P[i * na + j] = dd_d(W[i * nx + j]);
    for (int k = N - 1; k >= 0; --k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        for (int i = 0; i < na; ++i)
            for (int c = 0; c < nu; ++c) {
                dd_t v = P[i * na + nx + c];
                for (int s = 0; s < nx; ++s) v = dd_fmad(v, P[i * na + s], Bk[s * nu + c]);
                PB[i * nu + c] = v;
            }
        for (int c = 0; c < nu; ++c)
            for (int e = 0; e < nu; ++e) {
                dd_t v = dd_add(dd_d(2.0 * S->R[c * nu + e]), dd_add(dd_d(2.0 * S->dR[c * nu + e]), PB[(nx + c) * nu + e]));
                for (int s = 0; s < nx; ++s) v = dd_fmad(v, PB[s * nu + e], Bk[s * nu + c]);
                if (c == e) { int r = ms + 2 * (k * nu + c); v = dd_add(v, dd_add(dd_d(th[r]), dd_d(th[r + 1]))); }
                H[c * nu + e] = v;
            }
        /* PA = P[:, :nx] A_k (na x nx) */
        for (int i = 0; i < na; ++i)
            for (int j = 0; j < nx; ++j) {
                dd_t v = dd_d(0.0);
                for (int s = 0; s < nx; ++s) v = dd_fmad(v, P[i * na + s], Ak[s * nx + j]);
                PA[i * nx + j] = v;
            }
        for (int c = 0; c < nu; ++c)
            for (int j = 0; j < na; ++j) {
                dd_t v;
                if (j < nx) {
                    v = PA[(nx + c) * nx + j];
                    for (int s = 0; s < nx; ++s) v = dd_fmad(v, PA[s * nx + j], Bk[s * nu + c]);
                } else {
                    v = dd_d(-2.0 * S->dR[c * nu + (j - nx)]);
                }
                Hy[c * na + j] = v;
            }
        for (int j = 0; j < nu; ++j) {
            dd_t d = H[j * nu + j];
            for (int p = 0; p < j; ++p) d = dd_add(d, dd_neg(dd_mul(Lf[j * nu + p], Lf[j * nu + p])));
            if (!(d.hi > 0.0)) return -1;
            d = dd_sqrt(d);
            Lf[j * nu + j] = d;
            for (int i = j + 1; i < nu; ++i) {
                dd_t v = H[i * nu + j];
                for (int p = 0; p < j; ++p) v = dd_add(v, dd_neg(dd_mul(Lf[i * nu + p], Lf[j * nu + p])));
                Lf[i * nu + j] = dd_div(v, d);
            }
        }
        for (int c = 0; c < nu; ++c) {
            dd_t e[NU_MAX];
            for (int i = 0; i < nu; ++i) e[i] = dd_d(i == c ? 1.0 : 0.0);
            for (int i = 0; i < nu; ++i) {
                dd_t v = e[i];
                for (int p = 0; p < i; ++p) v = dd_add(v, dd_neg(dd_mul(Lf[i * nu + p], e[p])));
                e[i] = dd_div(v, Lf[i * nu + i]);
            }
            for (int i = nu - 1; i >= 0; --i) {
                dd_t v = e[i];
                for (int p = i + 1; p < nu; ++p) v = dd_add(v, dd_neg(dd_mul(Lf[p * nu + i], e[p])));
                e[i] = dd_div(v, Lf[i * nu + i]);
            }
            for (int i = 0; i < nu; ++i) Hi[i * nu + c] = e[i];
        }
        double* Fk = F + (size_t)k * sF;
        for (int c = 0; c < nu; ++c)
            for (int j = 0; j < na; ++j) {
                dd_t v = dd_d(0.0);
                for (int e = 0; e < nu; ++e) v = dd_add(v, dd_neg(dd_mul(Hi[c * nu + e], Hy[e * na + j])));
                Kk[c * na + j] = v;
                Fk[c * na + j] = v.hi;
            }
        for (int c = 0; c < nu * nu; ++c) Fk[nu * na + c] = Hi[c].hi;
        if (k == 0) break;
        stage_w(S, a, th, Dsig, k - 1, W);
        /* P_k = blkdiag(W_k + A'Pxx A, 2dR) + Hvy'K */
        for (int i = 0; i < na; ++i)
            for (int j = 0; j <= i; ++j) {
                dd_t v;
                if (i < nx) {
                    v = dd_d(W[i * nx + j]);
                    for (int s = 0; s < nx; ++s) v = dd_fmad(v, PA[s * nx + j], Ak[s * nx + i]);
                } else {
                    v = dd_d((j >= nx) ? 2.0 * S->dR[(i - nx) * nu + (j - nx)] : 0.0);
                }
                for (int c = 0; c < nu; ++c) v = dd_fma(v, Hy[c * na + i], Kk[c * na + j]);
                Pn[i * na + j] = v;
                Pn[j * na + i] = v;
            }
        memcpy(P, Pn, sizeof(dd_t) * na * na);
    }
    return 0;
}

/* out = rhs - K v, the product in double-double (refinement residual; K as in kmul) */
static void kres_dd(const shared_t* S, const agent_t* a, const double* th, const double* Dsig, const double* v,
                    const double* rhs, double* out, dd_t* X) {
    const int nx = S->nx, nu = S->nu, N = S->N, ms = N * S->mc;
    double W[NA_MAX * NA_MAX];
    dd_t psi[NA_MAX], tmp[NA_MAX], yk[NA_MAX];
    for (int s = 0; s < nx; ++s) X[s] = dd_d(0.0);
    for (int k = 0; k < N; ++k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        for (int s = 0; s < nx; ++s) {
            dd_t acc = dd_d(0.0);
            for (int t = 0; t < nx; ++t) acc = dd_fmad(acc, X[k * nx + t], Ak[s * nx + t]);
            for (int i = 0; i < nu; ++i) acc = dd_add(acc, dd_mul(dd_d(Bk[s * nu + i]), dd_d(v[k * nu + i])));
            X[(k + 1) * nx + s] = acc;
        }
    }
    for (int k = N; k >= 1; --k) { /* W_k X_k into X (in place, stage by stage from the end) */
        stage_w(S, a, th, Dsig, k - 1, W);
        for (int s = 0; s < nx; ++s) {
            dd_t acc = dd_d(0.0);
            for (int u = 0; u < nx; ++u) acc = dd_fmad(acc, X[k * nx + u], W[s * nx + u]);
            yk[s] = acc;
        }
        for (int s = 0; s < nx; ++s) X[k * nx + s] = yk[s];
    }
    for (int s = 0; s < nx; ++s) psi[s] = X[N * nx + s];
    for (int k = N - 1; k >= 0; --k) {
        const double* Ak = a->A + (size_t)k * nx * nx;
        const double* Bk = a->B + (size_t)k * nx * nu;
        for (int i = 0; i < nu; ++i) {
            dd_t acc = dd_d(0.0);
            for (int s = 0; s < nx; ++s) acc = dd_fmad(acc, psi[s], Bk[s * nu + i]);
            for (int j = 0; j < nu; ++j) {
                const double vk = v[k * nu + j];
                const dd_t dk = dd_ts(vk, k ? -v[(k - 1) * nu + j] : 0.0);
                const dd_t dn = (k + 1 < N) ? dd_ts(v[(k + 1) * nu + j], -vk) : dd_d(0.0);
                acc = dd_add(acc, dd_mul(dd_d(2.0 * S->R[i * nu + j]), dd_d(vk)));
                acc = dd_fmad(acc, dd_add(dk, dd_neg(dn)), 2.0 * S->dR[i * nu + j]);
            }
            const int r = ms + 2 * (k * nu + i);
            acc = dd_fmad(acc, dd_add(dd_d(th[r]), dd_d(th[r + 1])), v[k * nu + i]);
            dd_t res = dd_add(dd_d(rhs[k * nu + i]), dd_neg(acc));
            out[k * nu + i] = res.hi;
        }
        if (k > 0) {
            for (int t = 0; t < nx; ++t) {
                dd_t acc = X[k * nx + t];
                for (int s = 0; s < nx; ++s) acc = dd_fmad(acc, psi[s], Ak[s * nx + t]);
                tmp[t] = acc;
            }
            for (int t = 0; t < nx; ++t) psi[t] = tmp[t];
        }
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
    dd_t* Xdd;
    double *bU, *bsig, *Gam, *K, *X, *dX, *U, *dU, *sig, *dsig, *Dsig, *rsig, *t, *lam, *th, *rho, *rt, *rp, *w,
        *dt_a, *dl_a, *dtv, *dlv, *GdU, *ybar, *gU, *rd, *rhs, *psi, *tmp, *W, *Yk, *F;
    unsigned char* act;
} work_t;

/* value of row r at (X, U, sigma): stage rows c'X_{k+1} (+ sign sigma_kj), input rows +-u */
static double row_val(const shared_t* S, const agent_t* a, const double* X, const double* U, const double* sig, int r) {
    const int nx = S->nx, ns = S->ns, mc = S->mc, ms = S->N * mc;
    if (r < ms) {
        const int k = r / mc, rr = r % mc;
        const double* c = a->C + ((size_t)k * mc + rr) * nx;
        double v = 0.0;
        for (int s = 0; s < nx; ++s) v += c[s] * X[(k + 1) * nx + s];
        const int j = S->row_slack[rr];
        if (j >= 0 && sig) v += S->row_sign[rr] * sig[k * ns + j];
        return v;
    }
    const int q = r - ms;
    return (q & 1) ? -U[q / 2] : U[q / 2];
}

/* The interior-point method's scaled residuals at (U, sigma, t, lambda) — the loop of solve_one
   (stationarity rd, slack stationarity rsig, rows rp, mu), into wk->rd / rsig / rp; X is
   re-simulated from U.  Returns the merit max(res, MU_FACTOR mu), *kkt = max(res, mu). */
static double merit_at(const shared_t* S, const agent_t* a, work_t* wk, const double* U, const double* sig,
                       const double* t, const double* lam, double* X, double* kkt) {
    const int nx = S->nx, nu = S->nu, N = S->N, ns = S->ns, mc = S->mc;
    const int n = N * nu, ms = N * mc, m = ms + 2 * nu * N;
    fwd_sim(S, a, a->x0, U, X);
    double* ybar = wk->ybar;
    for (int k = 0; k <= N; ++k)
        for (int s = 0; s < nx; ++s) {
            double v = 2.0 * a->p[k * nx + s];
            for (int t2 = 0; t2 < nx; ++t2) v += 2.0 * S->Q[s * nx + t2] * X[k * nx + t2];
            ybar[k * nx + s] = v;
        }
    double gscale = 1.0;
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
            gscale = nmax(gscale, fabs(wk->gU[k * nu + i]));
        }
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
            const int r = ms + (k * nu + i) * 2;
            wk->rd[k * nu + i] += v + lam[r] - lam[r + 1];
        }
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < ns; ++j) {
            double v = 2.0 * S->Qs[j] * sig[k * ns + j];
            for (int r = 0; r < mc; ++r)
                if (S->row_slack[r] == j) v += S->row_sign[r] * lam[k * mc + r];
            wk->rsig[k * ns + j] = v;
        }
    double mu = 0.0, nrp = 0.0, nrd = 0.0, nrs = 0.0, scale_p = 1.0, qs_max = 1.0;
    int mact = 0;
    for (int r = 0; r < m; ++r) {
        if (!wk->act[r]) { wk->rp[r] = 0.0; continue; }
        wk->rp[r] = row_val(S, a, X, U, sig, r) + t[r] - wk->w[r];
        nrp = nmax(nrp, fabs(wk->rp[r]));
        mu += t[r] * lam[r];
        ++mact;
        if (fabs(wk->w[r]) > scale_p) scale_p = fabs(wk->w[r]);
    }
    for (int j = 0; j < ns; ++j) if (2 * S->Qs[j] > qs_max) qs_max = 2 * S->Qs[j];
    mu = mact ? mu / mact : 0.0;
    for (int c = 0; c < n; ++c) nrd = nmax(nrd, fabs(wk->rd[c]));
    for (int q = 0; q < N * ns; ++q) nrs = nmax(nrs, fabs(wk->rsig[q]));
    const double res = nmax(nmax(nrd / gscale, nrs / qs_max), nrp / scale_p);
    *kkt = nmax(res, mu);
    return nmax(res, MU_FACTOR * mu);
}

#ifndef POLISH_MAX_ACTIVE
#define POLISH_MAX_ACTIVE 96  /* kPolishMaxActive (mpc_polish.hip): larger active sets are not polished.  The
                                 kernel lowers it in steps of 8 until its LDS image fits (pol_layout); the
                                 caller passes that value in (newton bits 16..23, cmpc_plan_info's
                                 polish_max_active) so both sides polish the same agents */
#endif
#ifdef LAB_SIGMA2
#ifndef LAB_SIGMA2_RULE
#define LAB_SIGMA2_RULE(s) fmax(10.0 * (s), 0.1)
#endif
#ifndef LAB_SIGMA2_MARGIN
#define LAB_SIGMA2_MARGIN 1.0
#endif
#endif
#ifndef POLISH_DEGENERATE
#define POLISH_DEGENERATE 1e-9 /* kPolishDegenerate (internal.h) */
#endif
#ifndef POLISH_STEPS
#define POLISH_STEPS 3        /* kPolishSteps: Newton steps on the (linear) equality-constrained KKT system */
#endif
#ifndef POLISH_PASSES
#define POLISH_PASSES 2       /* kPolishPasses: active-set corrections (negative multipliers out, violated rows in) */
#endif

/* Polish (CMPC_FLAG_POLISH) — OSQP's `polish=True` (LPV_Planner.py:233) restated for the
   interior-point iterate.  From an iterate at the rounding floor (t, lambda), the active set
   A = {r : lambda_r > t_r} is taken as exact: the equality-constrained QP
       min f(U) + sum Qs sigma^2   s.t.   row_r(U, sigma) = w_r  (r in A)
   is solved by Newton steps on its (linear) KKT system from (U, sigma, lambda_A), each through the
   range-space form:  H = the condensed Hessian of f (the Newton matrix without any theta: 2Q
   stage weights, 2R, 2dR; well conditioned), G_A = the active rows as functions of U (c'Gamma_{k+1}
   or +-e_i), E = the slack coupling (sign_r sign_r' / 2Qs_j within a slack group):
       S dlam = rA' - G_A H^-1 rU,   dU = -H^-1 (rU + G_A' dlam),   S = G_A H^-1 G_A' + E,
       dsig = -(rsig + sign' dlam) / 2Qs,   rA' = rA - sign rsig / 2Qs.
   The polished point (t = max(w - row, 0), lambda = max(lambda_A, 0) on A, 0 elsewhere) replaces
   the iterate when its merit is below the best merit the method reached (status 1 below tol).
   The condensed Gamma (wk->Gam) must be built; wk->K is overwritten.  Returns the merit of the
   polished point (+inf when H or S is not positive definite or |A| > POLISH_MAX_ACTIVE), and
   the polished U, sigma, kkt in Up, sigp, *kkt. */
static double polish_one(const shared_t* S, const agent_t* a, work_t* wk, double tol, const double* U, const double* sig,
                         const double* t, const double* lam, double* Up, double* sigp, double* kkt) {
    const int nx = S->nx, nu = S->nu, N = S->N, ns = S->ns, mc = S->mc;
    const int n = N * nu, ms = N * mc, m = ms + 2 * nu * N;
    const int amax = S->polish_amax > 0 ? S->polish_amax : POLISH_MAX_ACTIVE;
    unsigned char* in = malloc((size_t)m);
    int* Ar = malloc(sizeof(int) * amax);
    double* GA = malloc(sizeof(double) * (2 * (size_t)amax * n + (size_t)amax * amax + 3 * (size_t)amax +
                                          3 * (size_t)n + (size_t)N * ns + (size_t)m));
    double *Y = GA + (size_t)amax * n, *Ssch = Y + (size_t)amax * n, *lA = Ssch + (size_t)amax * amax;
    double *rA = lA + amax, *dl = rA + amax, *v = dl + amax, *gv = v + n, *Uc = gv + n, *sc = Uc + n, *lamp = sc + N * ns;
    double best = INFINITY;
    double* X = wk->dX;
    const double* Gam = wk->Gam;
#ifndef POL_AFAC
#define POL_AFAC 1.0
#endif
    for (int r = 0; r < m; ++r) in[r] = wk->act[r] && lam[r] > POL_AFAC * t[r];
    /* H: the condensed Newton matrix with every theta = 0 (solve_one's K build) */
    double* K = wk->K;
    memset(K, 0, sizeof(double) * n * n);
    for (int k = 0; k < N; ++k) {
        const double* G = Gam + (size_t)(k + 1) * nx * n;
        const int ncol = (k + 1) * nu;
        double* Yk = wk->Yk;
        for (int s = 0; s < nx; ++s)
            for (int c2 = 0; c2 < ncol; ++c2) {
                double acc = 0.0;
                for (int u = 0; u < nx; ++u) acc += 2.0 * S->Q[s * nx + u] * G[u * n + c2];
                Yk[s * n + c2] = acc;
            }
        for (int c1 = 0; c1 < ncol; ++c1)
            for (int c2 = 0; c2 <= c1; ++c2) {
                double acc = 0.0;
                for (int s = 0; s < nx; ++s) acc += G[s * n + c1] * Yk[s * n + c2];
                K[IDX2(c1, c2, n)] += acc;
            }
    }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i)
            for (int j = 0; j < nu; ++j) {
                const int ci = k * nu + i, cj = k * nu + j;
                const double d = 2.0 * S->R[i * nu + j] + 2.0 * S->dR[i * nu + j] * (k + 1 < N ? 2.0 : 1.0);
                if (cj <= ci) K[IDX2(ci, cj, n)] += d;
                if (k > 0) K[IDX2(ci, (k - 1) * nu + j, n)] += -2.0 * S->dR[i * nu + j];
            }
    if (chol(K, n)) goto done;
    for (int pass = 0; pass < POLISH_PASSES; ++pass) {
        int nA = 0;
        for (int r = 0; r < m; ++r)
            if (in[r]) {
                if (nA == amax) goto done;
                Ar[nA++] = r;
            }
        /* G_A rows and Y = L^-1 G_A' */
        for (int q = 0; q < nA; ++q) {
            const int r = Ar[q];
            double* g = GA + (size_t)q * n;
            memset(g, 0, sizeof(double) * n);
            if (r < ms) {
                const int k = r / mc;
                const double* c = a->C + (size_t)r * nx;
                const double* G = Gam + (size_t)(k + 1) * nx * n;
                for (int col = 0; col < (k + 1) * nu; ++col) {
                    double acc = 0.0;
                    for (int s = 0; s < nx; ++s) acc += c[s] * G[s * n + col];
                    g[col] = acc;
                }
            } else {
                const int qq = r - ms;
                g[qq / 2] = (qq & 1) ? -1.0 : 1.0;
            }
            double* y = Y + (size_t)q * n;
            for (int i = 0; i < n; ++i) {
                double acc = g[i];
                for (int p2 = 0; p2 < i; ++p2) acc -= K[IDX2(i, p2, n)] * y[p2];
                y[i] = acc / K[IDX2(i, i, n)];
            }
        }
        /* S = G_A H^-1 G_A' + E = Y'Y + E */
        for (int q = 0; q < nA; ++q)
            for (int q2 = 0; q2 <= q; ++q2) {
                double acc = 0.0;
                for (int i = 0; i < n; ++i) acc += Y[(size_t)q * n + i] * Y[(size_t)q2 * n + i];
                const int r = Ar[q], r2 = Ar[q2];
                if (r < ms && r2 < ms && r / mc == r2 / mc) {
                    const int j = S->row_slack[r % mc];
                    if (j >= 0 && S->row_slack[r2 % mc] == j)
                        acc += S->row_sign[r % mc] * S->row_sign[r2 % mc] / (2.0 * S->Qs[j]);
                }
                Ssch[IDX2(q, q2, nA)] = acc;
            }
        if (chol(Ssch, nA)) goto done;
        /* Newton steps on the KKT system from (U, sigma, lambda_A) */
        memcpy(Uc, U, sizeof(double) * n);
        memcpy(sc, sig, sizeof(double) * N * ns);
        for (int r = 0; r < m; ++r) lamp[r] = 0.0;
        for (int q = 0; q < nA; ++q) lA[q] = lam[Ar[q]];
        double mp = INFINITY, kk = INFINITY;
        for (int step = 0; step < POLISH_STEPS; ++step) {
            for (int q = 0; q < nA; ++q) lamp[Ar[q]] = lA[q];
            /* residuals with t = 0 (rp = row - w on A): rU = wk->rd, rsig = wk->rsig */
            for (int r = 0; r < m; ++r) wk->dt_a[r] = 0.0;
            double kk0;
            merit_at(S, a, wk, Uc, sc, wk->dt_a, lamp, X, &kk0);
            for (int q = 0; q < nA; ++q) {
                const int r = Ar[q];
                double ra = wk->rp[r];
                if (r < ms) {
                    const int j = S->row_slack[r % mc];
                    if (j >= 0) ra -= S->row_sign[r % mc] * wk->rsig[(r / mc) * ns + j] / (2.0 * S->Qs[j]);
                }
                rA[q] = ra;
            }
            memcpy(v, wk->rd, sizeof(double) * n);
            chol_solve(K, n, v); /* H^-1 rU */
            for (int q = 0; q < nA; ++q) {
                double acc = rA[q];
                for (int i = 0; i < n; ++i) acc -= GA[(size_t)q * n + i] * v[i];
                dl[q] = acc;
            }
            chol_solve(Ssch, nA, dl);
            for (int i = 0; i < n; ++i) gv[i] = wk->rd[i];
            for (int q = 0; q < nA; ++q)
                for (int i = 0; i < n; ++i) gv[i] += GA[(size_t)q * n + i] * dl[q];
            chol_solve(K, n, gv);
            for (int i = 0; i < n; ++i) Uc[i] -= gv[i];
            for (int k = 0; k < N; ++k)
                for (int j = 0; j < ns; ++j) {
                    double acc = wk->rsig[k * ns + j];
                    for (int q = 0; q < nA; ++q) {
                        const int r = Ar[q];
                        if (r < ms && r / mc == k && S->row_slack[r % mc] == j) acc += S->row_sign[r % mc] * dl[q];
                    }
                    sc[k * ns + j] -= acc / (2.0 * S->Qs[j]);
                }
            for (int q = 0; q < nA; ++q) lA[q] += dl[q];
            /* the polished point as an interior-point iterate: t = 0 and lambda = max(lambda_A, 0) on A,
               t = max(w - row, 0) and lambda = 0 elsewhere; one Newton step normally reaches tol, a
               refinement step follows only when it does not */
            fwd_sim(S, a, a->x0, Uc, X);
            for (int r = 0; r < m; ++r) {
                lamp[r] = 0.0;
                wk->dt_a[r] = (wk->act[r] && !in[r]) ? fmax(wk->w[r] - row_val(S, a, X, Uc, sc, r), 0.0) : 1.0;
            }
            for (int q = 0; q < nA; ++q) {
                lamp[Ar[q]] = fmax(lA[q], 0.0);
                wk->dt_a[Ar[q]] = 0.0;
            }
            mp = merit_at(S, a, wk, Uc, sc, wk->dt_a, lamp, X, &kk);
            if (mp < tol) break;
        }
#ifdef POLISH_DEBUG
        fprintf(stderr, "PD pass %d nA %d merit %.2e\n", pass, nA, mp);
#endif
        if (mp < best) {
            best = mp;
            *kkt = kk;
            memcpy(Up, Uc, sizeof(double) * n);
            memcpy(sigp, sc, sizeof(double) * N * ns);
        }
        /* the next pass's active set: violated rows join it, negative multipliers leave it */
        int changed = 0;
        for (int r = 0; r < m; ++r)
            if (wk->act[r] && !in[r] && wk->w[r] - row_val(S, a, X, Uc, sc, r) < 0.0) in[r] = 1, changed = 1;
        for (int q = 0; q < nA; ++q)
            if (lA[q] < 0.0) in[Ar[q]] = 0, changed = 1;
        if (!changed) break;
    }
done:
    free(in);
    free(Ar);
    free(GA);
    return best;
}

#ifdef RIC_F32
/* lab: the fp64 restart of an fp32-mode solve that ends short of tol (Cfg::F32 of mpc_riccati.hip):
   f32_no = 1 while it runs (no fp32 stage), at tol * 1e-3 so that its rounding floor is the requested
   tol; an end with the best merit below the requested tol (f32_req) counts as solved */
static _Thread_local int f32_no = 0;
static _Thread_local double f32_req = 0.0;
static _Thread_local int f32_dd = 0;   /* the last pass (mpc_launch rescue 3): double-double from the start */
long cmpc_f32_restarts = 0;
#endif
static int solve_one_base(const shared_t* S, const agent_t* a, double tol, int max_iter, work_t* wk,
                          double* z, double* kkt_out, int* iters_out);

/* Solve one agent.  Returns OSQP-style status: 1 solved, 2 solved inaccurate, -2 max_iter, -10 unsolved. */
static int solve_one(const shared_t* S, const agent_t* a, double tol, int max_iter, work_t* wk,
                     double* z, double* kkt_out, int* iters_out) {
    int st = solve_one_base(S, a, tol, max_iter, wk, z, kkt_out, iters_out);
#ifdef RIC_F32
    if (S->newton == 3 && st != 1) {
        const int it1 = *iters_out;
#pragma omp atomic
        cmpc_f32_restarts += 1;
        f32_no = 1;
        f32_req = tol;
        st = solve_one_base(S, a, tol * 1e-3, max_iter, wk, z, kkt_out, iters_out);
        *iters_out += it1;
        if (st != 1) {  /* ... and still short: the fp64 kernel's pass with double-double from the start */
            const int it2 = *iters_out;
            f32_dd = 1;
            st = solve_one_base(S, a, tol * 1e-3, max_iter, wk, z, kkt_out, iters_out);
            f32_dd = 0;
            *iters_out += it2;
        }
        f32_no = 0;
        f32_req = 0.0;
    }
#endif
    return st;
}

static int solve_one_base(const shared_t* S, const agent_t* a, double tol, int max_iter, work_t* wk,
                          double* z, double* kkt_out, int* iters_out) {
    /* newton 4: the product's CMPC_FLAG_RESCUE policy — the condensed method; at a factorisation
       breakdown the solve continues from that iterate with the Riccati double-double Newton solve
       (newton 3), its best-iterate bookkeeping restarted (the kernels hand the iterate from
       mpc_ipm3 / mpc_ipm to mpc_riccati through the rescue scratch) */
    shared_t S_cond, S_ric;
    /* 4: CMPC_FLAG_RESCUE | CMPC_FLAG_FINISH (every breakdown is continued); 5: CMPC_FLAG_RESCUE
       (a breakdown already at the rounding floor, best merit < 1e3 tol, stops there: status 2) */
    const int warm_rescue = S->newton == 4 || S->newton == 5, finish = S->newton == 4;
#ifdef LAB_STOPDUMP
    int it_switch = 0;
#endif
    if (warm_rescue) {
        S_cond = *S;
        S_cond.newton = 0;
        S_ric = *S;
        S_ric.newton = 3;
        S_ric.refine_dd = RIC_REFINE_WARM;
        S = &S_cond;
    }
    const int nx = S->nx, nu = S->nu, N = S->N, ns = S->ns, mc = S->mc;
    const int n = N * nu, ms = N * mc, m = ms + 2 * nu * N;
    double* Gam = wk->Gam; /* (N+1) x nx x n; also for the polish */
    const int need_gam = !NEWTON_C || S->polish;
    if (need_gam) memset(Gam, 0, sizeof(double) * (size_t)(N + 1) * nx * n);
    for (int k = 0; k < N && need_gam; ++k) {
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
    if (a->U0) memcpy(U, a->U0, sizeof(double) * n); else memset(U, 0, sizeof(double) * n);
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

#ifdef SIGMA_START
    /* slack-consistent start: sigma_j = the projection of 0 onto the interval the group's rows
       allow at X (most relaxed feasible slack); the binding row carries lambda = |2 Qs sigma|,
       the slack stationarity 2 Qs sigma + sum sign lambda = 0 */
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < ns; ++j) {
            double lo = -INFINITY, hi = INFINITY;
            for (int r = 0; r < mc; ++r) {
                if (S->row_slack[r] != j || !wk->act[k * mc + r]) continue;
                double g; ROWVAL(X, U, (const double*)NULL, k * mc + r, g);
                const double e = wk->w[k * mc + r] - g; /* sign sigma <= e */
                if (S->row_sign[r] > 0) hi = fmin(hi, e); else lo = fmax(lo, -e);
            }
            double s = 0.0;
            if (hi < 0.0) s = hi; else if (lo > 0.0) s = lo;
            sig[k * ns + j] = SIGMA_START * s;
        }
#endif
    for (int r = 0; r < m; ++r) {
        if (!wk->act[r]) { t[r] = 1.0; lam[r] = 0.0; continue; }
        double g; ROWVAL(X, U, sig, r, g);
        double s0 = wk->w[r] - g;
        const double fl = S->newton ? T0_FLOOR : T0_FLOOR_COND; /* kT0Floor / kT0FloorCond (internal.h) */
        t[r] = s0 > fl ? s0 : fl;
#ifdef LAM0_CENTRE
        lam[r] = LAM0_CENTRE / t[r]; /* lab: centred start, t lambda equal on every row */
#else
        lam[r] = 1.0;
#endif
#ifdef SIGMA_START
        if (r < ms) {
            const int j = S->row_slack[r % mc];
            if (j >= 0) {
                const double sg = sig[(r / mc) * ns + j];
                if (S->row_sign[r % mc] * sg < 0.0 && s0 < 1e-12 + fabs(sg) * 1e-9) lam[r] = fmax(1.0, LAMF * 2.0 * S->Qs[j] * fabs(sg));
            }
        }
#endif
    }
    double scale_p = 1.0;
    for (int r = 0; r < m; ++r) if (wk->act[r] && fabs(wk->w[r]) > scale_p) scale_p = fabs(wk->w[r]);
    double qs_max = 1.0;
    for (int j = 0; j < ns; ++j) if (2 * S->Qs[j] > qs_max) qs_max = 2 * S->Qs[j];

    /* best iterate by merit max(res, 1e4 mu) (< tol <=> converged): returned when the
       method stops short of convergence (max_iter, factorisation breakdown, stagnation) */
    double best_m = INFINITY, best_kkt = INFINITY;
    int best_it = 0, stop = 0, pol_done = 0; /* stop: 0 max_iter, 1 converged, 2 breakdown, 3 stagnation, 4 non-finite */
    double *bU = wk->bU, *bsig = wk->bsig;
    int it;
    double kkt = INFINITY;
    double alpha_prev = 1.0; /* step of the previous iteration (kShortStep rule) */
#ifdef RIC_F32
    int f32_on = !f32_no;    /* lab: this agent still factors in fp32 */
#endif
#ifndef DD_STALL
#define DD_STALL 2           /* kDdStall of mpc_riccati.hip */
#endif
    int dd_on = 0;           /* newton 3: this solve has switched to double-double near the solution */
    int kkt_stop = 0;        /* lab RIC_F32 last pass: stopped at kkt < the requested tol */
#ifdef RIC_F32
    dd_on = f32_dd;
#endif
#ifdef LAB_SIGMA2
    /* lab: a second corrector with another centring parameter per iteration (a second wavefront's
       work in a two-wave kernel); the longer step wins, ties to the first */
    double* s2_save = malloc(sizeof(double) * ((size_t)n + (size_t)(N + 1) * nx + (size_t)N * ns + 2 * (size_t)m));
#endif
#ifdef GONDZIO
    /* lab: Gondzio centrality correctors (up to GONDZIO per iteration) on the Mehrotra direction */
    long gz_used = 0;
    double* gz_corr = calloc((size_t)m, sizeof(double));
    double* gz_save = malloc(sizeof(double) * ((size_t)n + (size_t)(N + 1) * nx + (size_t)N * ns + 2 * (size_t)m));
#ifndef GZ_DA
#define GZ_DA 0.2
#endif
#ifndef GZ_TRIG
#define GZ_TRIG 0.9
#endif
#endif
    for (it = 1; it <= max_iter; ++it) {
#ifdef POLISH_AT
        /* lab: one polish attempt from the iterate of iteration POLISH_AT (the condensed method) */
        if (!S->newton && it == POLISH_AT + 1) {  /* before this iteration's residuals */
            double pk;
            const double pm = polish_one(S, a, wk, tol, U, sig, t, lam, wk->dU, wk->dsig, &pk);
#pragma omp atomic
            lab_pol_tried += 1;
            if (pm < tol) {
#pragma omp atomic
                lab_pol_ok += 1;
                memcpy(U, wk->dU, sizeof(double) * n);
                memcpy(sig, wk->dsig, sizeof(double) * N * ns);
                kkt = pk;
                stop = 1;
                break;
            }
        }
#endif
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
        const double merit = nmax(res, MU_FACTOR * mu);
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
#ifdef LAB_DEGEN
        if (merit < tol) {
            double v1 = 0, v2 = 0, v3 = 0; int r1 = -1;
            for (int r = 0; r < m; ++r) if (wk->act[r]) { double v = fmin(t[r], lam[r]); if (v > v1) { v3 = v2; v2 = v1; v1 = v; r1 = r; } else if (v > v2) { v3 = v2; v2 = v; } else if (v > v3) v3 = v; }
            fprintf(stderr, "DEGEN it %d mu %.2e top min(t,lam) %.2e (row %d t %.2e lam %.2e) %.2e %.2e\n", it, mu, v1, r1, r1 >= 0 ? t[r1] : 0., r1 >= 0 ? lam[r1] : 0., v2, v3);
        }
#endif
        if (merit < tol) { stop = 1; break; }
#ifdef RIC_F32
        if (f32_dd && kkt < f32_req) { stop = 1; kkt_stop = 1; break; }  /* the last pass: at the KKT bar */
#endif
        /* near-converged but no progress for STALL_ITERS iterations: rounding floor reached */
        if (best_m < 1e3 * tol && it - best_it >= STALL_ITERS) {
            stop = 3;
            break;
        }
        /* continued (rescue) solve: no new best iterate for WARM_STALL iterations ends it
           (kWarmStall of the kernels) */
        if (warm_rescue && S->newton && it - best_it >= WARM_STALL) {
            stop = 3;
            break;
        }

        /* ---- Newton matrix ---- */
        int hp = 0; /* Riccati: this iteration factors in double-double (newton == 3) */
        for (int r = 0; r < m; ++r) wk->th[r] = wk->act[r] ? lam[r] / t[r] : 0.0;
#ifdef RIC_F32
        if (f32_dd)  /* the last pass: th capped (kThCapLast of mpc_riccati.hip) */
            for (int r = 0; r < m; ++r) wk->th[r] = fmin(wk->th[r], 1e17);
#endif
#ifdef THMAX
        for (int r = 0; r < m; ++r) wk->th[r] = fmin(wk->th[r], THMAX);
#endif
        for (int k = 0; k < N; ++k)
            for (int j = 0; j < ns; ++j) {
                double v = 2.0 * S->Qs[j];
                for (int r = 0; r < mc; ++r) if (S->row_slack[r] == j) v += wk->th[k * mc + r];
                wk->Dsig[k * ns + j] = v;
            }
        double* K = wk->K;
        double* W = wk->W;
        if (S->newton) {
                        hp = 0;
            double thm_last = 0.0;
            if (S->newton == 3) {
                double thm = 0.0;
                for (int r = 0; r < m; ++r) if (wk->act[r] && wk->th[r] > thm) thm = wk->th[r];
                thm_last = thm;
                /* double-double only once the fp64 recursion stops making progress (no new best iterate
                   for DD_STALL iterations) or breaks down while max th > RIC_DD_TH — not at every such
                   iteration (kDdStall of mpc_riccati.hip): on 2048 cfg5 agents 3136 -> 181 dd iterations,
                   the same statuses to 2 agents and z to 5e-8; a continued (rescue) solve keeps it on */
                if (!dd_on && it - best_it >= DD_STALL) dd_on = 1;
                hp = thm > RIC_DD_TH && dd_on;
#ifdef DD_PROACTIVE
                hp = thm > RIC_DD_TH;   /* lab: the round-2 rule */
#endif
#ifdef DD_COUNT
                if (hp) {
#pragma omp atomic
                    cmpc_dd_iters += 1;
                }
#endif
            }
#ifdef RIC_QUAD
            if (ric_factor_q(S, a, wk->th, wk->Dsig, wk->F)) { stop = 2; break; }
#else
#ifdef RIC_F32
            if (f32_on && (it - best_it >= F32_STALL || best_m < F32_SWITCH_M)) {
                f32_on = 0;
#pragma omp atomic
                cmpc_f64_agents += 1;
            }
            if (f32_on) {
                if (ric_factor_f32(S, a, wk->th, wk->Dsig, wk->F)) {
                    f32_on = 0;
#pragma omp atomic
                    cmpc_f64_agents += 1;
                }
            }
            {
                const int was = f32_on;
#pragma omp atomic
                cmpc_f32_iters += f32_on;
#pragma omp atomic
                cmpc_f64_iters += !f32_on;
                (void)was;
            }
            if (!f32_on)
#endif
            if (!hp && S->newton == 3 && thm_last > RIC_DD_TH && ric_factor(S, a, wk->th, wk->Dsig, wk->F)) {
                dd_on = 1;   /* fp64 breakdown above the threshold: this iteration and the rest in double-double */
                hp = 1;
#ifdef DD_COUNT
#pragma omp atomic
                cmpc_dd_iters += 1;
#endif
                if (ric_factor_dd(S, a, wk->th, wk->Dsig, wk->F)) { stop = 2; break; }
            } else if (hp || S->newton != 3 || !(thm_last > RIC_DD_TH))
            if (hp ? ric_factor_dd(S, a, wk->th, wk->Dsig, wk->F) : ric_factor(S, a, wk->th, wk->Dsig, wk->F)) { stop = 2; break; }
#endif
        }
#ifdef LOWRANK
        /* lab: slack-free state rows whose weight exceeds LOWRANK leave the normal matrix (M) and
           return as a rank-|L| correction (Sherman-Morrison-Woodbury on the augmented system):
           K = M + G_L' Th_L G_L,  K^-1 r = M^-1 r - Y S^-1 G_L M^-1 r,  Y = M^-1 G_L',
           S = Th_L^-1 + G_L Y.  A dense row with theta ~ 1e20 no longer swamps M. */
        int nL = 0, Lr[LR_MAX];
        double Lth[LR_MAX];
        for (int r = 0; r < ms && !S->newton; ++r) {
            if (!wk->act[r] || S->row_slack[r % mc] >= 0 || !(wk->th[r] > LOWRANK)) continue;
            int pos = nL < LR_MAX ? nL++ : -1;
            if (pos < 0) { /* keep the LR_MAX largest */
                int mn = 0;
                for (int l = 1; l < LR_MAX; ++l) if (Lth[l] < Lth[mn]) mn = l;
                if (wk->th[r] <= Lth[mn]) continue;
                wk->th[Lr[mn]] = Lth[mn];
                pos = mn;
            }
            Lr[pos] = r;
            Lth[pos] = wk->th[r];
            wk->th[r] = 0.0;
        }
#endif
        if (!NEWTON_C) memset(K, 0, sizeof(double) * n * n);
        for (int k = 0; k < N && !NEWTON_C; ++k) {
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
        for (int k = 0; k < N && !NEWTON_C; ++k)
            for (int i = 0; i < nu; ++i)
                for (int j = 0; j < nu; ++j) {
                    int ci = k * nu + i, cj = k * nu + j;
                    double v = 2.0 * S->R[i * nu + j] + 2.0 * S->dR[i * nu + j] * (k + 1 < N ? 2.0 : 1.0);
                    if (cj <= ci) K[IDX2(ci, cj, n)] += v;
                    if (k > 0 && 1) K[IDX2(ci, (k - 1) * nu + j, n)] += -2.0 * S->dR[i * nu + j];
                }
        for (int k = 0; k < N && !NEWTON_C; ++k)
            for (int i = 0; i < nu; ++i) {
                int r = ms + (k * nu + i) * 2;
                K[IDX2(k * nu + i, k * nu + i, n)] += wk->th[r] + wk->th[r + 1];
            }
#ifdef RIC_DEBUG
        const int chol_bad = chol(K, n);
        if (!S->newton && chol_bad) { stop = 2; break; }
#else
        if (!S->newton && chol(K, n)) {
#ifdef LAB_THDUMP
            /* lab: the rows whose weight broke the factorisation */
            fprintf(stderr, "breakdown it %d:", it);
            for (int r = 0; r < m; ++r)
                if (wk->act[r] && wk->th[r] > LAB_THDUMP)
                    fprintf(stderr, " r%d(k%d,%s%d th%.1e)", r, r < ms ? r / mc : (r - ms) / (2 * nu), r < ms ? "row" : "in",
                            r < ms ? r % mc : (r - ms) % (2 * nu), wk->th[r]);
            fprintf(stderr, "\n");
#endif
            if (warm_rescue && !S->newton && (finish || !(best_m < 1e3 * tol))) {
                if (S->polish) { /* polish the breakdown iterate first; hand over only if that misses tol */
                    double pk;
                    const double pm = polish_one(S, a, wk, tol, U, sig, t, lam, wk->dU, wk->dsig, &pk);
                    if (pm < tol) {
                        memcpy(U, wk->dU, sizeof(double) * n);
                        memcpy(sig, wk->dsig, sizeof(double) * N * ns);
                        kkt = pk;
                        stop = 1;
                        pol_done = 1;
                        break;
                    }
                }
#ifdef LAB_STOPDUMP
                it_switch = it;
#endif
                /* hand over: redo this iteration (its residuals are those of the same iterate) with
                   the Riccati solve; the best iterate is tracked afresh, as the rescue kernel does */
                S = &S_ric;
                dd_on = 1;   /* a continued solve factors in double-double whenever max th > RIC_DD_TH */
                best_m = INFINITY;
                best_kkt = INFINITY;
                best_it = 0;
                --it;
                continue;
            }
            stop = 2;
            break;
        }
#endif
#ifdef LOWRANK
        double *LG = NULL, *LY = NULL, LS[LR_MAX * LR_MAX];
        if (nL) {
            for (int l = 0; l < nL; ++l) wk->th[Lr[l]] = Lth[l];
            LG = malloc(sizeof(double) * 2 * (size_t)nL * n);
            LY = LG + (size_t)nL * n;
            for (int l = 0; l < nL; ++l) {
                const int k = Lr[l] / mc;
                const double* c_ = a->C + (size_t)Lr[l] * nx;
                const double* G = Gam + (size_t)(k + 1) * nx * n;
                for (int c = 0; c < n; ++c) {
                    double v = 0.0;
                    for (int s = 0; s < nx; ++s) v += c_[s] * G[s * n + c];
                    LG[(size_t)l * n + c] = v;
                }
                memcpy(LY + (size_t)l * n, LG + (size_t)l * n, sizeof(double) * n);
                chol_solve(K, n, LY + (size_t)l * n);
            }
            for (int l = 0; l < nL; ++l)
                for (int l2 = 0; l2 < nL; ++l2) {
                    double v = l == l2 ? 1.0 / Lth[l] : 0.0;
                    for (int c = 0; c < n; ++c) v += LG[(size_t)l * n + c] * LY[(size_t)l2 * n + c];
                    LS[l * nL + l2] = v;
                }
            if (chol(LS, nL)) { free(LG); stop = 2; break; }
        }
#endif

        /* ---- predictor / corrector ---- */
        double sig_c = 0.0, mu_aff = 0.0;
#ifdef LAB_SIGMA2
        int s2_stage = 0; double s2_al = 0.0, s2_sig1 = 0.0;
#endif
#ifdef RETRY_SIGMA
        int retried = 0;
#endif
#ifdef GONDZIO
        int gz_n = 0; double gz_al = 0.0;
        memset(gz_corr, 0, sizeof(double) * m);
#endif
        for (int pass = 0; pass < 2; ++pass) {
            for (int r = 0; r < m; ++r) {
                if (!wk->act[r]) { wk->rho[r] = 0.0; continue; }
                double rc = -t[r] * lam[r];
                if (pass) rc += sig_c * mu - wk->dt_a[r] * wk->dl_a[r];
#ifdef GONDZIO
                if (pass) rc += gz_corr[r];
#endif
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
#ifdef LOWRANK
            /* the separated rows' rho enters through the small system (bounded: rho/theta = rc/lam + rp) */
            for (int l = 0; l < nL; ++l) wk->rt[Lr[l]] = 0.0;
#endif
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
            if (S->newton) {
#ifdef RIC_F32
                if (f32_on) ric_solve_f32(S, a, wk->F, wk->rhs, wk->dU, wk->dX); else
#endif
                ric_solve(S, a, wk->F, wk->rhs, wk->dU, wk->dX);
                /* iterative refinement: dU += M^-1 (rhs - K dU) */
                const int nref = hp ? S->refine_dd : S->refine;
                for (int ir = 0; ir < nref; ++ir) {
#ifdef REF_COUNT
                    if (hp) fprintf(stderr, "REF\n");
#endif
                    double *kv = wk->Yk, *cr = wk->Yk + n, *cx = wk->Yk + 2 * n;
#ifdef KMUL_QUAD
                    kres_q(S, a, wk->th, wk->Dsig, wk->dU, wk->rhs, kv);
#else
                    if (hp) {
                        kres_dd(S, a, wk->th, wk->Dsig, wk->dU, wk->rhs, kv, wk->Xdd);
                    } else {
                        kmul(S, a, wk->th, wk->Dsig, wk->dU, kv, cx, ybar, wk->psi, wk->tmp);
                        for (int c = 0; c < n; ++c) kv[c] = wk->rhs[c] - kv[c];
                    }
#endif
#ifdef RIC_F32
                    if (f32_on) ric_solve_f32(S, a, wk->F, kv, cr, cx); else
#endif
                    ric_solve(S, a, wk->F, kv, cr, cx);
                    double cn = 0.0, un = 0.0;
                    for (int c = 0; c < n; ++c) {
                        wk->dU[c] += cr[c];
                        cn = fmax(cn, fabs(cr[c]));
                        un = fmax(un, fabs(wk->dU[c]));
                    }
                    if (cn <= REF_TOL * un) break;
                }
                if (nref) fwd_sim(S, a, NULL, wk->dU, wk->dX);
#ifdef RIC_DEBUG
                {
                    double* cu = wk->Yk;
                    memcpy(cu, wk->rhs, sizeof(double) * n);
                    double de = 0, dn = 0, thm = 0;
                    if (!chol_bad) {
                        chol_solve(K, n, cu);
                        for (int c = 0; c < n; ++c) { de = fmax(de, fabs(cu[c] - wk->dU[c])); dn = fmax(dn, fabs(cu[c])); }
                    }
                    for (int r = 0; r < m; ++r) if (wk->act[r]) thm = fmax(thm, wk->th[r]);
#ifdef RIC_QREF
                    if (it >= 46) {
                        double* qu = malloc(sizeof(double) * n);
                        condensed_q(S, a, wk->th, wk->Dsig, wk->rhs, qu);
#ifdef USE_QUAD_DIR
                        memcpy(wk->dU, qu, sizeof(double) * n);
                        fwd_sim(S, a, NULL, wk->dU, wk->dX);
#endif
                        double eq = 0, ec = 0, nq = 0;
                        for (int c = 0; c < n; ++c) { nq = fmax(nq, fabs(qu[c])); eq = fmax(eq, fabs(qu[c] - wk->dU[c])); if (!chol_bad) ec = fmax(ec, fabs(qu[c] - cu[c])); }
                        fprintf(stderr, "it %d pass %d vs quad: riccati %.2e condensed %.2e\n", it, pass, eq / nq, ec / nq);
                        free(qu);
                    }
#endif
                    fprintf(stderr, "it %d pass %d |dU_ric - dU_chol|/|dU| %.2e (chol %s) thmax %.1e\n", it, pass, de / dn, chol_bad ? "FAILED" : "ok", thm);
                    if (pass == 0) for (int r = 0; r < m; ++r) if (wk->act[r] && wk->th[r] > 1e10) fprintf(stderr, "   row %d (k %d rr %d) th %.1e t %.1e lam %.1e\n", r, r < ms ? r / mc : (r - ms) / (2 * nu), r < ms ? r % mc : (r - ms) % (2 * nu), wk->th[r], t[r], lam[r]);
                }
#endif
            } else {
                memcpy(wk->dU, wk->rhs, sizeof(double) * n);
                chol_solve(K, n, wk->dU);
#ifdef LOWRANK
                if (nL) {
                    double v[LR_MAX];
                    for (int l = 0; l < nL; ++l) {
                        double s = 0.0;
                        for (int c = 0; c < n; ++c) s += LG[(size_t)l * n + c] * wk->dU[c];
                        v[l] = s + wk->rho[Lr[l]] / Lth[l];
                    }
                    chol_solve(LS, nL, v);
                    for (int l = 0; l < nL; ++l)
                        for (int c = 0; c < n; ++c) wk->dU[c] -= LY[(size_t)l * n + c] * v[l];
                }
#endif
#ifdef DIRCHECK
                {   /* lab: relative Newton residual |rhs - K dU| / |rhs| of the direction, in double-double */
                    double* kv = wk->Yk;
#ifdef LOWRANK
                    for (int l = 0; l < nL; ++l)
                        for (int c = 0; c < n; ++c) wk->rhs[c] -= wk->rho[Lr[l]] * LG[(size_t)l * n + c];
#endif
                    kres_dd(S, a, wk->th, wk->Dsig, wk->dU, wk->rhs, kv, wk->Xdd);
                    double rn = 0.0, bn = 0.0, thm = 0.0;
                    for (int c = 0; c < n; ++c) { rn = fmax(rn, fabs(kv[c])); bn = fmax(bn, fabs(wk->rhs[c])); }
                    for (int r = 0; r < m; ++r) if (wk->act[r] && wk->th[r] > thm) thm = wk->th[r];
                    fprintf(stderr, "   it %d pass %d newton residual %.2e (|rhs| %.2e) thmax %.1e\n", it, pass, rn / bn, bn, thm);
                }
#endif
#ifdef CREFINE
                /* lab: iterative refinement of the condensed direction against the Newton residual
                   evaluated in double-double (the fp64 Cholesky as the preconditioner) */
                {
                    double thm = 0.0;
                    for (int r = 0; r < m; ++r) if (wk->act[r] && wk->th[r] > thm) thm = wk->th[r];
                    for (int ir = 0; ir < CREFINE && thm > CREF_TH; ++ir) {
                        double* kv = wk->Yk;
                        kres_dd(S, a, wk->th, wk->Dsig, wk->dU, wk->rhs, kv, wk->Xdd);
                        chol_solve(K, n, kv);
                        double cn = 0.0, un = 0.0;
                        for (int c = 0; c < n; ++c) {
                            wk->dU[c] += kv[c];
                            cn = fmax(cn, fabs(kv[c]));
                            un = fmax(un, fabs(wk->dU[c]));
                        }
                        if (cn <= REF_TOL * un) break;
                    }
                }
#endif
                fwd_sim(S, a, NULL, wk->dU, wk->dX);
            }
#ifdef ORACLE_TRACE
            for (int k = 0; k < N; ++k)
                if (k < 2 || k == N - 1)
                    fprintf(stderr, "  pass %d k %d du %.10e %.10e %.10e\n", pass, k, wk->dU[k * nu], wk->dU[k * nu + 1 % nu],
                            wk->dU[k * nu + 2 % nu]);
#endif
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
#ifdef SIGMA_EXP
                sig_c = mu > 0 ? pow(mu_aff / mu, SIGMA_EXP) : 0.0;
#else
                /* e = 3 for the stage-wise methods, 2 for the condensed one and its warm Riccati continuation
                   (internal.h) */
                sig_c = mu > 0 ? pow(mu_aff / mu, (S->newton && !warm_rescue) ? 3.0 : 2.0) : 0.0;
#endif
                if (alpha_prev < SHORT_STEP) sig_c = fmax(sig_c, SIGMA_MIN); /* kShortStep / kSigmaMin */
            } else {
#ifdef GONDZIO
                {
                    const size_t nX = (size_t)(N + 1) * nx, nS = (size_t)N * ns;
                    double* sv = gz_save;
                    if (gz_n > 0 && al < gz_al + 0.1 * GZ_DA) {
                        /* the correction did not lengthen the step enough: back to the saved direction */
                        memcpy(wk->dU, sv, sizeof(double) * n); sv += n;
                        memcpy(wk->dX, sv, sizeof(double) * nX); sv += nX;
                        memcpy(wk->dsig, sv, sizeof(double) * nS); sv += nS;
                        memcpy(dt, sv, sizeof(double) * m); sv += m;
                        memcpy(dl, sv, sizeof(double) * m);
                        al = gz_al;
                    } else if (gz_n < GONDZIO && al < GZ_TRIG) {
                        memcpy(sv, wk->dU, sizeof(double) * n); sv += n;
                        memcpy(sv, wk->dX, sizeof(double) * nX); sv += nX;
                        memcpy(sv, wk->dsig, sizeof(double) * nS); sv += nS;
                        memcpy(sv, dt, sizeof(double) * m); sv += m;
                        memcpy(sv, dl, sizeof(double) * m);
                        const double at = fmin(1.0, al + GZ_DA), mt = sig_c * mu;
                        for (int r = 0; r < m; ++r) {
                            if (!wk->act[r]) continue;
                            const double v = (t[r] + at * dt[r]) * (lam[r] + at * dl[r]);
                            double c = 0.0;
                            if (v < 0.1 * mt) c = 0.1 * mt - v;
                            else if (v > 10.0 * mt) c = fmax(10.0 * mt - v, -10.0 * mt);
                            gz_corr[r] += c;
                        }
                        gz_al = al;
                        ++gz_n;
                        ++gz_used;
                        pass = 0;
                        continue;
                    }
                }
#endif
#ifdef ETA_ADAPT
                al = fmax(0.995, 1.0 - ETA_ADAPT * mu) * al;
#elif defined(ETA_END)
                al = (merit < ETA_END ? ETA_FRAC : 0.995) * al; /* lab: longer steps near convergence */
#else
                al = 0.995 * al;
#endif
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
#ifdef LAB_SIGMA2
                {
                    const size_t nX = (size_t)(N + 1) * nx, nS = (size_t)N * ns;
                    if (s2_stage == 0) {
                        double* sv = s2_save;
                        memcpy(sv, wk->dU, sizeof(double) * n); sv += n;
                        memcpy(sv, wk->dX, sizeof(double) * nX); sv += nX;
                        memcpy(sv, wk->dsig, sizeof(double) * nS); sv += nS;
                        memcpy(sv, dt, sizeof(double) * m); sv += m;
                        memcpy(sv, dl, sizeof(double) * m);
                        s2_al = al;
                        s2_sig1 = sig_c;
                        s2_stage = 1;
                        sig_c = LAB_SIGMA2_RULE(sig_c);
                        pass = 0;
                        continue;
                    }
                    if (!(al > s2_al * LAB_SIGMA2_MARGIN)) { /* the first corrector's step */
                        double* sv = s2_save;
                        memcpy(wk->dU, sv, sizeof(double) * n); sv += n;
                        memcpy(wk->dX, sv, sizeof(double) * nX); sv += nX;
                        memcpy(wk->dsig, sv, sizeof(double) * nS); sv += nS;
                        memcpy(dt, sv, sizeof(double) * m); sv += m;
                        memcpy(dl, sv, sizeof(double) * m);
                        al = s2_al;
                        sig_c = s2_sig1;
                    }
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
                alpha_prev = al;
                for (int c = 0; c < n; ++c) U[c] += al * wk->dU[c];
                for (int q = 0; q < N * ns; ++q) sig[q] += al * wk->dsig[q];
                for (int r = 0; r < m; ++r)
                    if (wk->act[r]) { t[r] += al * dt[r]; lam[r] += al * dl[r]; }
                for (int q = 0; q < (N + 1) * nx; ++q) X[q] += al * wk->dX[q];
            }
        }
#ifdef LOWRANK
        free(LG);
#endif
    }
#ifdef GONDZIO
#pragma omp atomic
    cmpc_gz_solves += gz_used;
    free(gz_corr);
    free(gz_save);
#endif
    if (it > max_iter) it = max_iter;
#ifdef LAB_STOPDUMP
    if (it_switch) fprintf(stderr, "WARM switch %d after %d stop %d best_m %.2e\n", it_switch, it - it_switch, stop, best_m);
#endif
    /* polish (CMPC_FLAG_POLISH): the last solve of the rescue policy that an agent gets, when it stops
       short of tol — a condensed or continued solve at the rounding floor or at max_iter (status 2 /
       -2; an unsolved one goes on to the cold Riccati pass), the cold pass whatever its end — from its
       last iterate (the kernels' rescue image, flag 2) */
    double pol_m = INFINITY, pol_kkt = INFINITY;
    const int final_solve = !warm_rescue || best_m < 1e3 * tol || stop == 0;
    /* ... and a condensed solve that converged with a weakly active row (kPolishDegenerate, internal.h:
       t_r and lambda_r both ~sqrt(mu); the endpoint is then fixed only to ~3e-7 along that row) */
    int degen = 0;
    if (S->polish && stop == 1 && !S->newton && !pol_done) {
        double dg = 0.0;
        for (int r = 0; r < m; ++r)
            if (wk->act[r]) dg = fmax(dg, fmin(t[r], lam[r]));
        degen = dg > POLISH_DEGENERATE;
    }
    if (S->polish && ((stop != 1 && stop != 4 && final_solve) || degen))
        pol_m = polish_one(S, a, wk, tol, U, sig, t, lam, wk->dU, wk->dsig, &pol_kkt);
#ifdef LAB_DEGEN_COUNT
    if (degen) {
#pragma omp atomic
        cmpc_degen_flagged += 1;
        if (pol_m < best_m) {
#pragma omp atomic
            cmpc_degen_taken += 1;
        }
    }
#endif
#ifdef POLISH_DEBUG
    if (stop != 1) fprintf(stderr, "POL stop %d newton %d best_m %.2e pol_m %.2e\n", stop, S->newton, best_m, pol_m);
#endif
    int status;
    if (stop == 1 && !(degen && pol_m < best_m)) {
        status = kkt_stop ? 2 : 1;
    } else if (pol_m < best_m && pol_m < 1e3 * tol) { /* (mpc_polish.hip: never promotes past the floor) */
        memcpy(U, wk->dU, sizeof(double) * n);
        memcpy(sig, wk->dsig, sizeof(double) * N * ns);
        kkt = pol_kkt;
        status = pol_m < tol ? 1 : 2;
    } else {
        if (best_it > 0) { /* restore the best iterate */
            memcpy(U, bU, sizeof(double) * n);
            memcpy(sig, bsig, sizeof(double) * N * ns);
            kkt = best_kkt;
        }
        status = best_m < 1e3 * tol ? 2 : (stop == 0 ? -2 : -10);
#ifdef RIC_F32
        if (f32_no) status = best_m < f32_req ? 1 : (best_m < 1e3 * f32_req ? 2 : status);
#endif
#ifdef LAB_STOPDUMP
        fprintf(stderr, "STOP status %d stop %d newton %d it %d best_it %d best_m %.2e\n", status, stop, S->newton, it,
                best_it, best_m);
#endif
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

/* newton: 0 condensed Cholesky (default), 1 Riccati, 2 Riccati in Joseph form */
int cmpc_oracle_solve_ex(int nx, int nu, int N, int ns, int mc, int batch,
                         const double* Q, const double* R, const double* dR, const double* Qs,
                         const double* u_ub, const double* u_lb, const int* row_slack, const int* row_sign,
                         const double* A, const double* Bm, const double* x0, const double* u_prev,
                         const double* qlin, const double* Crow, const double* hrow,
                         double tol, int max_iter, int nthreads, int newton, int refine, const double* U0,
                         double* z, double* kkt, int* iters, int* status) {
    const int polish = (newton >> 8) & 1; /* newton | 0x100: CMPC_FLAG_POLISH */
    const int polish_amax = (newton >> 16) & 0xff; /* newton | amax << 16: the kernel's active-set capacity */
    newton &= 0xff;
    shared_t S = {nx, nu, N, ns, mc, Q, R, dR, Qs, u_ub, u_lb, row_slack, row_sign, newton, refine, RIC_REFINE_MAX,
                  polish, polish_amax};
    if (newton && (nx + nu > NA_MAX || nu > NU_MAX)) return -1;
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
        work_t wk = {0};
        const size_t nF = (size_t)N * (nu * (nx + nu) + nu * nu);
#ifdef RIC_DEBUG
        const size_t nG = (size_t)(N + 1) * nx * n, nK = (size_t)n * n;
#else
        const int cond = newton == 0 || newton == 4 || newton == 5 || polish; /* condensed Newton matrix (or H) */
        const size_t nG = cond ? (size_t)(N + 1) * nx * n : 0, nK = cond ? (size_t)n * n : 0;
#endif
        size_t need = nF + (size_t)n + (size_t)N * ns + nG + nK + 4 * (size_t)(N + 1) * nx + 4 * (size_t)n +
                      4 * (size_t)N * ns + 12 * (size_t)m + 2 * (size_t)nx + (size_t)nx * nx + (size_t)n * 3 + (size_t)nx * n + 2 * (size_t)n + (size_t)(N + 1) * nx;
        double* buf = (double*)calloc(need, sizeof(double));
        unsigned char* act = (unsigned char*)calloc(m, 1);
        if (!buf || !act) {
#pragma omp atomic write
            err = 1;
        } else {
            double* p = buf;
#define TAKE(f, cnt) do { wk.f = p; p += (cnt); } while (0)
            TAKE(bU, n); TAKE(bsig, N * ns);
            TAKE(Gam, nG); TAKE(K, nK); TAKE(F, nF);
            TAKE(X, (N + 1) * nx); TAKE(dX, (N + 1) * nx); TAKE(ybar, (N + 1) * nx); TAKE(W, nx * nx);
            TAKE(U, n); TAKE(dU, n); TAKE(gU, n); TAKE(rd, n); TAKE(rhs, n);
            TAKE(sig, N * ns); TAKE(dsig, N * ns); TAKE(Dsig, N * ns); TAKE(rsig, N * ns);
            TAKE(t, m); TAKE(lam, m); TAKE(th, m); TAKE(rho, m); TAKE(rt, m); TAKE(rp, m); TAKE(w, m);
            TAKE(dt_a, m); TAKE(dl_a, m); TAKE(dtv, m); TAKE(dlv, m); TAKE(GdU, m);
            TAKE(psi, nx); TAKE(tmp, nx); TAKE(Yk, (size_t)nx * n + 2 * (size_t)n + (size_t)(N + 1) * nx);
#undef TAKE
            wk.act = act;
            wk.Xdd = (dd_t*)malloc(sizeof(dd_t) * (size_t)(N + 1) * nx);
#pragma omp for schedule(dynamic, 4)
            for (int b = 0; b < batch; ++b) {
                agent_t ag = {A + (size_t)b * N * nx * nx, Bm + (size_t)b * N * nx * nu, x0 + (size_t)b * nx,
                              u_prev + (size_t)b * nu, qlin + (size_t)b * (N + 1) * nx,
                              Crow + (size_t)b * N * mc * nx, hrow + (size_t)b * N * mc, U0 ? U0 + (size_t)b * n : NULL};
                status[b] = solve_one(&S, &ag, tol, max_iter, &wk, z + b * nz, kkt + b, iters + b);
            }
        }
        if (buf && act) free(wk.Xdd);
        free(buf);
        free(act);
    }
    return err ? -1 : 0;
}

int cmpc_oracle_solve(int nx, int nu, int N, int ns, int mc, int batch,
                      const double* Q, const double* R, const double* dR, const double* Qs,
                      const double* u_ub, const double* u_lb, const int* row_slack, const int* row_sign,
                      const double* A, const double* Bm, const double* x0, const double* u_prev,
                      const double* qlin, const double* Crow, const double* hrow,
                      double tol, int max_iter, int nthreads,
                      double* z, double* kkt, int* iters, int* status) {
    return cmpc_oracle_solve_ex(nx, nu, N, ns, mc, batch, Q, R, dR, Qs, u_ub, u_lb, row_slack, row_sign, A, Bm, x0,
                                u_prev, qlin, Crow, hrow, tol, max_iter, nthreads, 0, 0, NULL, z, kkt, iters, status);
}
