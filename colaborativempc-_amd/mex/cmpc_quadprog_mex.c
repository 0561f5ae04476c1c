/* cmpc_quadprog — MATLAB MEX gateway over libcmpc's batched dense QP (cmpc_solve_qp_batch).
 *
 *   [x, fval, exitflag, output, lambda] = cmpc_quadprog(H, f, A, b, Aeq, beq, lb, ub [, x0, opts])
 *
 * Drop-in for the quadprog call YALMIP makes in
 * Matlab-tests/yalmip/yalmip/YALMIP-master/solvers/callquadprog.m:63-69
 * ([x,fmin,flag,output,lambda] = quadprog(Q,c,A,b,Aeq,beq,lb,ub,x0,ops)) and that
 * PLAN_NL_LPV_MPC_dt_WORKS_Oval.m:240-244 reaches through the optimizer object.
 *
 *  - Arguments as quadprog: [] for absent constraints; +-Inf bounds are inactive.  Full or
 *    SPARSE doubles: YALMIP hands quadprog the sparse Q, A, Aeq it slices out of F_struc
 *    (yalmip2quadprog.m:38-70; they stay sparse unless ops.LargeScale is set to 'off').
 *  - Batch: H n x n x B, f n x B (or n x 1 x B), A m x n x B, b m x B, ... solves B
 *    independent QPs in one GPU launch (pages must share sizes); outputs get a trailing
 *    batch dimension (x n x B, fval / exitflag 1 x B).
 *  - x0 is ignored (interior point), as quadprog's interior-point-convex algorithm does.
 *  - opts: struct with optional fields MaxIterations, OptimalityTolerance.
 *  - exitflag: 1 optimal, 0 iteration limit, -2 infeasible, -3 unbounded, -6 non-convex.
 *  - lambda: struct(ineqlin, eqlin, lower, upper); output: struct(iterations, algorithm,
 *    message, firstorderopt).
 *  - Errors through mexErrMsgIdAndTxt: cmpc:quadprog:args (shapes/types), cmpc:device.
 *
 * Struct form (cmpc_solve_mpc_batch — the structured LTV agent-QP of
 * PlannerLPV, LPV_Planner.py:279-475, for a batch of agents in one launch):
 *
 *   [z, kkt, iters, status] = cmpc_quadprog(S)
 *
 *   S.nx S.nu S.N S.ns           scalars;  S.Q nx x nx, S.R S.dR nu x nu, S.Qs ns x 1,
 *   S.u_lb S.u_ub nu x 1,        S.row_slack S.row_sign mc x 1 (slack index 0-based, -1 none),
 *   S.A nx x nx x N x B,         S.B nx x nu x N x B,   S.x0 nx x B,  S.u_prev nu x B,
 *   S.qlin nx x (N+1) x B,       S.C mc x nx x N x B,   S.h mc x N x B   (MATLAB order:
 *   A(i,j,k,b) = A_k(i,j) of agent b), optional S.tol, S.max_iter.
 *   z is nz x B in the reference layout, status per agent (OSQP codes, cmpc.h).
 *
 * Build in MATLAB:  mex -largeArrayDims cmpc_quadprog_mex.c -I<repo>/include -L<repo>/colaborativempc-_amd/lib -lcmpc
 * CI builds it against a mock mex.h (tests/mex_mock) because there is no MATLAB.
 */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "cmpc.h"
#include "mex.h"

static cmpc_ctx* g_ctx = NULL;

static void cleanup(void) {
    if (g_ctx) cmpc_destroy(g_ctx);
    g_ctx = NULL;
}

static size_t dim_or1(const mxArray* a, int k) {
    const mwSize nd = mxGetNumberOfDimensions(a);
    return (mwSize)k < nd ? (size_t)mxGetDimensions(a)[k] : 1;
}

static void require_double(const mxArray* a, const char* name) {
    if (!mxIsDouble(a) || mxIsComplex(a))
        mexErrMsgIdAndTxt("cmpc:quadprog:args", "%s must be a real double array", name);
}

/* densified copies of sparse arguments, freed at the end of the call */
#define MAX_DENSE 8
static double* g_dense[MAX_DENSE];
static int g_ndense = 0;

static void free_dense(void) {
    for (int i = 0; i < g_ndense; ++i) mxFree(g_dense[i]);
    g_ndense = 0;
}

/* column-major m x n copy of a sparse (CSC) matrix */
static const double* densify(const mxArray* a) {
    const size_t m = mxGetM(a), n = mxGetN(a);
    const size_t cnt = m * n;
    double* d = (double*)mxCalloc(cnt > 0 ? cnt : 1, sizeof(double));
    const double* pr = mxGetPr(a);
    const mwIndex* ir = mxGetIr(a);
    const mwIndex* jc = mxGetJc(a);
    for (size_t j = 0; j < n; ++j)
        for (mwIndex k = jc[j]; k < jc[j + 1]; ++k) d[j * m + ir[k]] = pr[k];
    if (g_ndense < MAX_DENSE) g_dense[g_ndense++] = d;
    return d;
}

/* per-page element count check: a must hold batch pages of exactly `per` elements
   (a sparse argument is one 2-D page) */
static const double* page_data(const mxArray* a, size_t per, size_t batch, const char* name) {
    if (mxIsEmpty(a)) return NULL;
    require_double(a, name);
    const size_t numel = mxGetNumberOfElements(a);
    if (numel != per * batch)
        mexErrMsgIdAndTxt("cmpc:quadprog:args", "%s has %zu elements, expected %zu (x %zu pages)", name, numel, per,
                          batch);
    return mxIsSparse(a) ? densify(a) : mxGetPr(a);
}

/* ---- struct form: the structured agent-QP batch (cmpc_solve_mpc_batch) ---- */
static const mxArray* sfield(const mxArray* S, const char* name, size_t numel, int required) {
    const mxArray* v = mxGetField(S, 0, name);
    if (!v || mxIsEmpty(v)) {
        if (required) mexErrMsgIdAndTxt("cmpc:quadprog:args", "struct form: field %s is required", name);
        return NULL;
    }
    require_double(v, name);
    if (mxIsSparse(v)) mexErrMsgIdAndTxt("cmpc:quadprog:args", "struct form: field %s must be full", name);
    if (numel && mxGetNumberOfElements(v) != numel)
        mexErrMsgIdAndTxt("cmpc:quadprog:args", "struct form: field %s has %zu elements, expected %zu", name,
                          mxGetNumberOfElements(v), numel);
    return v;
}

static int sint(const mxArray* S, const char* name) { return (int)mxGetScalar(sfield(S, name, 1, 1)); }

/* MATLAB page (r x c, column-major) -> row-major r x c, for `pages` consecutive pages */
static double* rowmajor(const double* src, size_t r, size_t c, size_t pages) {
    const size_t cnt = r * c * pages;
    double* d = (double*)mxCalloc(cnt > 0 ? cnt : 1, sizeof(double));
    for (size_t p = 0; p < pages; ++p)
        for (size_t i = 0; i < r; ++i)
            for (size_t j = 0; j < c; ++j) d[(p * r + i) * c + j] = src[p * r * c + j * r + i];
    return d;
}

static void mpc_struct(int nlhs, mxArray* plhs[], const mxArray* S) {
    if (nlhs > 4) mexErrMsgIdAndTxt("cmpc:quadprog:args", "struct form: at most 4 outputs");
    const int nx = sint(S, "nx"), nu = sint(S, "nu"), N = sint(S, "N"), ns = sint(S, "ns");
    if (nx < 1 || nu < 1 || N < 1 || ns < 0) mexErrMsgIdAndTxt("cmpc:quadprog:args", "struct form: bad dimensions");
    const mxArray* rs = sfield(S, "row_slack", 0, 1);
    const int mc = (int)mxGetNumberOfElements(rs);
    const mxArray* x0 = sfield(S, "x0", 0, 1);
    const size_t B = mxGetNumberOfElements(x0) / (size_t)nx;
    if (B * (size_t)nx != mxGetNumberOfElements(x0)) mexErrMsgIdAndTxt("cmpc:quadprog:args", "x0 must be nx x B");
    int rsl[CMPC_MAX_MC], rsg[CMPC_MAX_MC];
    if (mc > CMPC_MAX_MC) mexErrMsgIdAndTxt("cmpc:quadprog:args", "struct form: too many rows per stage");
    const double* prs = mxGetPr(rs);
    const double* psg = mxGetPr(sfield(S, "row_sign", (size_t)mc, 1));
    for (int r = 0; r < mc; ++r) {
        rsl[r] = (int)prs[r];
        rsg[r] = (int)psg[r];
    }
    double* Q = rowmajor(mxGetPr(sfield(S, "Q", (size_t)nx * nx, 1)), nx, nx, 1);
    double* R = rowmajor(mxGetPr(sfield(S, "R", (size_t)nu * nu, 1)), nu, nu, 1);
    double* dR = rowmajor(mxGetPr(sfield(S, "dR", (size_t)nu * nu, 1)), nu, nu, 1);
    const double dummy = 1.0;
    cmpc_mpc_weights w = {Q, R, dR, ns ? mxGetPr(sfield(S, "Qs", (size_t)ns, 1)) : &dummy,
                          mxGetPr(sfield(S, "u_ub", (size_t)nu, 1)), mxGetPr(sfield(S, "u_lb", (size_t)nu, 1)), rsl, rsg};
    double* A = rowmajor(mxGetPr(sfield(S, "A", (size_t)nx * nx * N * B, 1)), nx, nx, (size_t)N * B);
    double* Bm = rowmajor(mxGetPr(sfield(S, "B", (size_t)nx * nu * N * B, 1)), nx, nu, (size_t)N * B);
    double* C = rowmajor(mxGetPr(sfield(S, "C", (size_t)mc * nx * N * B, 1)), mc, nx, (size_t)N * B);
    cmpc_mpc_data in = {A, Bm, mxGetPr(x0), mxGetPr(sfield(S, "u_prev", (size_t)nu * B, 1)),
                        mxGetPr(sfield(S, "qlin", (size_t)nx * (N + 1) * B, 1)), C,
                        mxGetPr(sfield(S, "h", (size_t)mc * N * B, 1))};
    cmpc_mpc_dims dims = {nx, nu, N, ns, mc, (int)B};
    const size_t nz = (size_t)(nx + ns) * (N + 1) + 2 * (size_t)nu * N;
    mxArray* Z = mxCreateDoubleMatrix(nz, B, mxREAL);
    mxArray* KK = mxCreateDoubleMatrix(1, B, mxREAL);
    mxArray* IT = mxCreateDoubleMatrix(1, B, mxREAL);
    mxArray* ST = mxCreateDoubleMatrix(1, B, mxREAL);
    int* iters = (int*)mxCalloc(B ? B : 1, sizeof(int));
    int* status = (int*)mxCalloc(B ? B : 1, sizeof(int));
    cmpc_mpc_out out = {mxGetPr(Z), mxGetPr(KK), iters, status};
    cmpc_opts o;
    memset(&o, 0, sizeof(o));
    const mxArray* v = sfield(S, "tol", 1, 0);
    if (v) o.tol = mxGetScalar(v);
    v = sfield(S, "max_iter", 1, 0);
    if (v) o.max_iter = (int)mxGetScalar(v);
    const int rc = cmpc_solve_mpc_batch(g_ctx, &dims, &w, &in, &out, &o);
    mxFree(Q); mxFree(R); mxFree(dR); mxFree(A); mxFree(Bm); mxFree(C);
    if (rc != CMPC_OK) mexErrMsgIdAndTxt("cmpc:solve", "cmpc_solve_mpc_batch failed (%d): %s", rc, cmpc_last_error(g_ctx));
    for (size_t b = 0; b < B; ++b) {
        mxGetPr(IT)[b] = iters[b];
        mxGetPr(ST)[b] = status[b];
    }
    mxFree(iters);
    mxFree(status);
    plhs[0] = Z;
    if (nlhs > 1) plhs[1] = KK;
    if (nlhs > 2) plhs[2] = IT;
    if (nlhs > 3) plhs[3] = ST;
}

static void ensure_ctx(void) {
    if (!g_ctx) {
        if (cmpc_create(&g_ctx, 0) != CMPC_OK) {
            g_ctx = NULL;
            mexErrMsgIdAndTxt("cmpc:device", "cmpc_quadprog: no usable MI355X (gfx950) device");
        }
        mexAtExit(cleanup);
    }
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    /* forget (do not free) the list: a previous call that ended in mexErrMsgIdAndTxt left its
       mxCalloc buffers to MATLAB, which frees non-persistent memory when a MEX call errors out */
    g_ndense = 0;
    if (nrhs == 1 && mxIsStruct(prhs[0])) {
        ensure_ctx();
        mpc_struct(nlhs, plhs, prhs[0]);
        return;
    }
    if (nrhs < 2 || nrhs > 10) mexErrMsgIdAndTxt("cmpc:quadprog:args", "usage: cmpc_quadprog(H,f,A,b,Aeq,beq,lb,ub[,x0,opts]) or cmpc_quadprog(S)");
    if (nlhs > 5) mexErrMsgIdAndTxt("cmpc:quadprog:args", "at most 5 outputs");
    const mxArray* H = prhs[0];
    require_double(H, "H");
    const size_t n = dim_or1(H, 0);
    if (n == 0 || dim_or1(H, 1) != n) mexErrMsgIdAndTxt("cmpc:quadprog:args", "H must be n x n (x B)");
    const size_t batch = mxGetNumberOfElements(H) / (n * n);
    const mxArray* empty = NULL;
    const mxArray* arg[8];
    for (int i = 0; i < 8; ++i) arg[i] = i < nrhs ? prhs[i] : empty;
    /* m_ineq / m_eq from A, Aeq (first dimension) */
    const size_t mi = (arg[2] && !mxIsEmpty(arg[2])) ? dim_or1(arg[2], 0) : 0;
    const size_t me = (arg[4] && !mxIsEmpty(arg[4])) ? dim_or1(arg[4], 0) : 0;
    if (mi && dim_or1(arg[2], 1) != n) mexErrMsgIdAndTxt("cmpc:quadprog:args", "A must have n columns");
    if (me && dim_or1(arg[4], 1) != n) mexErrMsgIdAndTxt("cmpc:quadprog:args", "Aeq must have n columns");
    cmpc_qp_data in;
    memset(&in, 0, sizeof(in));
    in.H = mxIsSparse(H) ? densify(H) : mxGetPr(H);
    in.f = page_data(arg[1], n, batch, "f");
    if (!in.f) mexErrMsgIdAndTxt("cmpc:quadprog:args", "f is required");
    if (mi) {
        in.A = page_data(arg[2], mi * n, batch, "A");
        if (!arg[3] || mxIsEmpty(arg[3])) mexErrMsgIdAndTxt("cmpc:quadprog:args", "A given without b");
        in.b = page_data(arg[3], mi, batch, "b");
    }
    if (me) {
        in.Aeq = page_data(arg[4], me * n, batch, "Aeq");
        if (!arg[5] || mxIsEmpty(arg[5])) mexErrMsgIdAndTxt("cmpc:quadprog:args", "Aeq given without beq");
        in.beq = page_data(arg[5], me, batch, "beq");
    }
    if (arg[6]) in.lb = page_data(arg[6], n, batch, "lb");
    if (arg[7]) in.ub = page_data(arg[7], n, batch, "ub");
    cmpc_opts o;
    memset(&o, 0, sizeof(o));
    if (nrhs >= 10 && !mxIsEmpty(prhs[9])) {
        if (!mxIsStruct(prhs[9])) mexErrMsgIdAndTxt("cmpc:quadprog:args", "opts must be a struct");
        const mxArray* v = mxGetField(prhs[9], 0, "MaxIterations");
        if (v && !mxIsEmpty(v)) o.max_iter = (int)mxGetScalar(v);
        v = mxGetField(prhs[9], 0, "OptimalityTolerance");
        if (v && !mxIsEmpty(v)) o.tol = mxGetScalar(v);
    }

    mwSize xd[2] = {(mwSize)n, (mwSize)batch};
    mxArray* X = mxCreateNumericArray(2, xd, mxDOUBLE_CLASS, mxREAL);
    mxArray* FV = mxCreateDoubleMatrix(1, batch, mxREAL);
    mxArray* EF = mxCreateDoubleMatrix(1, batch, mxREAL);
    mxArray* LI = mxCreateDoubleMatrix(mi, batch, mxREAL);
    mxArray* LE = mxCreateDoubleMatrix(me, batch, mxREAL);
    mxArray* LL = mxCreateDoubleMatrix(n, batch, mxREAL);
    mxArray* LU = mxCreateDoubleMatrix(n, batch, mxREAL);
    mxArray* IT = mxCreateDoubleMatrix(1, batch, mxREAL);
    mxArray* RS = mxCreateDoubleMatrix(1, batch, mxREAL);
    int* flags = (int*)mxCalloc(batch ? batch : 1, sizeof(int));
    int* iters = (int*)mxCalloc(batch ? batch : 1, sizeof(int));
    cmpc_qp_out out = {mxGetPr(X), mxGetPr(FV), flags, iters, mi ? mxGetPr(LI) : NULL, me ? mxGetPr(LE) : NULL,
                       mxGetPr(LL), mxGetPr(LU), mxGetPr(RS)};
    cmpc_qp_dims dims = {(int)n, (int)mi, (int)me, (int)batch, 1 /* column-major */};

    ensure_ctx();
    const int rc = cmpc_solve_qp_batch(g_ctx, &dims, &in, &out, &o);
    free_dense();
    if (rc != CMPC_OK) mexErrMsgIdAndTxt("cmpc:solve", "cmpc_solve_qp_batch failed (%d): %s", rc, cmpc_last_error(g_ctx));
    double* ef = mxGetPr(EF);
    double* it = mxGetPr(IT);
    for (size_t p = 0; p < batch; ++p) {
        ef[p] = flags[p];
        it[p] = iters[p];
    }
    mxFree(flags);
    mxFree(iters);

    plhs[0] = X;
    if (nlhs > 1) plhs[1] = FV;
    if (nlhs > 2) plhs[2] = EF;
    if (nlhs > 3) {
        const char* fo[] = {"iterations", "algorithm", "message", "firstorderopt"};
        mxArray* O = mxCreateStructMatrix(1, 1, 4, fo);
        mxSetField(O, 0, "iterations", IT);
        mxSetField(O, 0, "algorithm", mxCreateString("cmpc interior-point (MI355X, batched)"));
        mxSetField(O, 0, "message", mxCreateString(batch == 1 && ef[0] == 1 ? "Minimum found" : "See exitflag"));
        mxSetField(O, 0, "firstorderopt", RS);
        plhs[3] = O;
    }
    if (nlhs > 4) {
        const char* fl[] = {"ineqlin", "eqlin", "lower", "upper"};
        mxArray* Lm = mxCreateStructMatrix(1, 1, 4, fl);
        mxSetField(Lm, 0, "ineqlin", LI);
        mxSetField(Lm, 0, "eqlin", LE);
        mxSetField(Lm, 0, "lower", LL);
        mxSetField(Lm, 0, "upper", LU);
        plhs[4] = Lm;
    }
}
