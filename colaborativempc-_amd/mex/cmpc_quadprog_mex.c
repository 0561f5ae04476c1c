/* cmpc_quadprog — MATLAB MEX gateway over libcmpc's batched dense QP (cmpc_solve_qp_batch).
 *
 *   [x, fval, exitflag, output, lambda] = cmpc_quadprog(H, f, A, b, Aeq, beq, lb, ub [, x0, opts])
 *
 * Drop-in for the quadprog call YALMIP makes in
 * Matlab-tests/yalmip/yalmip/YALMIP-master/solvers/callquadprog.m:63-69
 * ([x,fmin,flag,output,lambda] = quadprog(Q,c,A,b,Aeq,beq,lb,ub,x0,ops)) and that
 * PLAN_NL_LPV_MPC_dt_WORKS_Oval.m:240-244 reaches through the optimizer object.
 *
 *  - Arguments as quadprog: [] for absent constraints; +-Inf bounds are inactive.
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
    if (!mxIsDouble(a) || mxIsComplex(a) || mxIsSparse(a))
        mexErrMsgIdAndTxt("cmpc:quadprog:args", "%s must be a real full double array", name);
}

/* per-page element count check: a must hold batch pages of exactly `per` elements */
static const double* page_data(const mxArray* a, size_t per, size_t batch, const char* name) {
    if (mxIsEmpty(a)) return NULL;
    require_double(a, name);
    const size_t numel = mxGetNumberOfElements(a);
    if (numel != per * batch)
        mexErrMsgIdAndTxt("cmpc:quadprog:args", "%s has %zu elements, expected %zu (x %zu pages)", name, numel, per,
                          batch);
    return mxGetPr(a);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 2 || nrhs > 10) mexErrMsgIdAndTxt("cmpc:quadprog:args", "usage: cmpc_quadprog(H,f,A,b,Aeq,beq,lb,ub[,x0,opts])");
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
    in.H = mxGetPr(H);
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

    if (!g_ctx) {
        if (cmpc_create(&g_ctx, 0) != CMPC_OK) {
            g_ctx = NULL;
            mexErrMsgIdAndTxt("cmpc:device", "cmpc_quadprog: no usable MI355X (gfx950) device");
        }
        mexAtExit(cleanup);
    }
    const int rc = cmpc_solve_qp_batch(g_ctx, &dims, &in, &out, &o);
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
