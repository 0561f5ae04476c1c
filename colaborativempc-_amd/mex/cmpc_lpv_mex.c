/* cmpc_lpv — MATLAB MEX gateway over libcmpc's reference-semantics LPV path (include/cmpc.h).
 *
 * The MATLAB host of north_star drives the reference's agent model (PlannerLPV,
 * planner/lib/plan_lib/distributedPlanner/LPV_Planner.py:115-182) and its consensus loop
 * (planner/scripts/LPV_HP_N_main.py:96-117; one process per agent over ROS in
 * ROS/src/planner_experiments/src/LPV_ROS_main.py:66-77,124-150) through these calls:
 *
 *   [z, status, kkt, iters, planes] = cmpc_lpv('solve', P, D)
 *       one control step of every agent in D (cmpc_solve_lpv_batch): LPV scheduling, planes,
 *       weights, QP build and solve on the GPU.
 *   h = cmpc_lpv('rounds_create', P, D, S)           cmpc_lpv_rounds_create: device-resident rounds
 *   [done, infeasible] = cmpc_lpv('rounds_step', h, k)   k rounds (gather, solve, advance, exchange)
 *   [z, status, kkt, iters, x0, planes] = cmpc_lpv('rounds_read', h)
 *   T = cmpc_lpv('rounds_get_traj', h)               this rank's predicted X, Y (host exchange)
 *   cmpc_lpv('rounds_set_traj', h, T)                the gathered exchange buffer (host exchange)
 *   cmpc_lpv('rounds_destroy', h)
 *   id = cmpc_lpv('comm_id');  cmpc_lpv('comm_init', nranks, rank, id)   RCCL exchange (one GPU per rank)
 *
 *   P: struct — model lf lr m I Cf Cr mu (config/base_class.py:20-28), limits vx_ref min_dist max_vel
 *      min_vel max_rs max_ls max_ac max_dc (:30-41), dt, wq, Q 9x9, Qs 3x1 (diagonal), R 2x2, dR 2x2
 *      (scripts/config_files/config_LPV.py:6-11), N, track (struct s0, len, curv, half_width: one
 *      entry per PointAndTangent row, track_initialization.py:220-300); optional tol, max_iter,
 *      rescue (default 1: CMPC_FLAG_RESCUE, as PlannerLPV), polish (default 1: CMPC_FLAG_POLISH with
 *      rescue, as PlannerLPV — OSQP's polish=True, LPV_Planner.py:233).
 *   D: struct, MATLAB order (B agents, last dimension): x0 9xB, x_last 9 x rows x B (rows N+1 at the
 *      first step, N afterwards), u_last 2xNxB, u_old 2xB, pose 2x(N+1)xB, x_agents 2 x nb x (N+1) x B
 *      (optional: none = no neighbours).  This is the C ABI's row-major layout read backwards, so
 *      nothing is transposed.  z is nz x B (nz = 12(N+1)+4N, LPV_Planner.py:164-178).
 *   S: struct — nbr nb x B (0-based global agent indices), optional n_total, self_offset, traj
 *      2 x (N+1) x n_total (the initial exchange buffer), host_exchange, halt (default 1).
 *
 * Handles are small integers (index into this gateway's table).  Errors through
 * mexErrMsgIdAndTxt: cmpc:lpv:args, cmpc:device, cmpc:solve.
 * Build in MATLAB:  mex -largeArrayDims cmpc_lpv_mex.c -I<repo>/include -L<repo>/colaborativempc-_amd/lib -lcmpc
 * CI builds it against the mock mex.h of tests/mex_mock.
 */
#include <math.h>
#include <string.h>

#include "cmpc.h"
#include "mex.h"

#define MAX_HANDLES 64

static cmpc_ctx* g_ctx = NULL;
static cmpc_lpv_rounds* g_h[MAX_HANDLES];
static int g_hN[MAX_HANDLES], g_hB[MAX_HANDLES], g_hnb[MAX_HANDLES], g_hT[MAX_HANDLES];

static void cleanup(void) {
    for (int i = 0; i < MAX_HANDLES; ++i)
        if (g_h[i]) {
            cmpc_lpv_rounds_destroy(g_h[i]);
            g_h[i] = NULL;
        }
    if (g_ctx) cmpc_destroy(g_ctx);
    g_ctx = NULL;
}

static void ensure_ctx(void) {
    if (!g_ctx) {
        if (cmpc_create(&g_ctx, 0) != CMPC_OK) {
            g_ctx = NULL;
            mexErrMsgIdAndTxt("cmpc:device", "cmpc_lpv: no usable MI355X (gfx950) device");
        }
        mexAtExit(cleanup);
    }
}

static void check(int rc, const char* what) {
    if (rc != CMPC_OK) mexErrMsgIdAndTxt("cmpc:solve", "%s failed (%d): %s", what, rc, cmpc_last_error(g_ctx));
}

static const mxArray* field(const mxArray* S, const char* name, size_t numel, int required) {
    const mxArray* v = mxGetField(S, 0, name);
    if (!v || mxIsEmpty(v)) {
        if (required) mexErrMsgIdAndTxt("cmpc:lpv:args", "field %s is required", name);
        return NULL;
    }
    if (!mxIsDouble(v) || mxIsComplex(v) || mxIsSparse(v))
        mexErrMsgIdAndTxt("cmpc:lpv:args", "field %s must be a full real double array", name);
    if (numel && mxGetNumberOfElements(v) != numel)
        mexErrMsgIdAndTxt("cmpc:lpv:args", "field %s has %zu elements, expected %zu", name, mxGetNumberOfElements(v),
                          numel);
    return v;
}

static double scalar(const mxArray* S, const char* name) { return mxGetScalar(field(S, name, 1, 1)); }

static double scalar_or(const mxArray* S, const char* name, double dflt) {
    const mxArray* v = field(S, name, 1, 0);
    return v ? mxGetScalar(v) : dflt;
}

static const mxArray* require_struct(const mxArray* a, const char* what) {
    if (!a || !mxIsStruct(a)) mexErrMsgIdAndTxt("cmpc:lpv:args", "%s must be a struct", what);
    return a;
}

/* P -> parameters, track, horizon, options */
typedef struct {
    cmpc_lpv_params prm;
    cmpc_track track;
    cmpc_opts opts;
    int N;
} lpv_setup;

static void read_params(const mxArray* P, lpv_setup* s) {
    require_struct(P, "P");
    memset(s, 0, sizeof(*s));
    cmpc_lpv_params* p = &s->prm;
    p->lf = scalar(P, "lf"); p->lr = scalar(P, "lr"); p->m = scalar(P, "m"); p->I = scalar(P, "I");
    p->Cf = scalar(P, "Cf"); p->Cr = scalar(P, "Cr"); p->mu = scalar(P, "mu");
    p->vx_ref = scalar(P, "vx_ref"); p->min_dist = scalar(P, "min_dist"); p->max_vel = scalar(P, "max_vel");
    p->min_vel = scalar(P, "min_vel"); p->max_rs = scalar(P, "max_rs"); p->max_ls = scalar(P, "max_ls");
    p->max_ac = scalar(P, "max_ac"); p->max_dc = scalar(P, "max_dc"); p->dt = scalar(P, "dt");
    p->wq = scalar(P, "wq");
    /* Q 9x9, R 2x2, dR 2x2: MATLAB column-major -> row-major (symmetric in practice; transposed anyway) */
    const double* Q = mxGetPr(field(P, "Q", 81, 1));
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) p->Q[i * 9 + j] = Q[j * 9 + i];
    const double* R = mxGetPr(field(P, "R", 4, 1));
    const double* dR = mxGetPr(field(P, "dR", 4, 1));
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) {
            p->R[i * 2 + j] = R[j * 2 + i];
            p->dR[i * 2 + j] = dR[j * 2 + i];
        }
    const mxArray* qs = field(P, "Qs", 0, 1);
    const size_t nq = mxGetNumberOfElements(qs);
    if (nq == 3) {
        for (int j = 0; j < 3; ++j) p->Qs[j] = mxGetPr(qs)[j];
    } else if (nq == 9) {  /* the reference passes Qs as a 3x3 (diagonal) matrix */
        for (int j = 0; j < 3; ++j) p->Qs[j] = mxGetPr(qs)[j * 4];
    } else {
        mexErrMsgIdAndTxt("cmpc:lpv:args", "Qs must be 3x1 or 3x3 (diagonal)");
    }
    s->N = (int)scalar(P, "N");
    const mxArray* T = require_struct(mxGetField(P, 0, "track"), "P.track");
    const mxArray* s0 = field(T, "s0", 0, 1);
    const size_t ns = mxGetNumberOfElements(s0);
    s->track.nseg = (int)ns;
    s->track.s0 = mxGetPr(s0);
    s->track.len = mxGetPr(field(T, "len", ns, 1));
    s->track.curv = mxGetPr(field(T, "curv", ns, 1));
    s->track.half_width = mxGetPr(field(T, "half_width", ns, 1));
    s->opts.tol = scalar_or(P, "tol", 0.0);
    s->opts.max_iter = (int)scalar_or(P, "max_iter", 0.0);
    s->opts.flags = scalar_or(P, "rescue", 1.0) != 0.0
                        ? CMPC_FLAG_RESCUE | (scalar_or(P, "polish", 1.0) != 0.0 ? CMPC_FLAG_POLISH : 0)
                        : 0;
}

/* D -> batch, neighbours, rows of x_last, data pointers (no copies: MATLAB order is the ABI's) */
typedef struct {
    int B, nb, rows;
    cmpc_lpv_data d;
} lpv_batch;

static void read_data(const mxArray* D, int N, lpv_batch* b) {
    require_struct(D, "D");
    const mxArray* x0 = field(D, "x0", 0, 1);
    const size_t B = mxGetNumberOfElements(x0) / 9;
    if (B * 9 != mxGetNumberOfElements(x0) || B == 0) mexErrMsgIdAndTxt("cmpc:lpv:args", "x0 must be 9 x B");
    const mxArray* xl = field(D, "x_last", 0, 1);
    const size_t rows = mxGetNumberOfElements(xl) / (9 * B);
    if (rows * 9 * B != mxGetNumberOfElements(xl) || (rows != (size_t)N && rows != (size_t)N + 1))
        mexErrMsgIdAndTxt("cmpc:lpv:args", "x_last must be 9 x (N or N+1) x B");
    const mxArray* xa = field(D, "x_agents", 0, 0);
    size_t nb = 0;
    if (xa) {
        nb = mxGetNumberOfElements(xa) / (2 * (size_t)(N + 1) * B);
        if (nb * 2 * (N + 1) * B != mxGetNumberOfElements(xa) || nb == 0)
            mexErrMsgIdAndTxt("cmpc:lpv:args", "x_agents must be 2 x nb x (N+1) x B");
    }
    b->B = (int)B;
    b->nb = (int)nb;
    b->rows = (int)rows;
    b->d.x0 = mxGetPr(x0);
    b->d.x_last = mxGetPr(xl);
    b->d.u_last = mxGetPr(field(D, "u_last", 2 * (size_t)N * B, 1));
    const mxArray* uo = field(D, "u_old", 2 * B, 0);
    b->d.u_old = uo ? mxGetPr(uo) : NULL;
    b->d.x_agents = xa ? mxGetPr(xa) : NULL;
    b->d.pose = mxGetPr(field(D, "pose", 2 * (size_t)(N + 1) * B, 1));
}

static mxArray* dmat3(size_t a, size_t b, size_t c) {
    mwSize d[3] = {(mwSize)a, (mwSize)b, (mwSize)c};
    return mxCreateNumericArray(3, d, mxDOUBLE_CLASS, mxREAL);
}

static mxArray* planes_array(int N, int nb, int B) {
    mwSize d[4] = {(mwSize)(nb ? nb : 1), 3, (mwSize)N, (mwSize)B};
    return mxCreateNumericArray(4, d, mxDOUBLE_CLASS, mxREAL);
}

static void solve(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 3) mexErrMsgIdAndTxt("cmpc:lpv:args", "usage: cmpc_lpv('solve', P, D)");
    lpv_setup s;
    read_params(prhs[1], &s);
    lpv_batch b;
    read_data(prhs[2], s.N, &b);
    double* zero_uo = NULL;
    if (!b.d.u_old) {  /* PlannerLPV's initial OldSteering / OldAccelera (LPV_Planner.py:86-87) */
        zero_uo = (double*)mxCalloc(2 * (size_t)b.B, sizeof(double));
        b.d.u_old = zero_uo;
    }
    const size_t nz = 12 * (size_t)(s.N + 1) + 4 * (size_t)s.N;
    mxArray* Z = mxCreateDoubleMatrix(nz, b.B, mxREAL);
    mxArray* KK = mxCreateDoubleMatrix(1, b.B, mxREAL);
    mxArray* IT = mxCreateDoubleMatrix(1, b.B, mxREAL);
    mxArray* ST = mxCreateDoubleMatrix(1, b.B, mxREAL);
    mxArray* PL = planes_array(s.N, b.nb, b.B);
    int* iters = (int*)mxCalloc(b.B, sizeof(int));
    int* status = (int*)mxCalloc(b.B, sizeof(int));
    cmpc_lpv_dims dims = {b.B, s.N, b.nb, b.rows};
    cmpc_lpv_out out = {mxGetPr(Z), b.nb ? mxGetPr(PL) : NULL, mxGetPr(KK), iters, status};
    ensure_ctx();
    const int rc = cmpc_solve_lpv_batch(g_ctx, &s.prm, &s.track, &dims, &b.d, &out, &s.opts);
    if (zero_uo) mxFree(zero_uo);
    check(rc, "cmpc_solve_lpv_batch");
    for (int i = 0; i < b.B; ++i) {
        mxGetPr(IT)[i] = iters[i];
        mxGetPr(ST)[i] = status[i];
    }
    mxFree(iters);
    mxFree(status);
    plhs[0] = Z;
    if (nlhs > 1) plhs[1] = ST;
    if (nlhs > 2) plhs[2] = KK;
    if (nlhs > 3) plhs[3] = IT;
    if (nlhs > 4) plhs[4] = PL;
}

static int handle_of(const mxArray* a) {
    if (!a || !mxIsDouble(a) || mxGetNumberOfElements(a) != 1) mexErrMsgIdAndTxt("cmpc:lpv:args", "bad rounds handle");
    const int h = (int)mxGetScalar(a) - 1;
    if (h < 0 || h >= MAX_HANDLES || !g_h[h]) mexErrMsgIdAndTxt("cmpc:lpv:args", "bad rounds handle");
    return h;
}

static void rounds_create(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs;
    if (nrhs != 4) mexErrMsgIdAndTxt("cmpc:lpv:args", "usage: h = cmpc_lpv('rounds_create', P, D, S)");
    lpv_setup s;
    read_params(prhs[1], &s);
    lpv_batch b;
    read_data(prhs[2], s.N, &b);
    if (b.rows != s.N + 1) mexErrMsgIdAndTxt("cmpc:lpv:args", "rounds start from Last_xPredicted with N+1 rows");
    const mxArray* S = require_struct(prhs[3], "S");
    const int n_total = (int)scalar_or(S, "n_total", (double)b.B);
    const int self_offset = (int)scalar_or(S, "self_offset", 0.0);
    const mxArray* nbr = field(S, "nbr", 0, b.nb > 0);
    int nb = nbr ? (int)(mxGetNumberOfElements(nbr) / (size_t)b.B) : 0;
    if (nbr && (size_t)nb * b.B != mxGetNumberOfElements(nbr)) mexErrMsgIdAndTxt("cmpc:lpv:args", "nbr must be nb x B");
    const mxArray* traj = field(S, "traj", 2 * (size_t)(s.N + 1) * n_total, 0);
    int* inbr = (int*)mxCalloc((size_t)(nb ? nb : 1) * b.B, sizeof(int));
    for (size_t i = 0; nbr && i < (size_t)nb * b.B; ++i) inbr[i] = (int)mxGetPr(nbr)[i];
    const int flags = (scalar_or(S, "host_exchange", 0.0) != 0.0 ? CMPC_ROUNDS_HOST_EXCHANGE : 0) |
                      (scalar_or(S, "halt", 1.0) != 0.0 ? 0 : CMPC_ROUNDS_NO_HALT);
    cmpc_lpv_rounds_dims dims = {n_total, b.B, self_offset, s.N, nb, flags};
    cmpc_lpv_rounds_init init = {b.d.x0, b.d.x_last, b.d.u_last, b.d.u_old, inbr, traj ? mxGetPr(traj) : NULL};
    int slot = -1;
    for (int i = 0; i < MAX_HANDLES && slot < 0; ++i)
        if (!g_h[i]) slot = i;
    if (slot < 0) {
        mxFree(inbr);
        mexErrMsgIdAndTxt("cmpc:lpv:args", "too many open rounds handles (%d)", MAX_HANDLES);
    }
    ensure_ctx();
    const int rc = cmpc_lpv_rounds_create(g_ctx, &s.prm, &s.track, &dims, &init, &s.opts, &g_h[slot]);
    mxFree(inbr);
    check(rc, "cmpc_lpv_rounds_create");
    g_hN[slot] = s.N;
    g_hB[slot] = b.B;
    g_hnb[slot] = nb;
    g_hT[slot] = n_total;
    plhs[0] = mxCreateDoubleMatrix(1, 1, mxREAL);
    mxGetPr(plhs[0])[0] = slot + 1;
}

static void rounds_step(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 3) mexErrMsgIdAndTxt("cmpc:lpv:args", "usage: [done, infeasible] = cmpc_lpv('rounds_step', h, k)");
    const int h = handle_of(prhs[1]);
    const int k = (int)mxGetScalar(prhs[2]);
    int done = 0, bad = 0;
    check(cmpc_lpv_rounds_step(g_h[h], k, &done, &bad), "cmpc_lpv_rounds_step");
    plhs[0] = mxCreateDoubleMatrix(1, 1, mxREAL);
    mxGetPr(plhs[0])[0] = done;
    if (nlhs > 1) {
        plhs[1] = mxCreateDoubleMatrix(1, 1, mxREAL);
        mxGetPr(plhs[1])[0] = bad;
    }
}

static void rounds_read(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 2) mexErrMsgIdAndTxt("cmpc:lpv:args", "usage: [z, status, kkt, iters, x0, planes] = cmpc_lpv('rounds_read', h)");
    const int h = handle_of(prhs[1]);
    const int N = g_hN[h], B = g_hB[h], nb = g_hnb[h];
    const size_t nz = 12 * (size_t)(N + 1) + 4 * (size_t)N;
    mxArray* Z = mxCreateDoubleMatrix(nz, B, mxREAL);
    mxArray* ST = mxCreateDoubleMatrix(1, B, mxREAL);
    mxArray* KK = mxCreateDoubleMatrix(1, B, mxREAL);
    mxArray* IT = mxCreateDoubleMatrix(1, B, mxREAL);
    mxArray* X0 = mxCreateDoubleMatrix(9, B, mxREAL);
    mxArray* PL = planes_array(N, nb, B);
    int* iters = (int*)mxCalloc(B, sizeof(int));
    int* status = (int*)mxCalloc(B, sizeof(int));
    cmpc_lpv_rounds_out o = {mxGetPr(Z), mxGetPr(KK), iters, status, mxGetPr(X0), nb ? mxGetPr(PL) : NULL};
    const int rc = cmpc_lpv_rounds_read(g_h[h], &o);
    if (rc == CMPC_OK)
        for (int i = 0; i < B; ++i) {
            mxGetPr(IT)[i] = iters[i];
            mxGetPr(ST)[i] = status[i];
        }
    mxFree(iters);
    mxFree(status);
    check(rc, "cmpc_lpv_rounds_read");
    plhs[0] = Z;
    if (nlhs > 1) plhs[1] = ST;
    if (nlhs > 2) plhs[2] = KK;
    if (nlhs > 3) plhs[3] = IT;
    if (nlhs > 4) plhs[4] = X0;
    if (nlhs > 5) plhs[5] = PL;
}

static void rounds_traj(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[], int set) {
    (void)nlhs;
    if (nrhs != (set ? 3 : 2)) mexErrMsgIdAndTxt("cmpc:lpv:args", "usage: rounds_get_traj(h) / rounds_set_traj(h, T)");
    const int h = handle_of(prhs[1]);
    const int N = g_hN[h];
    if (set) {
        const mxArray* T = prhs[2];
        if (!mxIsDouble(T) || mxGetNumberOfElements(T) != 2 * (size_t)(N + 1) * g_hT[h])
            mexErrMsgIdAndTxt("cmpc:lpv:args", "T must be 2 x (N+1) x n_total");
        check(cmpc_lpv_rounds_set_traj(g_h[h], mxGetPr(T)), "cmpc_lpv_rounds_set_traj");
        return;
    }
    mxArray* T = dmat3(2, N + 1, g_hB[h]);
    check(cmpc_lpv_rounds_get_traj(g_h[h], mxGetPr(T)), "cmpc_lpv_rounds_get_traj");
    plhs[0] = T;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char cmd[32];
    if (nrhs < 1 || !mxIsChar(prhs[0]) || mxGetString(prhs[0], cmd, sizeof cmd) != 0)
        mexErrMsgIdAndTxt("cmpc:lpv:args", "usage: cmpc_lpv('solve' | 'rounds_create' | 'rounds_step' | 'rounds_read' | "
                                           "'rounds_get_traj' | 'rounds_set_traj' | 'rounds_destroy' | 'comm_id' | "
                                           "'comm_init', ...)");
    if (!strcmp(cmd, "solve")) {
        solve(nlhs, plhs, nrhs, prhs);
    } else if (!strcmp(cmd, "rounds_create")) {
        rounds_create(nlhs, plhs, nrhs, prhs);
    } else if (!strcmp(cmd, "rounds_step")) {
        rounds_step(nlhs, plhs, nrhs, prhs);
    } else if (!strcmp(cmd, "rounds_read")) {
        rounds_read(nlhs, plhs, nrhs, prhs);
    } else if (!strcmp(cmd, "rounds_get_traj") || !strcmp(cmd, "rounds_set_traj")) {
        rounds_traj(nlhs, plhs, nrhs, prhs, cmd[7] == 's');
    } else if (!strcmp(cmd, "rounds_destroy")) {
        if (nrhs != 2) mexErrMsgIdAndTxt("cmpc:lpv:args", "usage: cmpc_lpv('rounds_destroy', h)");
        const int h = handle_of(prhs[1]);
        cmpc_lpv_rounds_destroy(g_h[h]);
        g_h[h] = NULL;
    } else if (!strcmp(cmd, "comm_id")) {
        unsigned char id[CMPC_COMM_ID_BYTES];
        if (cmpc_comm_id(id) != CMPC_OK) mexErrMsgIdAndTxt("cmpc:device", "cmpc_comm_id failed");
        plhs[0] = mxCreateDoubleMatrix(1, CMPC_COMM_ID_BYTES, mxREAL);
        for (int i = 0; i < CMPC_COMM_ID_BYTES; ++i) mxGetPr(plhs[0])[i] = id[i];
    } else if (!strcmp(cmd, "comm_init")) {
        if (nrhs != 4 || mxGetNumberOfElements(prhs[3]) != CMPC_COMM_ID_BYTES)
            mexErrMsgIdAndTxt("cmpc:lpv:args", "usage: cmpc_lpv('comm_init', nranks, rank, id)");
        unsigned char id[CMPC_COMM_ID_BYTES];
        for (int i = 0; i < CMPC_COMM_ID_BYTES; ++i) id[i] = (unsigned char)mxGetPr(prhs[3])[i];
        ensure_ctx();
        check(cmpc_comm_init(g_ctx, (int)mxGetScalar(prhs[1]), (int)mxGetScalar(prhs[2]), id), "cmpc_comm_init");
    } else {
        mexErrMsgIdAndTxt("cmpc:lpv:args", "unknown command '%s'", cmd);
    }
}
