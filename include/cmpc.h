/* cmpc.h — C ABI of the MI355X-native collaborative-MPC QP solver (libcmpc.so).
 *
 * Drop-in boundary for the reference's per-control-step distributed QP path
 * (MarcFacerias/ColaborativeMPC-; paths relative to planner/lib/plan_lib/):
 *
 *   reference call site                                  replaced by
 *   ---------------------------------------------------  ---------------------------------
 *   PlannerLPV.solve (distributedPlanner/                cmpc_solve_lpv_batch[_dev]
 *     LPV_Planner.py:115-182): _EstimateABC :477-591,     (LPV scheduling + hyperplanes +
 *     compute_hyperplane planes/compute_plane.py:41-68,   weights + QP build fused on the
 *     compute_weights utilities/misc.py:10-18, builders   GPU, then the batched condensed
 *     :251-475, osqp_solve_qp :192-249                     IPM; one call = every agent)
 *   osqp_solve_qp(P,q,G,h,A,b) (LPV_Planner.py:192-249)   cmpc_solve_mpc_batch[_dev] for the
 *     on the structured LTV QP                            structured form (any nx, nu, N)
 *   quadprog(H,f,A,b,Aeq,beq,lb,ub) reached through       cmpc_solve_qp_batch (dense
 *     YALMIP callquadprog.m:63-69                         standard form, quadprog semantics)
 *     (Matlab-tests/yalmip/.../solvers/callquadprog.m)
 *   ROS topic exchange of predicted trajectories          cmpc_allgather_trajectories (RCCL
 *     (ROS/src/planner_experiments/src/LPV_ROS_main.py     all-gather, cmpc_comm_*); the solver
 *     :66-77,124-150) / LPV_HP_N_main.py:117              reads neighbour rows from device memory
 *
 * Conventions
 *  - All floating point is IEEE fp64, row-major, batch-major (agent b's block is
 *    contiguous).  No torch / C++ types cross this boundary.
 *  - Plain entry points take HOST pointers (the library stages them through
 *    device memory); *_dev entry points take DEVICE pointers plus a hipStream_t
 *    passed as void* (0 = default stream) and never synchronise the host.
 *  - Return value: CMPC_OK (0) or a negative CMPC_ERR_* code (API error);
 *    cmpc_last_error() gives the message.  Numerical outcome is reported per
 *    problem in status[] with OSQP's status_val codes so the reference's
 *    feasibility rule (status in {1, 2, -2}, LPV_Planner.py:246-248) applies
 *    unchanged.
 *  - A context is bound to one device and is not re-entrant: one context per
 *    host thread / stream.  One process per GPU for multi-GPU.
 *  - There is no CPU fallback: without a usable gfx950 device every solve
 *    returns CMPC_ERR_DEVICE.
 */
#ifndef CMPC_H
#define CMPC_H

#ifdef __cplusplus
extern "C" {
#endif

#define CMPC_ABI_VERSION 6   /* 2: cmpc_lpv_advance_dev status / infeasible, cmpc_lpv_rounds_*; 3: cmpc_opts.order;
                                4: cmpc_comm_sum_i32, cmpc_plan_mpc; 5: CMPC_FLAG_POLISH;
                                6: cmpc_plan_info waves_per_agent / polish_lds_bytes / polish_max_active */

/* API error codes */
#define CMPC_OK 0
#define CMPC_ERR_ARG (-1)
#define CMPC_ERR_DEVICE (-2)
#define CMPC_ERR_UNSUPPORTED (-3)
#define CMPC_ERR_NOMEM (-4)

/* Per-problem status (OSQP status_val values, LPV_Planner.py:243-249) */
#define CMPC_SOLVED 1
#define CMPC_SOLVED_INACCURATE 2
#define CMPC_MAX_ITER_REACHED (-2)
#define CMPC_PRIMAL_INFEASIBLE (-3)
#define CMPC_UNSOLVED (-10)

/* Size limits of the one-wavefront-per-agent solver (n = N*nu condensed variables). */
#define CMPC_MAX_NX 12
#define CMPC_MAX_NU 4
#define CMPC_MAX_NS 4
#define CMPC_MAX_MC 16
#define CMPC_MAX_NCOND 64      /* condensed one-wavefront-per-agent solvers (fp64); beyond it the
                                  stage-wise Riccati solver runs any horizon whose rows fit LDS
                                  (N = 125, nb <= 4 at nx = 9) */

typedef struct cmpc_ctx cmpc_ctx;

#define CMPC_FLAG_GENERIC 1  /* force the generic (runtime-dimension) kernel */
#define CMPC_FLAG_FP32 8     /* fp32 path (BASELINE cfg5): the Riccati factorisation and Newton recursions in
                                fp32 with fp64 iterates / residuals and a per-agent fp64 finish (opts.tol
                                ~1e-6) — on the stage-wise Riccati kernel where it has an fp32 instantiation
                                (nx,nu,mc = 6,3,6), on the lane-per-agent kernel with CMPC_FLAG_LANE or where
                                only that one is instantiated (nx,nu,mc,ns = 6,3,6,3 or 4,2,6,3); other
                                dimensions: CMPC_ERR_UNSUPPORTED */
#define CMPC_FLAG_RICCATI 16 /* force the stage-wise Riccati solver (fp64; the default when N*nu > 64) */
#define CMPC_FLAG_RESCUE 32 /* condensed solves (fp64): an agent whose factorisation breaks down short of
                               1e3 tol (status CMPC_UNSOLVED) continues from its last iterate on the
                               stage-wise Riccati solver (double-double near the solution) in a second
                               launch; a third launch restarts cold the rare one that fails again */
#define CMPC_FLAG_FINISH 64 /* with CMPC_FLAG_RESCUE: a breakdown whose best iterate already meets 1e3 tol
                               (status 2) is continued too, to full tolerance (slower; fewer status 2) */
#define CMPC_FLAG_LANE 128  /* lane-per-agent stage-wise solver in fp64 (one lane per agent, 64 agents per
                               wavefront: large batches of long horizons); CMPC_ERR_UNSUPPORTED for
                               dimensions it is not instantiated for (see CMPC_FLAG_FP32) */
#define CMPC_FLAG_POLISH 256 /* with CMPC_FLAG_RESCUE: OSQP's polish=True (LPV_Planner.py:233) for the interior-
                               point iterate — a condensed breakdown at the rounding floor (status 2) takes
                               its active set {lambda_r > t_r} as exact, solves that equality-constrained QP
                               (range-space KKT, two active-set corrections) and returns it when its merit
                               is lower (status 1 below tol) */
#define CMPC_FLAG_ONE_WAVE 512  /* the condensed kernel's fused double-integrator instantiation: one wavefront per
                                   agent (the default there); the stage-wise Riccati kernel: one wavefront per agent
                                   also where its latency mode (four per agent) would apply */
#define CMPC_FLAG_TWO_WAVES 1024 /* ... two wavefronts per agent (a 128-lane workgroup: split K build, the
                                   predictor's right-hand side on the second wave); bit-identical results, no
                                   faster at 512 agents on one MI355X, so opt-in.  Applies to the
                                   fused double-integrator round only (cmpc_di_solve_dev, the DS instantiation);
                                   other solves run one wavefront per agent.  Setting both wave flags is
                                   CMPC_ERR_ARG */
#define CMPC_FLAG_ALL (CMPC_FLAG_GENERIC | CMPC_FLAG_FP32 | CMPC_FLAG_RICCATI | CMPC_FLAG_RESCUE | CMPC_FLAG_FINISH | \
                       CMPC_FLAG_LANE | CMPC_FLAG_POLISH | CMPC_FLAG_ONE_WAVE | CMPC_FLAG_TWO_WAVES)
                       /* other bits: CMPC_ERR_ARG */

typedef struct {
    double tol;    /* relative stationarity/feasibility tolerance (complementarity: 1e-4*tol); <= 0 selects 1e-9 */
    int max_iter;  /* interior-point iteration cap; <= 0 selects 60 */
    int flags;     /* CMPC_FLAG_* */
    void* stamps;  /* optional DEVICE buffer, batch x 16 uint64: per-section shader-clock counts of the
                      specialised kernel (diagnostic; NULL in production) */
    const int* order; /* optional DEVICE array, batch int32, a permutation of 0..batch-1: the launch order of
                         the stage-wise Riccati solver (workgroup i solves agent order[i]; every output stays
                         at its agent's index).  With many agents per SIMD the launch ends with its slowest
                         solves; listing last round's agents by descending IPM iterations starts them first
                         (cmpc.rounds.DIRounds(lpt=True)).  The lane-per-agent solver (CMPC_FLAG_FP32 /
                         LANE) packs its wavefronts in this order, so each holds agents of similar
                         iteration counts.  Honoured by cmpc_solve_mpc_batch_dev; NULL:
                         identity.  Entries are clamped into range.  A non-permutation is undefined
                         behaviour: a missing agent is left unsolved, and a duplicated one is solved by
                         two workgroups (lanes) at once into the same scratch and outputs (a data race).
                         The library does not check it (the device array is read by the kernels only);
                         cmpc.rounds.DIRounds builds it by argsort, always a permutation.
                         Exception: a lane-per-agent batch whose scratch reaches 2 GiB runs as consecutive
                         sub-launches in agent order (mpc_lane.hip) and ignores both `order` and `stamps`
                         (same results; only the wavefront packing is lost).  cfg5 (8192 agents) stays
                         below that size; the bound is ~19.7k agents at N = 50. */
} cmpc_opts;

int cmpc_abi_version(void);
/* Create a context on HIP device `device` (ordinal among visible devices). */
int cmpc_create(cmpc_ctx** ctx, int device);
int cmpc_destroy(cmpc_ctx* ctx);
const char* cmpc_last_error(const cmpc_ctx* ctx);

/* ------------------------------------------------------------------------
 * Structured LTV agent-QP batch (the hot path).  For every agent b:
 *
 *   z = [xi_0 .. xi_N | u_0 .. u_{N-1} | du_0 .. du_{N-1}],  xi_k = [x_k (nx) | s_k (ns)]
 *   min  1/2 z'Pz + q'z  with  P = 2 blkdiag((Q (+) diag(Qs))^(N+1), R^N, dR^N),
 *                              q = 2 [qlin_0 .. qlin_N (state part), 0, 0]
 *   s.t. x_0 = x0,  x_{k+1} = A_k x_k + B_k u_k,  du_0 = u_0 - u_prev,  du_k = u_k - u_{k-1}
 *        C_{k,r} . x_k + sign_r * s_k[slack_r] <= h_{k,r}   (k = 1..N, r < mc; slack_r = -1: none)
 *        u_lb <= u_k <= u_ub   (rows ordered [u_i <= ub_i; -u_i <= -lb_i] per input, per stage)
 *
 * which is exactly the reference-form QP of PlannerLPV (LPV_Planner.py:279-475) for
 * nx=9, ns=3, nu=2 (cost :382-427, equalities :429-475, rows :251-380).  Rows with an
 * infinite bound are inactive.  Solved in condensed form (x eliminated; H = G'WG built
 * on MFMA) by a Mehrotra interior-point method, one wavefront per agent.
 * ---------------------------------------------------------------------- */
typedef struct {
    int nx, nu, N, ns, mc; /* state, input, horizon, slacks per stage, state rows per stage */
    int batch;             /* number of agents */
} cmpc_mpc_dims;

typedef struct { /* batch-shared (always HOST pointers; copied into the launch) */
    const double* Q;      /* nx*nx */
    const double* R;      /* nu*nu */
    const double* dR;     /* nu*nu */
    const double* Qs;     /* ns (diagonal slack weights, > 0) */
    const double* u_ub;   /* nu (+inf allowed) */
    const double* u_lb;   /* nu (-inf allowed) */
    const int* row_slack; /* mc: slack index used by row r, or -1 */
    const int* row_sign;  /* mc: +1 / -1 coefficient of that slack */
} cmpc_mpc_weights;

typedef struct { /* per-agent, batch-major */
    const double* A;      /* batch x N x nx x nx */
    const double* B;      /* batch x N x nx x nu */
    const double* x0;     /* batch x nx */
    const double* u_prev; /* batch x nu */
    const double* qlin;   /* batch x (N+1) x nx */
    const double* C;      /* batch x N x mc x nx   (stage k = 1..N) */
    const double* h;      /* batch x N x mc */
} cmpc_mpc_data;

typedef struct {
    double* z;    /* batch x nz,  nz = (nx+ns)(N+1) + 2 nu N  (reference layout) */
    double* kkt;  /* batch: final scaled KKT residual (may be NULL) */
    int* iters;   /* batch (may be NULL) */
    int* status;  /* batch: CMPC_SOLVED ... (may be NULL) */
} cmpc_mpc_out;

int cmpc_solve_mpc_batch(cmpc_ctx* ctx, const cmpc_mpc_dims* dims, const cmpc_mpc_weights* w,
                         const cmpc_mpc_data* host_in, const cmpc_mpc_out* host_out,
                         const cmpc_opts* opts);
int cmpc_solve_mpc_batch_dev(cmpc_ctx* ctx, const cmpc_mpc_dims* dims, const cmpc_mpc_weights* w,
                             const cmpc_mpc_data* dev_in, const cmpc_mpc_out* dev_out,
                             const cmpc_opts* opts, void* hip_stream);

/* The solver a structured batch would run, and how many of its workgroups share a CU — host only
 * (no context, no device).  Every solver uses more than 256 VGPRs + AGPRs per lane, so one
 * wavefront per SIMD (4 workgroups per CU at most); the LDS image then decides: wg_per_cu =
 * min(4, 160 KB / lds_bytes).  The lane-per-agent solver packs 32 agents per workgroup.  Errors as
 * cmpc_solve_mpc_batch (CMPC_ERR_UNSUPPORTED, CMPC_ERR_ARG). */
#define CMPC_SOLVER_CONDENSED_V3 1 /* specialised condensed kernel (mpc_ipm3: PlannerLPV row pattern) */
#define CMPC_SOLVER_CONDENSED 2    /* generic condensed kernel */
#define CMPC_SOLVER_RICCATI 3      /* stage-wise Riccati kernel (long horizons, fp32 path) */
#define CMPC_SOLVER_LANE 4         /* lane-per-agent stage-wise kernel */
typedef struct {
    int solver;        /* CMPC_SOLVER_* */
    int lds_bytes;     /* dynamic LDS per workgroup */
    int wg_per_cu;     /* workgroups resident per CU */
    int agents_per_wg; /* 1, or 32 (lane solver) */
    int waves_per_agent;   /* wavefronts of one agent's workgroup: 1; 4 for the stage-wise Riccati kernel's latency
                              mode (an LDS image over half a CU, the PlannerLPV agent at the reference's N = 125:
                              the agent's workgroup gets all four SIMDs of its CU; CMPC_FLAG_ONE_WAVE keeps one);
                              (2: the condensed kernel's CMPC_FLAG_TWO_WAVES mode of a fused double-integrator round,
                              cmpc_di_solve_dev, which the plan of a structured batch does not describe) */
    /* The rescue policy (CMPC_FLAG_RESCUE [| CMPC_FLAG_POLISH]) adds launches the fields above do not
     * describe: the polish kernel (before the Riccati hand-over and after the Riccati passes; one
     * 256-thread workgroup per agent, agents without a flag return at once) and two Riccati passes.
     * polish_lds_bytes: the polish workgroup's LDS (0 when the polish does not run); polish_max_active:
     * the largest active set it polishes (kPolishMaxActive = 96, lowered in steps of 8 until the image
     * fits 160 KB; larger active sets keep the interior-point result) */
    int polish_lds_bytes;
    int polish_max_active;
} cmpc_plan_info;
int cmpc_plan_mpc(const cmpc_mpc_dims* dims, const cmpc_mpc_weights* w, const cmpc_opts* opts,
                  cmpc_plan_info* out);

/* ------------------------------------------------------------------------
 * Reference-semantics LPV batch: one call = PlannerLPV.solve for every agent
 * (LPV_Planner.py:115-182) with the reference's exact quirks (lagged plane and
 * weight indexing, u not shifted, ey half-width from the previous prediction's s,
 * vx < 0.2 branch).  n_s = 9 states [vx vy wz ey epsi theta s X Y], 3 slacks,
 * 2 inputs [delta a].
 * ---------------------------------------------------------------------- */
#define CMPC_MAX_SEG 32

typedef struct {
    double lf, lr, m, I, Cf, Cr, mu;                   /* model_param (config/base_class.py:20-28) */
    double vx_ref, min_dist, max_vel, min_vel;         /* sys_lim (config/base_class.py:30-41) */
    double max_rs, max_ls, max_ac, max_dc;
    double dt, wq;                                     /* sample time, coverage weight */
    double Q[81], Qs[3], R[4], dR[4];                  /* gains (scripts/config_files/config_LPV.py:6-11) */
} cmpc_lpv_params;

typedef struct {     /* one lane of Map.PointAndTangent (track_initialization.py:220-300) */
    int nseg;        /* rows */
    const double* s0;         /* nseg: cumulative s at segment start (column 3) */
    const double* len;        /* nseg: segment length (column 4) */
    const double* curv;       /* nseg: signed curvature (column 5) */
    const double* half_width; /* nseg: Map.halfWidth */
} cmpc_track;

typedef struct {
    int batch, N, nb;  /* agents, horizon, neighbours per agent (same for all agents) */
    int last_rows;     /* rows of Last_xPredicted: N+1 at the first step, N afterwards */
} cmpc_lpv_dims;

typedef struct {   /* per-agent, batch-major */
    const double* x0;       /* batch x 9 */
    const double* x_last;   /* batch x last_rows x 9   (Last_xPredicted) */
    const double* u_last;   /* batch x N x 2           (uPred, not shifted) */
    const double* u_old;    /* batch x 2               ([OldSteering, OldAccelera]) */
    const double* x_agents; /* batch x (N+1) x nb x 2  (neighbour X,Y; NULL => planes 0, weights 1) */
    const double* pose;     /* batch x (N+1) x 2       (own previous X,Y) */
} cmpc_lpv_data;

typedef struct {
    double* z;       /* batch x nz (nz = 12(N+1) + 4N) */
    double* planes;  /* batch x N x 3 x nb (may be NULL) — compute_plane.py layout */
    double* kkt;     /* may be NULL */
    int* iters;      /* may be NULL */
    int* status;     /* may be NULL */
} cmpc_lpv_out;

int cmpc_solve_lpv_batch(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* track,
                         const cmpc_lpv_dims* dims, const cmpc_lpv_data* host_in,
                         const cmpc_lpv_out* host_out, const cmpc_opts* opts);
int cmpc_solve_lpv_batch_dev(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* track,
                             const cmpc_lpv_dims* dims, const cmpc_lpv_data* dev_in,
                             const cmpc_lpv_out* dev_out, const cmpc_opts* opts, void* hip_stream);

/* The LPV builder alone, DEVICE pointers: the structured agent-QP that
 * cmpc_solve_lpv_batch_dev hands its solver, for hosts that inspect or extend it before
 * cmpc_solve_mpc_batch_dev.  _EstimateABC (LPV_Planner.py:477-591: A_k = I + dt A_c, B_k = dt B_c
 * at the scheduling point of Last_xPredicted row k and uPred row k, curvature / half-width by
 * track-segment lookup misc.py:78-126), compute_hyperplane (compute_plane.py:41-68) and
 * compute_weights (misc.py:10-18) feed the rows (:251-380) and the linear cost (:382-427):
 *   A batch x N x 9 x 9, B batch x N x 9 x 2, qlin batch x (N+1) x 9, C batch x N x (4+nb) x 9,
 *   h batch x N x (4+nb), planes batch x N x 3 x nb (may be NULL), err batch (1: s of the
 *   previous prediction lies on no track segment — the reference raises there, misc.py:97). */
typedef struct {
    double *A, *B, *qlin, *C, *h, *planes;
    int* err;
} cmpc_lpv_build_out;

int cmpc_lpv_build_dev(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* track,
                       const cmpc_lpv_dims* dims, const cmpc_lpv_data* dev_in, const cmpc_lpv_build_out* dev_out,
                       void* hip_stream);

/* ------------------------------------------------------------------------
 * Synthetic agent family of BASELINE.json configs 1-5 (no reference counterpart:
 * the reference's model is the 9-state LPV bicycle; BASELINE fixes a double
 * integrator).  State [p (dim) | v (dim)], input a (dim), dim = 2 (nx=4, nu=2) or
 * 3 (nx=6, nu=3); 3 slacks; rows per stage mirror PlannerLPV's
 * (LPV_Planner.py:279-380) with v_x for vx, p_y - lane for ey and (p_x, p_y) for
 * (X, Y).  Per consensus round: _build rebuilds C, h, qlin of every local agent
 * from the previous round's exchanged trajectories (DEVICE pointers); _advance
 * applies the round update of LPV_HP_N_main.py:106-117 (x0 <- x_1,
 * u_prev <- u_0, trajectory <- predicted positions) and writes this rank's rows
 * of the exchange buffer.
 * ---------------------------------------------------------------------- */
typedef struct {
    int dim;                                   /* 2 or 3 */
    double v_ref, q_v, q_lane, hw, min_vel, max_vel, min_dist, wq;
} cmpc_di_params;

typedef struct {
    int batch, N, nb;   /* local agents, horizon, neighbours per agent */
    int self_offset;    /* global index of local agent 0 in traj_all */
} cmpc_di_dims;

int cmpc_di_build_dev(cmpc_ctx* ctx, const cmpc_di_params* prm, const cmpc_di_dims* dims,
                      const int* nbr /* batch x nb, global agent indices */,
                      const double* lane /* batch */,
                      const double* traj_all /* n_total x (N+1) x 2 */,
                      double* qlin /* batch x (N+1) x nx */, double* C /* batch x N x (4+nb) x nx */,
                      double* h /* batch x N x (4+nb) */, void* hip_stream);
/* Fused build + solve of one round (LPV_HP_N_main.py:96-117, build and solve of every agent):
 * where the v3 one-wave kernel covers the problem, each agent's rows and linear cost are built
 * from traj_all straight into the solver's LDS (bit-identical to cmpc_di_build_dev) — qlin / C
 * / h of `data` are then neither written nor read; otherwise this is cmpc_di_build_dev into
 * data->qlin / C / h (written despite the const) followed by cmpc_solve_mpc_batch_dev.
 * dims must describe the same agents: batch and N equal, nx = 2 dim, nu = dim, mc = 4 + nb. */
int cmpc_di_solve_dev(cmpc_ctx* ctx, const cmpc_di_params* prm, const cmpc_di_dims* ddims, const int* nbr,
                      const double* lane, const double* traj_all, const cmpc_mpc_dims* dims,
                      const cmpc_mpc_weights* w, const cmpc_mpc_data* data, const cmpc_mpc_out* out,
                      const cmpc_opts* opts, void* hip_stream);
int cmpc_di_advance_dev(cmpc_ctx* ctx, const cmpc_di_params* prm, const cmpc_di_dims* dims,
                        const double* z /* batch x nz */, double* x0 /* batch x nx */,
                        double* u_prev /* batch x nu */, double* traj_local /* batch x (N+1) x 2 */,
                        void* hip_stream);

/* Device-resident LPV consensus round (LPV_HP_N_main.py:96-117), DEVICE pointers, dims =
 * {batch, N, nb, self_offset} of the cmpc_di_dims struct:
 *   cmpc_lpv_gather_dev:  x_agents (batch x (N+1) x nb x 2) <- traj_all rows nbr[b][j] and pose
 *     (batch x (N+1) x 2) <- traj_all row self_offset + b — agents[:, ns[i], :] / agents[:, i, :]
 *     (:99-104); traj_all is n_total x (N+1) x 2, nbr batch x nb global agent indices;
 *   cmpc_solve_lpv_batch_dev on those buffers;
 *   cmpc_lpv_advance_dev: from z (reference layout): x0 <- xPred[1], x_last <- xPred[1:] written
 *     DENSE as batch x N x 9 (last_rows = N from the second round on, :115), u_last <- uPred
 *     (batch x N x 2, not shifted), u_old <- uPred[0] (:179-180), traj_local (batch x (N+1) x 2)
 *     <- xPred[:, X, Y] (:117); status (may be NULL) / infeasible (may be NULL, DEVICE int): the
 *     count of agents the reference calls infeasible (status not in {1, 2, -2}, LPV_Planner.py:243-249)
 *     is added to *infeasible; an agent whose z is not finite is not advanced (no NaN is exchanged);
 *   then the all-gather of traj_local into traj_all (cmpc_allgather_trajectories or torch). */
int cmpc_lpv_gather_dev(cmpc_ctx* ctx, const cmpc_di_dims* dims, const int* nbr, const double* traj_all,
                        double* x_agents, double* pose, void* hip_stream);
int cmpc_lpv_advance_dev(cmpc_ctx* ctx, const cmpc_di_dims* dims, const double* z, double* x0, double* x_last,
                         double* u_last, double* u_old, double* traj_local, const int* status, int* infeasible,
                         void* hip_stream);

/* ------------------------------------------------------------------------
 * Consensus rounds behind a handle (LPV_HP_N_main.py:96-117; the one-process-per-agent ROS
 * variant ROS/src/planner_experiments/src/LPV_ROS_main.py:66-77,124-150), for hosts without
 * torch or device memory of their own (MATLAB through the MEX gateway, plain C).  The handle
 * owns every device buffer of this rank's agents and the node-global exchange buffer; a round
 * is gather -> cmpc_solve_lpv_batch_dev -> cmpc_lpv_advance_dev -> exchange, all on the
 * context's stream, so consecutive rounds never touch the host.
 *
 * Sharding: this rank holds agents [self_offset, self_offset + batch) of n_total.  The exchange
 * of a round is the identity when batch == n_total; otherwise an RCCL all-gather over the
 * context's communicator (cmpc_comm_init; ranks hold equal contiguous shards in rank order),
 * or — CMPC_ROUNDS_HOST_EXCHANGE — the host's: after cmpc_lpv_rounds_step the host reads this
 * rank's positions (cmpc_lpv_rounds_get_traj), exchanges them its own way (MPI, sockets) and
 * hands the gathered buffer back (cmpc_lpv_rounds_set_traj) before the next step.
 *
 * Failure semantics (LPV_Planner.py:243-249, LPV_HP_N_main.py:102-111): an agent is
 * infeasible when its status is not in {1, 2, -2}; the reference quits the experiment there.
 * cmpc_lpv_rounds_step counts infeasible agents per round on the device and stops after the
 * first round that has any (rounds_done < rounds).  Sharded over RCCL, the count is the
 * node's (cmpc_comm_sum_i32 over the ranks), so every rank stops in the same round; with
 * CMPC_ROUNDS_HOST_EXCHANGE (one round per step) *infeasible is this rank's count and the
 * host combines them as it exchanges positions.  An agent whose solution is not finite
 * (track lookup failed, the reference raises) keeps its previous state and trajectory, so no
 * NaN reaches a neighbour.
 * ---------------------------------------------------------------------- */
typedef struct cmpc_lpv_rounds cmpc_lpv_rounds;

#define CMPC_ROUNDS_HOST_EXCHANGE 1  /* the host exchanges positions between steps */
#define CMPC_ROUNDS_NO_HALT 2        /* run all requested rounds even after an infeasible agent */

typedef struct {
    int n_total;      /* agents over all ranks */
    int batch;        /* agents of this rank */
    int self_offset;  /* global index of this rank's agent 0 */
    int N, nb;        /* horizon, neighbours per agent */
    int flags;        /* CMPC_ROUNDS_* */
} cmpc_lpv_rounds_dims;

typedef struct {   /* HOST pointers, this rank's agents, batch-major (copied at create) */
    const double* x0;      /* batch x 9 */
    const double* x_last;  /* batch x (N+1) x 9: the first round's Last_xPredicted */
    const double* u_last;  /* batch x N x 2 */
    const double* u_old;   /* batch x 2, or NULL (zeros: PlannerLPV's initial OldSteering/OldAccelera) */
    const int* nbr;        /* batch x nb global agent indices (the reference: all other agents) */
    const double* traj;    /* n_total x (N+1) x 2 initial exchange buffer (the reference's `agents`);
                              NULL: only valid when batch == n_total, taken from x_last[:, :, 7:9] */
} cmpc_lpv_rounds_init;

typedef struct {   /* HOST pointers (any may be NULL): the latest round of this rank's agents */
    double* z;       /* batch x nz (nz = 12(N+1) + 4N) */
    double* kkt;     /* batch */
    int* iters;      /* batch */
    int* status;     /* batch */
    double* x0;      /* batch x 9: the next round's initial states */
    double* planes;  /* batch x N x 3 x nb */
} cmpc_lpv_rounds_out;

int cmpc_lpv_rounds_create(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* track,
                           const cmpc_lpv_rounds_dims* dims, const cmpc_lpv_rounds_init* init,
                           const cmpc_opts* opts, cmpc_lpv_rounds** out);
/* Runs up to `rounds` rounds; *rounds_done (may be NULL) receives the number completed and
 * *infeasible (may be NULL) the infeasible-agent count of the last one.  Synchronises the host. */
int cmpc_lpv_rounds_step(cmpc_lpv_rounds* h, int rounds, int* rounds_done, int* infeasible);
int cmpc_lpv_rounds_read(cmpc_lpv_rounds* h, const cmpc_lpv_rounds_out* host_out);
/* Host exchange: this rank's predicted positions (batch x (N+1) x 2) / the gathered buffer
 * (n_total x (N+1) x 2, rank order). */
int cmpc_lpv_rounds_get_traj(cmpc_lpv_rounds* h, double* traj_local);
int cmpc_lpv_rounds_set_traj(cmpc_lpv_rounds* h, const double* traj_all);
/* Destroy every handle of a context before cmpc_destroy(ctx). */
int cmpc_lpv_rounds_destroy(cmpc_lpv_rounds* h);


/* ------------------------------------------------------------------------
 * Dense standard-form QP batch with MATLAB quadprog semantics (the MEX drop-in
 * for quadprog(H,f,A,b,Aeq,beq,lb,ub) as YALMIP calls it, callquadprog.m:63-69,
 * and the generic back end of the osqp_solve_qp adapter, LPV_Planner.py:192-249):
 *
 *   min 1/2 x'Hx + f'x   s.t.  A x <= b,  Aeq x = beq,  lb <= x <= ub
 *
 * HOST pointers, batch-major (problem p's block contiguous).  H n x n (its symmetric
 * part is used), A m_ineq x n, Aeq m_eq x n, row-major unless col_major (MATLAB
 * layout).  A/b, Aeq/beq, lb, ub may be NULL (absent); +-inf bounds are inactive;
 * all-zero constraint rows are dropped (or make the problem infeasible).
 * exitflag: CMPC_QP_CONVERGED 1, CMPC_QP_MAXITER 0, CMPC_QP_INFEASIBLE -2,
 * CMPC_QP_UNBOUNDED -3, CMPC_QP_NONCONVEX -6 (quadprog's codes).
 * ---------------------------------------------------------------------- */
#define CMPC_QP_CONVERGED 1
#define CMPC_QP_MAXITER 0
#define CMPC_QP_INFEASIBLE (-2)
#define CMPC_QP_UNBOUNDED (-3)
#define CMPC_QP_NONCONVEX (-6)

typedef struct {
    int n, m_ineq, m_eq, batch;
    int col_major;
} cmpc_qp_dims;

typedef struct {
    const double *H, *f, *A, *b, *Aeq, *beq, *lb, *ub;
} cmpc_qp_data;

typedef struct {
    double* x;               /* batch x n */
    double* fval;            /* batch (may be NULL) */
    int* exitflag;           /* batch (may be NULL) */
    int* iters;              /* batch (may be NULL) */
    double* lambda_ineqlin;  /* batch x m_ineq (may be NULL) */
    double* lambda_eqlin;    /* batch x m_eq (may be NULL) */
    double* lambda_lower;    /* batch x n (may be NULL) */
    double* lambda_upper;    /* batch x n (may be NULL) */
    double* residual;        /* batch: final scaled KKT merit (may be NULL) */
} cmpc_qp_out;

int cmpc_solve_qp_batch(cmpc_ctx* ctx, const cmpc_qp_dims* dims, const cmpc_qp_data* host_in,
                        const cmpc_qp_out* host_out, const cmpc_opts* opts);

/* ------------------------------------------------------------------------
 * OCD coupling-dual round (planner/scripts/NL_EU_N_main.py:119-162; ROS variant
 * ROS/src/planner_experiments/src/OCD_ROS_main.py:200-239), DEVICE pointers:
 *   lam[b, s, k-1] += alpha * (dth - ||p_g(k) - p_j(k)||),  g = self_offset + b,
 *   j = nbr[b, s], for k = 1..N and only when g < j (the reference fills i < j);
 *   p from traj_all (n_total x (N+1) x 2).  alpha = 0.25 in the reference
 *   (config/NL/config.py:5-8), dth its safety distance.
 * cmpc_ocd_converged_dev: close[b] = numpy allclose(x_old[b], x_pred[b], atol, rtol)
 *   over `per` values per agent (the reference's convergence test, :143-162).
 * ---------------------------------------------------------------------- */
typedef struct {
    int batch, N, nb, self_offset;
} cmpc_ocd_dims;

int cmpc_ocd_update_dev(cmpc_ctx* ctx, const cmpc_ocd_dims* dims, double alpha, double dth, const int* nbr,
                        const double* traj_all, double* lam, void* hip_stream);
int cmpc_ocd_converged_dev(cmpc_ctx* ctx, int batch, int per, double atol, double rtol, const double* x_old,
                           const double* x_pred, int* close, void* hip_stream);

/* ----------------------------------------------------------------------
 * Multi-GPU exchange (RCCL over xGMI).  One process per GPU, one
 * context per process.  Replaces the per-round exchange of predicted trajectories —
 * the ROS topics of ROS/src/planner_experiments/src/LPV_ROS_main.py:66-77 (publish)
 * and :124-150 (subscribe), the in-process np.swapaxes of LPV_HP_N_main.py:117 —
 * for hosts that shard agents without torch (a MATLAB / C host).
 *
 *   cmpc_comm_id:   rank 0 creates the communicator id; the host hands its
 *                   CMPC_COMM_ID_BYTES bytes to every rank (MPI, a file, a socket).
 *   cmpc_comm_init: every rank joins (collective; blocks until all ranks joined).
 *   cmpc_allgather_trajectories: traj_all (nranks*count doubles, DEVICE) receives every
 *                   rank's traj_local (count doubles, DEVICE) in rank order; stream-ordered
 *                   (hip_stream as void*, 0 = default).  For the position exchange of a
 *                   round, count = local agents * (N+1) * 2.
 *   cmpc_comm_sum_i32: buf (count int32, DEVICE) <- its sum over every rank of the
 *                   communicator, in place, stream-ordered (one RCCL all-reduce).  The
 *                   rounds use it for the halt decision: the reference's loop stops for
 *                   every agent at once when one is infeasible (LPV_HP_N_main.py:102-111),
 *                   so every rank must see the node's infeasible count, not its own.
 *                   Without a communicator (one rank) it leaves buf unchanged.
 *   cmpc_comm_destroy: leaves the communicator (cmpc_destroy does it too).
 * ---------------------------------------------------------------------- */
#define CMPC_COMM_ID_BYTES 128
int cmpc_comm_id(unsigned char id[CMPC_COMM_ID_BYTES]);
int cmpc_comm_init(cmpc_ctx* ctx, int nranks, int rank, const unsigned char id[CMPC_COMM_ID_BYTES]);
int cmpc_allgather_trajectories(cmpc_ctx* ctx, const double* traj_local, double* traj_all, unsigned long long count,
                                void* hip_stream);
int cmpc_comm_sum_i32(cmpc_ctx* ctx, int* buf, unsigned long long count, void* hip_stream);
int cmpc_comm_destroy(cmpc_ctx* ctx);

/* Device self-test of the f64 MFMA fragment mapping used by the solver
 * (D = A*B for one 16x16x4 tile, A,B host 16x4 / 4x16 row-major, D host 16x16). */
int cmpc_selftest_mfma(cmpc_ctx* ctx, const double* A, const double* B, double* D);

#ifdef __cplusplus
}
#endif
#endif /* CMPC_H */
