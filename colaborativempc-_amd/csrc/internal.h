// Internal declarations shared by the HIP translation units of libcmpc.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "cmpc.h"

namespace cmpc {

constexpr int kWave = 64;

// Batch-shared constants of the structured agent QP.  Passed BY VALUE as a
// kernel argument (lands in the scalar constant path; no per-call memcpy, so a
// launch is graph-capturable).
struct MpcConst {
    int nx, nu, N, ns, mc;
    int n;      // condensed variables N*nu
    int ms;     // state rows N*mc
    int m;      // all rows ms + 2*nu*N
    int nxp;    // nx rounded up to the MFMA K granularity (4)
    int npad;   // n rounded up to 16 (MFMA tile)
    int ldk;    // leading dimension of the LDS Hessian (odd)
    int max_iter;
    int riccati;  // 1: stage-wise Riccati kernel (fp64, N*nu > 64 or CMPC_FLAG_RICCATI)
    int rescue;   // 1: CMPC_FLAG_RESCUE on a condensed solve (Riccati re-solve of broken-down agents); 2: its
                  // cold second pass; 3: the fp32 path's fp64 pass over the agents short of tol (mpc_launch)
    int lpv;      // 1: data made by lpv_build.hip with Q diagonal (the v3 kernel's LS layout applies); 2: and Q zero
                  // on states 1, 2, 5, 6 (the LS kernel's L5 contraction, the reference's config_LPV.py:7)
    int finish;   // 1: CMPC_FLAG_FINISH (rescue also continues breakdowns at the rounding floor)
    int lane;     // lane-per-agent kernel (mpc_lane.hip): 1 fp64 (CMPC_FLAG_LANE), 2 mixed fp32 (CMPC_FLAG_FP32 | LANE,
                  // or CMPC_FLAG_FP32 on dimensions without an fp32 Riccati instantiation)
    int f32;      // 1: CMPC_FLAG_FP32 on the stage-wise Riccati kernel (Cfg::F32; riccati = 1 as well)
    int polish;   // 1: CMPC_FLAG_POLISH (with rescue): active-set polish of breakdowns at the rounding floor
    int waves;    // fused DS instantiation of the v3 kernel: wavefronts per agent (0, 1: one; 2: CMPC_FLAG_TWO_WAVES)
    unsigned long long ws_stride;  // doubles of MpcPtrs::ws per agent (set by mpc_launch; 0: no scratch)
    double tol;
    double qs_max;  // max(1, 2*max(Qs)) — slack residual scale
    double R[CMPC_MAX_NU * CMPC_MAX_NU];
    double dR[CMPC_MAX_NU * CMPC_MAX_NU];
    double Qs[CMPC_MAX_NS];
    double u_ub[CMPC_MAX_NU];
    double u_lb[CMPC_MAX_NU];
    int row_slack[CMPC_MAX_MC];
    int row_sign[CMPC_MAX_MC];
    // last: a kernel that copies the struct to LDS (mpc_riccati.hip) copies only its first nx * nx
    // entries (mpc_const_used_doubles), 864 B less at nx = 6
    double Q[CMPC_MAX_NX * CMPC_MAX_NX];
};

// doubles of an MpcConst up to the last Q entry an nx x nx problem reads
__host__ __device__ inline int mpc_const_used_doubles(const MpcConst& c) {
    return (int)((offsetof(MpcConst, Q) + sizeof(double) * (size_t)c.nx * c.nx + 7) / 8);
}

struct DiConst {
    int N, nb, nx, nu, ns, dim, self_offset;
    double v_ref, q_v, q_lane, hw, min_vel, max_vel, min_dist, wq;
};

// Fused double-integrator round (cmpc_di_solve_dev): when `on`, the v3 kernel builds each
// agent's stage rows and linear cost from the exchanged trajectories straight into LDS
// (di_rows.h, the arithmetic of di_build_kernel) instead of reading qlin / C / h.
struct DiFuse {
    const int* nbr;
    const double* lane;
    const double* traj_all;
    DiConst c;
    int on;
};

struct MpcPtrs {
    const double* A;
    const double* B;
    const double* x0;
    const double* up;
    const double* p;
    const double* C;
    const double* h;
    double* z;
    double* kkt;
    int* iters;
    int* status;
    unsigned long long* stamps;  // optional: batch x kStampSlots per-section s_memtime counts (v3 kernel)
    double* ws;                  // device scratch, batch x mpc_ws_doubles(c) (Riccati kernel; else unused)
    DiFuse fuse;                 // fused row build (v3 kernel only; on = 0 elsewhere)
    const int* order;            // optional launch order (Riccati kernel: workgroup i solves agent order[i])
    // optional device scratch of batch + 1 ints for the polish launch's compacted agent list (mpc_polish.hip):
    // without it every workgroup maps to its own agent and the flagged ones queue behind each other on a CU
    int* plist = nullptr;
};

// Interior-point safeguards shared by both solver kernels and the C oracle (oracle/cmpc_oracle.c).
//  * kNbhdGamma: after each step every active pair keeps t_r lam_r >= gamma * mu (wide
//    neighbourhood, step backtracked by 0.8).  Without it Mehrotra's corrector can cycle on
//    degenerate collision rows: two rows alternately block the step and mu stalls near 1e-5.
//  * kStallIters: once the merit max(res, 1e4 mu) is below 1e3 tol, that many iterations
//    without a new best stop the solve (rounding floor); the best iterate is returned.
// diagnostic stamps of the v3 kernel: batch x kStampSlots uint64 (last slot = iterations)
constexpr int kStampSlots = 16;
constexpr double kNbhdGamma = 0.01;
constexpr int kMaxBacktrack = 30;
constexpr int kStallIters = 3;
// Starting point: t_r = max(w_r - g_r(U=0), kT0Floor), lambda_r = 1.  Floor 0.5 rather than 1:
// over the first 100 cfg3 rounds (1024 agents, tools/ipm_lab.py) the sum over rounds of the
// slowest agent's iteration count drops 1951 -> 1801 (the kernel time follows the slowest
// agent) with no max-iteration agent (floors 0.4 and 0.7 each had one); mean 9.39 -> 9.32.
constexpr double kT0Floor = 0.5;
// ... for the condensed kernels (mpc_ipm3, mpc_ipm) since round 5: 0.1.  Measured again on the current
// method (tools/ipm_lab.py, 100 cfg3 rounds of 1024 agents): the sum of the per-round slowest agent's
// iterations 1801 -> 1621 (floors 0.04 .. 0.15 all give 1566 .. 1621; 0.02 and below fail agents), mean
// 9.32 -> 9.13; reference-model rounds (tools/lpv_lab.py, 22 rounds of 1023 agents, rescue policy): 553 ->
// 500, max 45 -> 38, mean 14.5 -> 13.6.  The stage-wise kernels keep 0.5: on cfg5 (N = 50, Riccati) the
// total iterations, which set that launch, rose 2 % with 0.1.
constexpr double kT0FloorCond = 0.1;
// Mehrotra's centring parameter sigma = (mu_aff / mu)^e: e = 3 in the stage-wise kernels, e = 2 in the condensed
// ones since round 5 (tools/ipm_lab.py, 100 cfg3 rounds: sum of the per-round slowest agent's iterations 1621 ->
// 1580; tools/lpv_lab.py, 22 reference-model rounds: 500 -> 490 and 23 % fewer rounding-floor exits, 718 -> 554;
// on cfg5's Riccati solves e = 2 cost 1.5 % more iterations, so those keep 3; a warm Riccati continuation of a
// condensed solve, CMPC_FLAG_RESCUE, keeps the e = 2 of the solve it continues).
// Stall guard: after an iteration whose step was below kShortStep, the corrector's centring
// parameter is at least kSigmaMin.  On the BASELINE cfg5 population (N=50, nx=6 nu=3) about 1
// agent in 10^4 otherwise stalls at steps ~1e-3, blocked by a terminal collision row, and runs
// to max_iter (tools/cfg5_diag.py: 21 such agents in 10 rounds; with the guard 0, all at most
// 43 iterations); the cfg3 rounds and every captured reference QP never trigger it (identical
// iterates, tools/ipm_lab.py).
constexpr double kShortStep = 0.02;

// Degenerate endpoints (CMPC_FLAG_POLISH).  A solve that converges (merit < tol) with a weakly active row
// — t_r and lambda_r both of order sqrt(mu) instead of one of them ~0 — is fixed only to ~sqrt(mu) ~ 3e-7
// along that row's direction: on bench.py's lpv_rounds population the GPU and the C restatement, each at
// its own ulp-different endpoint, land 5e-7 .. 1e-6 apart there (tools/lpv_margin.py, round 5: every
// such agent had one row, the last stage's input bound, with min(t, lambda) ~ 2-4e-7 and the next row
// below 1e-11).  Those agents join the polish launch (rescue image flag 2 with their merit): the active
// set's equality-constrained QP gives the optimum to ~1e-13 in KKT, and it replaces the endpoint only
// when its merit is lower.  The threshold sits orders of magnitude from both populations.
constexpr double kPolishDegenerate = 1e-9;
constexpr double kSigmaMin = 0.5;
enum { kStopMaxIter = 0, kStopConverged = 1, kStopBreakdown = 2, kStopStalled = 3, kStopNonFinite = 4 };

// Per-agent status of a solve that ended without meeting the tolerance (best merit best_m).
__host__ __device__ inline int stop_status(int stop, double best_m, double tol) {
    if (best_m < 1e3 * tol) return CMPC_SOLVED_INACCURATE;
    return stop == kStopMaxIter ? CMPC_MAX_ITER_REACHED : CMPC_UNSOLVED;
}

constexpr size_t kMaxLdsBytes = 160 * 1024;

// Rescue hand-over (CMPC_FLAG_RESCUE).  A condensed kernel whose factorisation breaks down leaves
// its iterate at the start of the agent's scratch (MpcPtrs::ws + b * ws_stride):
//   [flag, iterations done, U (n), sig (N ns), t (m), lam (m)]   (rows in the oracle's order)
// and the Riccati rescue launch continues the same interior-point solve from it (double-double
// Newton solves near the solution) instead of starting cold; flag 0: no hand-over (cold start).
// oracle/cmpc_oracle.c restates it (newton 4).
__host__ __device__ inline size_t hand_doubles(const MpcConst& c) {
    return 2 + (size_t)c.n + (size_t)c.N * c.ns + 2 * (size_t)c.m;
}
__host__ __device__ inline size_t hand_t(const MpcConst& c) { return 2 + (size_t)c.n + (size_t)c.N * c.ns; }
// A continued (handed-over) solve without a new best iterate for kWarmStall iterations ends there
// (best iterate; CMPC_UNSOLVED above the rounding floor, which the cold second pass re-solves).
// Over 22 closed-loop rounds of bench.py's lpv_rounds population (tools/lpv_lab.py, the C
// restatement): no unsolved or max-iteration agent, 279 of 22 506 at the rounding floor (714 with
// the cold rescue alone); without it two continued solves ran to max_iter.  Every continued
// iteration runs in double-double: 3 (the kStallIters of the condensed solve) and 8 gave the same
// statuses in the lab, so the short one is kept.
constexpr int kWarmStall = 3;
// A breakdown whose best iterate is already at the rounding floor (merit < 1e3 tol, status 2) is
// handed over only with CMPC_FLAG_FINISH (MpcConst::finish): on bench.py's lpv_rounds population
// that finishes ~60 % of the status-2 agents (720 -> 284 of 20 460) at 112k instead of 178k
// agent-QP/s (every dd iteration of a continued solve costs ~1 ms at N = 30).
__host__ __device__ inline bool hand_over(int stop, double best_m, const MpcConst& c) {
    return stop == kStopBreakdown && (c.finish || !(best_m < 1e3 * c.tol));
}

// v3 kernel, fused double-integrator round: two wavefronts per agent (MpcConst::waves == 2)
bool mpc3_two_waves(const MpcConst& c, int batch);

// Active-set polish (mpc_polish.hip): agents whose rescue image carries flag 2.
size_t mpc_polish_lds_bytes(const MpcConst& c);
int mpc_polish_max_active(const MpcConst& c);  // the layout's active-set capacity (LDS-limited)
hipError_t mpc_polish_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s);
// Stage-wise Riccati kernel (mpc_riccati.hip): any horizon whose per-agent rows fit LDS.
size_t mpc_riccati_lds_bytes(const MpcConst& c);
bool mpc_riccati_f32_supported(const MpcConst& c);  // Cfg::F32 instantiations (BASELINE cfg5 dimensions)
bool mpc_riccati_mw(const MpcConst& c);             // the Riccati latency mode (four wavefronts per agent) applies
size_t mpc_riccati_ws_doubles(const MpcConst& c);
hipError_t mpc_riccati_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s);
// Lane-per-agent stage-wise kernel (mpc_lane.hip): the dimension sets it is instantiated for.
bool mpc_lane_supported(const MpcConst& c);
size_t mpc_lane_ws_doubles(const MpcConst& c);
hipError_t mpc_lane_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s);
// Device scratch (doubles per agent) the solver chosen for c needs in MpcPtrs::ws (0: none).
inline size_t mpc_ws_doubles(const MpcConst& c) {
    if (c.lane) return mpc_lane_ws_doubles(c);
    return (c.riccati || c.rescue) ? mpc_riccati_ws_doubles(c) : 0;
}

// Fills the derived fields of MpcConst; returns CMPC_OK or an error code with msg.
int mpc_prepare(const cmpc_mpc_dims* d, const cmpc_mpc_weights* w, const cmpc_opts* o,
                MpcConst* c, const char** msg);
size_t mpc_lds_bytes(const MpcConst& c);
// flags: CMPC_FLAG_GENERIC forces the generic kernel (diagnostics)
hipError_t mpc_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, int flags = 0);
// v3 kernels of mpc_ipm3.hip (PlannerLPV row pattern, N <= 32); false when none covers the problem.
bool mpc3_try_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* err);
// LDS bytes of the v3 instantiation mpc3_try_launch would run for c (0: none covers it)
size_t mpc3_lds_bytes(const MpcConst& c);
size_t mpc_lane_lds_bytes(const MpcConst& c);

// LPV reference-semantics builder (scheduling + planes + weights + rows).
struct LpvConst {
    int N, nb, last_rows, nseg, mc;
    double lf, lr, m, I, Cf, Cr, mu;
    double vx_ref, min_dist, max_vel, min_vel, max_rs, max_ls, max_ac, max_dc;
    double dt, wq, Q00;
    double s0[CMPC_MAX_SEG], len[CMPC_MAX_SEG], curv[CMPC_MAX_SEG], hw[CMPC_MAX_SEG];
    double track_len;
};

struct LpvPtrs {
    const double* x_last;
    const double* u_last;
    const double* x_agents;
    const double* pose;
    double* A;
    double* B;
    double* p;
    double* C;
    double* h;
    double* planes;
    int* err;  // per agent: 0 ok, 1 track lookup failed (reference raises)
};

hipError_t lpv_build_launch(const LpvConst& c, const LpvPtrs& p, int batch, hipStream_t s);
// Where the builder flagged agent b (track lookup failed, the reference raises): status[b] =
// CMPC_UNSOLVED (status may be null) and z[b, :] = NaN.
hipError_t lpv_mark_launch(const int* err, int* status, double* z, int nz, int batch, hipStream_t s);
// device-resident LPV round (lpv_round.hip): neighbour / own positions from the exchange buffer,
// and the round update from the solution
hipError_t lpv_gather_launch(int N, int nb, int self_offset, const int* nbr, const double* traj_all, double* x_agents,
                             double* pose, int batch, hipStream_t s);
// status / infeasible (both may be null): count the agents the reference calls infeasible
// (status not in {1, 2, -2}) into *infeasible; an agent with a non-finite z is not advanced
hipError_t lpv_advance_launch(int N, const double* z, double* x0, double* x_last, double* u_last, double* u_old,
                              double* traj_local, int batch, hipStream_t s, const int* status = nullptr,
                              int* infeasible = nullptr);

// Synthetic double-integrator family (bench workload).

struct DiPtrs {
    const int* nbr;
    const double* lane;
    const double* traj_all;
    double* qlin;
    double* C;
    double* h;
};

hipError_t di_build_launch(const DiConst& c, const DiPtrs& p, int batch, hipStream_t s);
hipError_t di_advance_launch(const DiConst& c, const double* z, double* x0, double* up, double* traj, int batch,
                             hipStream_t s);

hipError_t selftest_mfma_launch(const double* A, const double* B, double* D, hipStream_t s);

// OCD coupling-dual round (ocd.hip).
struct OcdConst {
    int batch, N, nb, self_offset;
    double alpha, dth;
};
hipError_t ocd_update_launch(const OcdConst& c, const int* nbr, const double* traj, double* lam, hipStream_t s);
hipError_t ocd_close_launch(int batch, int per, double atol, double rtol, const double* xo, const double* xp,
                            int* close, hipStream_t s);

// Dense standard-form QP batch (quadprog semantics), qp_dense.hip.
struct QpConst {
    int n, mi, me;   // variables, general inequality rows, equality rows
    int col_major;   // matrices A, Aeq given column-major (MATLAB)
    int max_iter, refine;
    double tol, reg; // tolerance; quasi-definite regularisation rho = delta
};

struct QpPtrs {
    const double *H, *f, *A, *b, *Aeq, *beq, *lb, *ub;  // batch-major; A/b, Aeq/beq, lb, ub may be null
    double *x, *fval, *lam_ineq, *lam_eq, *lam_lo, *lam_up, *merit;
    int *exitflag, *iters;
    double* ws;  // batch x qp_ws_doubles
};

size_t qp_ws_doubles(int n, int mi, int me);
hipError_t qp_launch(const QpConst& c, const QpPtrs& p, int batch, hipStream_t s);

}  // namespace cmpc
