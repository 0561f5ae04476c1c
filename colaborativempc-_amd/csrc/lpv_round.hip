// Device-resident LPV consensus round (LPV_HP_N_main.py:96-117) around cmpc_solve_lpv_batch_dev:
//   gather:  each agent's neighbour positions x_agents (N+1, nb, 2) and its own previous positions
//            `pose` (N+1, 2) from the node-global exchange buffer traj_all (n_total, N+1, 2) —
//            the reference's agents[:, ns[i], :] and agents[:, i, :] (:99-104)
//   advance: from the solution z (reference layout, LPV_Planner.py:164-178): x0 <- xPred[1],
//            Last_xPredicted <- xPred[1:] (N rows, :115), uPred <- u (not shifted, :114),
//            [OldSteering, OldAccelera] <- u_0 (:179-180), and this rank's rows of the exchange
//            buffer <- xPred[:, 7:9] (X, Y; :117)
// Pure data movement, one workgroup per agent.
#include "internal.h"

namespace cmpc {

namespace {
constexpr int kNs = 9, kNexp = 12, kNu = 2;  // states, states + slacks per stage, inputs

__global__ __launch_bounds__(kWave) void lpv_gather_kernel(int N, int nb, int self_offset, const int* __restrict__ nbr,
                                                           const double* __restrict__ traj_all, double* x_agents,
                                                           double* pose) {
    const int b = blockIdx.x;
    const size_t row = (size_t)(N + 1) * 2;
    const double* own = traj_all + (size_t)(self_offset + b) * row;
    for (int i = threadIdx.x; i < (int)row; i += kWave) pose[(size_t)b * row + i] = own[i];
    if (!x_agents) return;
    // x_agents[b][k][j][c] = traj_all[nbr[b][j]][k][c]
    const int per = (N + 1) * nb * 2;
    for (int i = threadIdx.x; i < per; i += kWave) {
        const int c = i & 1, j = (i >> 1) % nb, k = (i >> 1) / nb;
        x_agents[(size_t)b * per + i] = traj_all[(size_t)nbr[(size_t)b * nb + j] * row + (size_t)k * 2 + c];
    }
}

__global__ __launch_bounds__(kWave) void lpv_advance_kernel(int N, const double* __restrict__ z, double* x0,
                                                            double* x_last, double* u_last, double* u_old,
                                                            double* traj_local, const int* __restrict__ status,
                                                            int* infeasible) {
    const int b = blockIdx.x;
    const size_t nz = (size_t)kNexp * (N + 1) + 2 * (size_t)kNu * N;
    const double* zb = z + (size_t)b * nz;
    const double* up = zb + (size_t)kNexp * (N + 1);
    // the reference's feasibility rule (LPV_Planner.py:243-249): status in {1, 2, -2}
    if (status && infeasible && threadIdx.x == 0) {
        const int st = status[b];
        if (st != CMPC_SOLVED && st != CMPC_SOLVED_INACCURATE && st != CMPC_MAX_ITER_REACHED) atomicAdd(infeasible, 1);
    }
    // an agent without a finite solution (the builder's track lookup failed: the reference raises,
    // misc.py:97) keeps its state and its previous trajectory: no NaN reaches a neighbour
    bool bad = false;
    for (size_t i = threadIdx.x; i < nz; i += kWave) bad |= !isfinite(zb[i]);
    if (__any(bad)) return;
    for (int i = threadIdx.x; i < N * kNs; i += kWave) {  // xPred[1:], rows 1..N
        const int k = i / kNs + 1, s = i - (k - 1) * kNs;
        x_last[(size_t)b * N * kNs + i] = zb[(size_t)k * kNexp + s];  // dense (B, N, 9) from now on
    }
    if (threadIdx.x < kNs) x0[(size_t)b * kNs + threadIdx.x] = zb[kNexp + threadIdx.x];
    for (int i = threadIdx.x; i < N * kNu; i += kWave) u_last[(size_t)b * N * kNu + i] = up[i];
    if (threadIdx.x < kNu) u_old[(size_t)b * kNu + threadIdx.x] = up[threadIdx.x];
    for (int i = threadIdx.x; i < 2 * (N + 1); i += kWave) {
        const int k = i >> 1, c = i & 1;
        traj_local[(size_t)b * 2 * (N + 1) + i] = zb[(size_t)k * kNexp + 7 + c];
    }
}
}  // namespace

hipError_t lpv_gather_launch(int N, int nb, int self_offset, const int* nbr, const double* traj_all, double* x_agents,
                             double* pose, int batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(lpv_gather_kernel, dim3(batch), dim3(kWave), 0, s, N, nb, self_offset, nbr, traj_all,
                       x_agents, pose);
    return hipGetLastError();
}

hipError_t lpv_advance_launch(int N, const double* z, double* x0, double* x_last, double* u_last, double* u_old,
                              double* traj_local, int batch, hipStream_t s, const int* status, int* infeasible) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(lpv_advance_kernel, dim3(batch), dim3(kWave), 0, s, N, z, x0, x_last, u_last, u_old,
                       traj_local, status, infeasible);
    return hipGetLastError();
}

}  // namespace cmpc
