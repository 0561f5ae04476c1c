// Synthetic double-integrator agent family (BASELINE configs 1-5): per consensus
// round, rebuild each agent's stage rows and linear cost from the trajectories
// exchanged in the previous round, with the reference's structure and quirks
// (planner/lib/plan_lib/distributedPlanner/LPV_Planner.py):
//   rows per stage k=1..N  [-v_x <= -min_vel ; v_x + s0 <= max_vel ;
//                           (p_y - lane) + s1 <= hw ; -(p_y - lane) + s1 <= hw ;
//                           a_i . p - s2 <= -d/2 - b_i  (i < nb) ]          (:279-380, :251-276)
//   planes from row k-1 of the previous trajectories, weights from row k     (:269-272, misc.py:10-18)
//   p_k = [-lane q_y on p_y, -v_ref q_v on v_x] + wq sum_i w_i a_i on p      (:382-427)
// plus the round advance of LPV_HP_N_main.py:106-117 (x0 <- x_1, u_prev <- u_0,
// exchanged positions <- predicted p_k).  Element-wise per (agent, stage).
#include <cmath>

#include "di_rows.h"
#include "internal.h"

namespace cmpc {

__global__ __launch_bounds__(kWave) void di_build_kernel(const DiConst c, const DiPtrs P) {
    const int b = blockIdx.x;
    const int N = c.N, nx = c.nx, mc = 4 + c.nb;
    const double lane = P.lane[b];
    const double* own = P.traj_all + (size_t)(c.self_offset + b) * (N + 1) * 2;
    const int* nbr = P.nbr + (size_t)b * c.nb;
    double* qlin = P.qlin + (size_t)b * (N + 1) * nx;
    double* C = P.C + (size_t)b * N * mc * nx;
    double* h = P.h + (size_t)b * N * mc;
    for (int k = threadIdx.x; k <= N; k += kWave) {
        const int h1 = k > 0 ? k - 1 : 0;
        di_stage_rows(c, nbr, lane, P.traj_all, own, k, qlin + (size_t)k * nx, C + (size_t)h1 * mc * nx,
                      h + (size_t)h1 * mc);
    }
}

// x0 <- x_1, u_prev <- u_0, traj <- predicted (p_x, p_y) for k = 0..N  (z in reference layout)
__global__ void di_advance_kernel(const DiConst c, const double* __restrict__ z, double* x0, double* up,
                                  double* traj, int batch) {
    const int b = blockIdx.x;
    const int N = c.N, nx = c.nx, nxe = nx + c.ns, nu = c.nu;
    const size_t nz = (size_t)nxe * (N + 1) + 2 * (size_t)nu * N;
    const double* zb = z + (size_t)b * nz;
    for (int k = threadIdx.x; k <= N; k += blockDim.x) {
        traj[((size_t)b * (N + 1) + k) * 2 + 0] = zb[k * nxe + 0];
        traj[((size_t)b * (N + 1) + k) * 2 + 1] = zb[k * nxe + 1];
    }
    if (threadIdx.x < nx) x0[(size_t)b * nx + threadIdx.x] = zb[nxe + threadIdx.x];
    if (threadIdx.x < nu) up[(size_t)b * nu + threadIdx.x] = zb[(size_t)nxe * (N + 1) + threadIdx.x];
}

hipError_t di_build_launch(const DiConst& c, const DiPtrs& p, int batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(di_build_kernel, dim3(batch), dim3(kWave), 0, s, c, p);
    return hipGetLastError();
}

hipError_t di_advance_launch(const DiConst& c, const double* z, double* x0, double* up, double* traj, int batch,
                             hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(di_advance_kernel, dim3(batch), dim3(kWave), 0, s, c, z, x0, up, traj, batch);
    return hipGetLastError();
}

}  // namespace cmpc
