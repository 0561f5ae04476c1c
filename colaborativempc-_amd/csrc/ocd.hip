// OCD (optimality condition decomposition) coupling-dual round of the collaborative loop,
// reference planner/scripts/NL_EU_N_main.py:119-162 (ROS variant OCD_ROS_main.py:200-239):
//   cost[i,j,k-1] = D - ||p_i(k) - p_j(k)||   (eval_constraintEU, config/NL/config.py:19-23), i < j
//   lambda += alpha * cost                      (alpha = get_alpha() = 0.25, config/NL/config.py:5-8)
//   converged_i = allclose(x_old_i, x_pred_i, atol)   (numpy allclose: |a-b| <= atol + rtol |b|)
// on the neighbour graph (lambda[b, s, k] pairs agent b with nbr[b, s]) instead of the
// reference's dense n_agents^2 array.  Element-wise; built with -ffp-contract=off so the
// distance rounds the way numpy evaluates it.
#include <cmath>

#include "internal.h"

namespace cmpc {

__global__ void ocd_update_kernel(const OcdConst c, const int* __restrict__ nbr, const double* __restrict__ traj,
                                  double* __restrict__ lam) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (agent, slot, k-1)
    const int per = c.nb * c.N;
    if (i >= c.batch * per) return;
    const int b = i / per, r = i - b * per, s = r / c.N, k = r - s * c.N + 1;
    const int gi = c.self_offset + b, gj = nbr[b * c.nb + s];
    if (!(gi < gj)) return;  // the reference fills cost[i, j] for i < j only
    const double* pi = traj + ((size_t)gi * (c.N + 1) + k) * 2;
    const double* pj = traj + ((size_t)gj * (c.N + 1) + k) * 2;
    const double dx = pi[0] - pj[0], dy = pi[1] - pj[1];
    const double dx2 = dx * dx, dy2 = dy * dy;
    const double cost = c.dth - sqrt(dx2 + dy2);
    const double step = c.alpha * cost;
    lam[i] = lam[i] + step;
}

__global__ void ocd_close_kernel(int batch, int per, double atol, double rtol, const double* __restrict__ xo,
                                 const double* __restrict__ xp, int* __restrict__ close) {
    const int b = blockIdx.x;
    __shared__ int ok;
    if (threadIdx.x == 0) ok = 1;
    __syncthreads();
    for (int e = threadIdx.x; e < per; e += blockDim.x) {
        const double a = xo[(size_t)b * per + e], v = xp[(size_t)b * per + e];
        const double d = fabs(a - v), lim = atol + rtol * fabs(v);
        if (!(d <= lim)) ok = 0;  // NaN is never close (numpy equal_nan=False)
    }
    __syncthreads();
    if (threadIdx.x == 0) close[b] = ok;
}

hipError_t ocd_update_launch(const OcdConst& c, const int* nbr, const double* traj, double* lam, hipStream_t s) {
    const int total = c.batch * c.nb * c.N;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(ocd_update_kernel, dim3((total + 255) / 256), dim3(256), 0, s, c, nbr, traj, lam);
    return hipGetLastError();
}

hipError_t ocd_close_launch(int batch, int per, double atol, double rtol, const double* xo, const double* xp,
                            int* close, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(ocd_close_kernel, dim3(batch), dim3(64), 0, s, batch, per, atol, rtol, xo, xp, close);
    return hipGetLastError();
}

}  // namespace cmpc
