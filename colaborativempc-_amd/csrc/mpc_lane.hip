// Lane-per-agent stage-wise interior-point solver: one LANE of a wavefront owns one agent, so a
// wavefront advances 64 agents at once with no cross-lane traffic at all — the layout for large
// batches of long-horizon agents (BASELINE cfg5: 8192 agents per GPU, N = 50, nx = 6, nu = 3),
// where the one-wave-per-agent Riccati kernel (mpc_riccati.hip) leaves most lanes idle in every
// serial step of the stage recursion.
//
// Method: the SAME Mehrotra predictor-corrector as every other solver of libcmpc (internal.h:
// residuals, scaling, merit, safeguards, termination; oracle/cmpc_oracle.c restates it), with the
// Newton system solved stage-wise by the Riccati recursion of mpc_riccati.hip on the augmented
// state y_k = [dX_k; dU_{k-1}] (oracle ric_factor / ric_solve, standard form).  The QP is the one
// PlannerLPV assembles (planner/lib/plan_lib/distributedPlanner/LPV_Planner.py:279-475).
//
// Sweeps.  Everything an iteration needs is produced by four passes over the horizon, each stage
// read once per pass straight from the caller's agent-major inputs:
//   S1 backward: the step of the previous iteration applied (lazily), residual adjoints (gradient
//      scale, dual residual), primal / slack residuals, complementarity, the Riccati factorisation
//      and the predictor's backward solve;
//   S2 forward:  predictor feedback solve, predictor row steps (stored), the affine step and
//      mu_aff (as a quadratic in the step length);
//   S3 backward: corrector right-hand side and backward solve (same gains);
//   S4 forward:  corrector feedback solve, the direction (stored), the step bound;
// then one pass over the rows for the neighbourhood backtracking.  Per-agent scratch is lane-
// interleaved (element i of agent b at ws[i * batch + b]) so every access of a wavefront is one
// coalesced 512-byte (fp64) line set.
//
// Precision (template MIXED).  MIXED = false: everything fp64.  MIXED = true (CMPC_FLAG_FP32,
// BASELINE cfg5's "fp32 path with tolerance check vs fp64 reference"): the Riccati factorisation,
// its gains and both Newton solves' recursions run in fp32; iterates, residuals, the row algebra
// and the state recursion of the direction stay fp64, so the iterate never drifts from the
// simulation of its inputs.  An agent whose fp32 factorisation breaks down, or that makes no
// progress for kF32Stall iterations, continues in fp64 (per lane: the wave runs both paths only
// while its lanes disagree).  tools/f32_lab.py measured the scheme on the C restatement
// (oracle RIC_F32): 99.3 % CMPC_SOLVED at tol 1e-6 on 2048 cfg5 agents, z within 2e-4 of the
// fp64 double-double solve, ~12 % of agents finishing in fp64 (two iterations on average).
#include "lane_body.h"

namespace cmpc {

// One wavefront per kLaneAP agents (lanes kLaneAP..63 leave at once); dynamic LDS: its two stage images.
template <int NX, int NU, int MC, int NS, bool MIXED>
__global__ __launch_bounds__(kWave) void mpc_lane_kernel(const MpcConst c, const MpcPtrs P, int batch) {
    extern __shared__ __attribute__((aligned(16))) char lane_smem[];
    if (threadIdx.x >= kLaneAP) return;
    const int b = blockIdx.x * kLaneAP + threadIdx.x;
    // launch order (cmpc_opts.order): slot b holds agent order[b] (clamped; lane_pack gathered it),
    // so the agents of a wavefront have similar iteration counts and leave it together
    if (b < batch)
        lane_agent<NX, NU, MC, NS, MIXED>(c, P, batch, b, lane_smem,
                                          P.order ? min(max(P.order[b], 0), batch - 1) : b);
}

size_t mpc_lane_ws_doubles(const MpcConst& c) { return lane_layout(c).total; }

// agent-major inputs -> the pair-interleaved copy of lane_body.h (element e of agent b at
// ((e / 2) * batch + b) * 2 + e % 2), through a 64 x 64 LDS tile so that the reads (along e) and
// the writes (along b) are both coalesced
__global__ __launch_bounds__(256) void lane_pack_kernel(const double* __restrict__ src, double* __restrict__ dst,
                                                        int batch, int T, const int* __restrict__ order) {
    __shared__ double tile[64][65];
    const int e0 = blockIdx.x * 64, b0 = blockIdx.y * 64, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int b = b0 + r, e = e0 + tx;
        if (b < batch && e < T) {
            const int a = order ? min(max(order[b], 0), batch - 1) : b;  // slot b <- agent order[b]
            tile[r][tx] = src[(size_t)a * T + e];
        }
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int e = e0 + r, b = b0 + tx;
        if (b < batch && e < T) dst[((size_t)(e >> 1) * batch + b) * 2 + (e & 1)] = tile[tx][r];
    }
}

static hipError_t lane_pack(const double* src, double* dst, int batch, int T, const int* order, hipStream_t s) {
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(lane_pack_kernel, dim3((T + 63) / 64, (batch + 63) / 64), dim3(256), 0, s, src, dst, batch, T,
                       order);
    return hipGetLastError();
}

template <int NX, int NU, int MC, int NS>
static bool lane_try(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s, hipError_t* e) {
    if (c.nx != NX || c.nu != NU || c.mc != MC || c.ns != NS) return false;
    const dim3 grid((batch + kLaneAP - 1) / kLaneAP);
    const size_t lds = 2 * (size_t)IMap<NX, NU, MC, NS>::bytes;
    const void* fn = c.lane == 2 ? (const void*)mpc_lane_kernel<NX, NU, MC, NS, true>
                                 : (const void*)mpc_lane_kernel<NX, NU, MC, NS, false>;
    if ((*e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) != hipSuccess) return true;
    if (c.lane == 2) hipLaunchKernelGGL((mpc_lane_kernel<NX, NU, MC, NS, true>), grid, dim3(kWave), lds, s, c, p, batch);
    else hipLaunchKernelGGL((mpc_lane_kernel<NX, NU, MC, NS, false>), grid, dim3(kWave), lds, s, c, p, batch);
    *e = hipGetLastError();
    return true;
}

bool mpc_lane_supported(const MpcConst& c) {
    return (c.nx == 6 && c.nu == 3 && c.mc == 6 && c.ns == 3) || (c.nx == 4 && c.nu == 2 && c.mc == 6 && c.ns == 3);
}

size_t mpc_lane_lds_bytes(const MpcConst& c) {
    if (c.nx == 6 && c.nu == 3 && c.mc == 6 && c.ns == 3) return 2 * (size_t)IMap<6, 3, 6, 3>::bytes;
    if (c.nx == 4 && c.nu == 2 && c.mc == 6 && c.ns == 3) return 2 * (size_t)IMap<4, 2, 6, 3>::bytes;
    return 0;
}

hipError_t mpc_lane_launch(const MpcConst& c, const MpcPtrs& p, int batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    if (!p.ws) return hipErrorInvalidValue;
    const LaneLayout L = lane_layout(c);
    // The kernel addresses the launch's scratch through one buffer resource with 32-bit offsets
    // (lane_body.h): a batch whose scratch reaches 2 GiB (cfg5 N = 50: ~19.7k agents; N = 125: ~8k)
    // runs as consecutive sub-launches, each with its own agents' pointers and the scratch reused
    // from its base (an agent's results depend on its own data only).  The launch order indexes the
    // whole batch, so the sub-launches run in agent order.
    const size_t per = L.total * sizeof(double);
    if (per * (size_t)batch >= 0x7fffffffull) {
        const int chunk = (int)((0x7fffffffull / per) / kLaneAP * kLaneAP);
        if (chunk < kLaneAP) return hipErrorInvalidValue;
        const int N = c.N, nx = c.nx, nu = c.nu, mc = c.mc;
        const size_t nz = (size_t)(nx + c.ns) * (N + 1) + 2 * (size_t)c.n;
        for (int b0 = 0; b0 < batch; b0 += chunk) {
            const size_t o = (size_t)b0;
            MpcPtrs q = p;
            q.A = p.A + o * N * nx * nx;
            q.B = p.B + o * N * nx * nu;
            q.x0 = p.x0 + o * nx;
            q.up = p.up + o * nu;
            q.p = p.p + o * (N + 1) * nx;
            q.C = p.C + o * N * mc * nx;
            q.h = p.h + o * N * mc;
            q.z = p.z + o * nz;
            if (p.kkt) q.kkt = p.kkt + o;
            if (p.iters) q.iters = p.iters + o;
            if (p.status) q.status = p.status + o;
            q.stamps = nullptr;
            q.order = nullptr;
            hipError_t e = mpc_lane_launch(c, q, batch - b0 < chunk ? batch - b0 : chunk, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const size_t S = (size_t)batch;
    const int N = c.N, nx = c.nx, nu = c.nu, mc = c.mc;
    hipError_t e;
    if ((e = lane_pack(p.A, p.ws + L.iA * S, batch, N * nx * nx, p.order, s)) != hipSuccess) return e;
    if ((e = lane_pack(p.B, p.ws + L.iB * S, batch, N * nx * nu, p.order, s)) != hipSuccess) return e;
    if ((e = lane_pack(p.C, p.ws + L.iC * S, batch, N * mc * nx, p.order, s)) != hipSuccess) return e;
    if ((e = lane_pack(p.h, p.ws + L.ih * S, batch, N * mc, p.order, s)) != hipSuccess) return e;
    if ((e = lane_pack(p.p, p.ws + L.ip * S, batch, (N + 1) * nx, p.order, s)) != hipSuccess) return e;
    e = hipErrorInvalidValue;
    if (lane_try<6, 3, 6, 3>(c, p, batch, s, &e)) return e;  // BASELINE cfg5 (3-D double integrator, nb = 2)
    if (lane_try<4, 2, 6, 3>(c, p, batch, s, &e)) return e;  // cfg1-4 shape (2-D double integrator, nb = 2)
    return hipErrorInvalidValue;
}

}  // namespace cmpc
