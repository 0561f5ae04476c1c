// Reference-semantics builder: for every agent and stage, the quantities
// PlannerLPV.solve derives from its inputs before calling OSQP
// (planner/lib/plan_lib/distributedPlanner/LPV_Planner.py:115-157):
//   - LPV scheduling A_k, B_k                      _EstimateABC :477-591
//     (track lookups curvature / get_ey            utilities/misc.py:78-126)
//   - separating hyperplanes                       planes/compute_plane.py:41-68
//   - coverage weights                             utilities/misc.py:10-18
//   - stage rows C_k, h_k and linear cost p_k      :251-380, :382-427
// written in the structured layout the batched solver consumes.  Element-wise
// per (agent, stage); HBM-bound and tiny next to the solve.  Built with
// -ffp-contract=off so each expression rounds the way numpy evaluates it.
#include <cmath>

#include "internal.h"

namespace cmpc {

// Segment index of s (after lap wrapping, misc.py:84-91), -1 when the
// reference would raise (no / several matching segments, misc.py:97).
__device__ __forceinline__ int seg_lookup(const LpvConst& c, double s) {
    int laps = 0;
    while (s > c.track_len) {
        s = s - c.track_len;
        if (++laps > 100000) return -1;
    }
    if (s < 0) s = 0;
    int hit = -1, cnt = 0;
    for (int i = 0; i < c.nseg; ++i)
        if (s >= c.s0[i] && s < c.s0[i] + c.len[i]) {
            hit = i;
            ++cnt;
        }
    return cnt == 1 ? hit : -1;
}

__global__ __launch_bounds__(kWave) void lpv_build_kernel(const LpvConst c, const LpvPtrs P) {
    const int b = blockIdx.x;
    const int N = c.N, nb = c.nb, mc = c.mc;
    const double* xl = P.x_last + (size_t)b * c.last_rows * 9;
    const double* ul = P.u_last + (size_t)b * N * 2;
    const double* xa = P.x_agents ? P.x_agents + (size_t)b * (N + 1) * nb * 2 : nullptr;
    const double* po = P.pose + (size_t)b * (N + 1) * 2;
    double* A = P.A + (size_t)b * N * 81;
    double* B = P.B + (size_t)b * N * 18;
    double* p = P.p + (size_t)b * (N + 1) * 9;
    double* C = P.C + (size_t)b * N * mc * 9;
    double* h = P.h + (size_t)b * N * mc;
    double* planes = P.planes ? P.planes + (size_t)b * N * 3 * nb : nullptr;
    int bad = 0;

    for (int k = threadIdx.x; k <= N; k += kWave) {
        // linear cost on stage k: p_k[0] = -vx_ref*Q00 (all k), coverage on X,Y for k >= 1
        double* pk = p + k * 9;
        for (int s = 0; s < 9; ++s) pk[s] = 0.0;
        pk[0] = -c.vx_ref * c.Q00;
        if (k == 0) continue;
        const int h1 = k - 1;  // plane / weight row used by stage k (lagged, LPV_Planner.py:269-272,421)
        double px = 0.0, py = 0.0;
        double* Ck = C + (size_t)h1 * mc * 9;
        double* hk = h + (size_t)h1 * mc;
        for (int i = 0; i < nb; ++i) {
            double ax = 0.0, ay = 0.0, bb = 0.0, wgt = 1.0;
            if (xa) {
                // compute_plane.py:49-63 (keep_sign=True)
                const double ex = po[h1 * 2], ey = po[h1 * 2 + 1];
                const double nx_ = xa[(h1 * nb + i) * 2], ny_ = xa[(h1 * nb + i) * 2 + 1];
                double dx = nx_ - ex, dy = ny_ - ey;
                const double nrm = sqrt(dx * dx + dy * dy);
                ax = dx / nrm;
                ay = dy / nrm;
                bb = -0.5 * (ax * (ex + nx_) + ay * (ey + ny_));
                // misc.py:10-18: distance on rows 1..N, weight (2D - dist)/nb
                const double qx = po[k * 2] - xa[(k * nb + i) * 2];
                const double qy = po[k * 2 + 1] - xa[(k * nb + i) * 2 + 1];
                const double dist = sqrt(qx * qx + qy * qy);
                wgt = (2.0 * c.min_dist - dist) / nb;
            }
            if (planes) {
                planes[(h1 * 3 + 0) * nb + i] = ax;
                planes[(h1 * 3 + 1) * nb + i] = ay;
                planes[(h1 * 3 + 2) * nb + i] = bb;
            }
            double* cr = Ck + (4 + i) * 9;
            for (int s = 0; s < 9; ++s) cr[s] = 0.0;
            cr[7] = ax;
            cr[8] = ay;
            hk[4 + i] = -c.min_dist / 2 - bb;
            px = px + c.wq * wgt * ax;
            py = py + c.wq * wgt * ay;
        }
        pk[7] = px;
        pk[8] = py;

        // ---- LPV scheduling for row h1 of the previous prediction (LPV_Planner.py:493-585) ----
        const double* st = xl + h1 * 9;
        const double vx = st[0], vy = st[1], eyv = st[3], epsi = st[4], theta = st[5], sv = st[6];
        const int sg = seg_lookup(c, sv);
        if (sg < 0) {
            // the reference raises here (misc.py:97): write a defined stage (A = I, B = 0, zero
            // half-width) so the solver runs on known data, and flag the agent; lpv_mark_kernel
            // then reports it CMPC_UNSOLVED and NaN-fills its z
            bad = 1;
            double* Ak = A + (size_t)h1 * 81;
            for (int i = 0; i < 81; ++i) Ak[i] = (i % 10) == 0 ? 1.0 : 0.0;
            double* Bk = B + (size_t)h1 * 18;
            for (int i = 0; i < 18; ++i) Bk[i] = 0.0;
            for (int r = 0; r < 4; ++r)
                for (int s = 0; s < 9; ++s) Ck[r * 9 + s] = 0.0;
            Ck[0 * 9 + 0] = -1.0; hk[0] = -c.min_vel;
            Ck[1 * 9 + 0] = 1.0;  hk[1] = c.max_vel;
            Ck[2 * 9 + 3] = 1.0;  hk[2] = 0.0;
            Ck[3 * 9 + 3] = -1.0; hk[3] = 0.0;
            continue;
        }
        const double cur = c.curv[sg];
        const double delta = ul[h1 * 2];
        double A12 = 0, A13 = 0, A22 = 0, A23 = 0, A32 = 0, A33 = 0, B11 = 0;
        if (!(vx < 0.2)) {
            const double sd = sin(delta), cd = cos(delta);
            A12 = (sd * c.Cf) / (c.m * vx);
            A13 = (sd * c.Cf * c.lf) / (c.m * vx) + vy;
            A22 = -(c.Cr + c.Cf * cd) / (c.m * vx);
            A23 = -(c.lf * c.Cf * cd - c.lr * c.Cr) / (c.m * vx) - vx;
            A32 = -(c.lf * c.Cf * cd - c.lr * c.Cr) / (c.I * vx);
            A33 = -(c.lf * c.lf * c.Cf * cd + c.lr * c.lr * c.Cr) / (c.I * vx);
            B11 = -(sd * c.Cf) / c.m;
        }
        const double se = sin(epsi), ce = cos(epsi), sth = sin(theta), cth = cos(theta);
        const double den = 1 - eyv * cur;
        double Ac[81];
        for (int i = 0; i < 81; ++i) Ac[i] = 0.0;
        Ac[0] = -c.mu; Ac[1] = A12; Ac[2] = A13;
        Ac[10] = A22; Ac[11] = A23;
        Ac[19] = A32; Ac[20] = A33;
        Ac[27] = se; Ac[28] = ce;
        Ac[36] = (1 / den) * (-ce * cur); Ac[37] = (1 / den) * (se * cur); Ac[38] = 1.0;
        Ac[47] = 1.0;
        Ac[54] = ce / den; Ac[55] = -se / den;
        Ac[63] = cth; Ac[64] = -sth;
        Ac[72] = sth; Ac[73] = cth;
        double* Ak = A + (size_t)h1 * 81;
        for (int i = 0; i < 81; ++i) Ak[i] = ((i % 10) == 0 ? 1.0 : 0.0) + c.dt * Ac[i];
        double* Bk = B + (size_t)h1 * 18;
        for (int i = 0; i < 18; ++i) Bk[i] = 0.0;
        const double cdl = cos(delta);
        Bk[0] = c.dt * B11;
        Bk[1] = c.dt * 1.0;
        Bk[2] = c.dt * ((cdl * c.Cf) / c.m);
        Bk[4] = c.dt * ((c.lf * c.Cf * cdl) / c.I);

        // ---- stage rows (LPV_Planner.py:292-303, :306-315): hw from the previous prediction's s ----
        const double hw = c.hw[sg];
        for (int r = 0; r < 4; ++r)
            for (int s = 0; s < 9; ++s) Ck[r * 9 + s] = 0.0;
        Ck[0 * 9 + 0] = -1.0; hk[0] = -c.min_vel;
        Ck[1 * 9 + 0] = 1.0;  hk[1] = c.max_vel;
        Ck[2 * 9 + 3] = 1.0;  hk[2] = hw;
        Ck[3 * 9 + 3] = -1.0; hk[3] = hw;
    }
    if (bad && P.err) P.err[b] = 1;
}

hipError_t lpv_build_launch(const LpvConst& c, const LpvPtrs& p, int batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(lpv_build_kernel, dim3(batch), dim3(kWave), 0, s, c, p);
    return hipGetLastError();
}

__global__ void lpv_mark_kernel(const int* err, int* status, double* z, int nz, int batch) {
    const int b = blockIdx.x;
    if (b >= batch || !err[b]) return;
    if (status && threadIdx.x == 0) status[b] = CMPC_UNSOLVED;
    for (int i = threadIdx.x; i < nz; i += blockDim.x) z[(size_t)b * nz + i] = __builtin_nan("");
}

hipError_t lpv_mark_launch(const int* err, int* status, double* z, int nz, int batch, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(lpv_mark_kernel, dim3(batch), dim3(kWave), 0, s, err, status, z, nz, batch);
    return hipGetLastError();
}

}  // namespace cmpc
