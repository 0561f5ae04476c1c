// Stage rows and linear cost of one synthetic double-integrator agent (the arithmetic of the
// per-round rebuild, see di_build.hip for the row pattern and the reference lines it follows).
// Shared by di_build_kernel (writes global qlin / C / h) and the fused round of the v3 solver
// (writes its LDS images), so both produce bit-identical rows: contraction is off inside.
#pragma once
#include <cmath>

#include "internal.h"

namespace cmpc {

// Stage k (0..N) of agent b: p_k -> pk[nx]; for k >= 1 also the rows of stage k (C_{k-1} ->
// Ck[mc*nx], h_{k-1} -> hk[mc], mc = 4 + nb).  own: the agent's exchanged trajectory
// ((N+1) x 2), nbr: its nb neighbour indices into traj_all.
// COMPACT (the v3 kernel's DS images, 2-D double integrator): Ck receives only the planes'
// coefficients [a_x, a_y] per neighbour (2 nb values); the other rows' coefficients are the
// constants -1 / +1 on v_x and +1 / -1 on p_y.  Same arithmetic, same bits.
template <bool COMPACT = false>
__device__ __forceinline__ void di_stage_rows(const DiConst& c, const int* nbr, double lane, const double* traj_all,
                                              const double* own, int k, double* pk, double* Ck, double* hk) {
#pragma clang fp contract(off)
    const int N = c.N, nb = c.nb, nx = c.nx, mc = 4 + nb, d = c.dim;
    const int ivx = d, ipy = 1;  // state = [p (dim) | v (dim)]
    for (int s = 0; s < nx; ++s) pk[s] = 0.0;
    pk[ivx] = -c.v_ref * c.q_v;
    pk[ipy] = -lane * c.q_lane;
    if (k == 0) return;
    const int h1 = k - 1;
    if (!COMPACT) {
        for (int i = 0; i < mc * nx; ++i) Ck[i] = 0.0;
        Ck[0 * nx + ivx] = -1.0;
        Ck[1 * nx + ivx] = 1.0;
        Ck[2 * nx + ipy] = 1.0;
        Ck[3 * nx + ipy] = -1.0;
    }
    hk[0] = -c.min_vel;
    hk[1] = c.max_vel;
    hk[2] = c.hw + lane;
    hk[3] = c.hw - lane;
    double px = 0.0, py = 0.0;
    for (int i = 0; i < nb; ++i) {
        const double* nt = traj_all + (size_t)nbr[i] * (N + 1) * 2;
        const double ex = own[h1 * 2], ey = own[h1 * 2 + 1];
        const double nx_ = nt[h1 * 2], ny_ = nt[h1 * 2 + 1];
        const double dx = nx_ - ex, dy = ny_ - ey;
        const double nrm = sqrt(dx * dx + dy * dy);
        const double ax = dx / nrm, ay = dy / nrm;
        const double bb = -0.5 * (ax * (ex + nx_) + ay * (ey + ny_));
        const double qx = own[k * 2] - nt[k * 2], qy = own[k * 2 + 1] - nt[k * 2 + 1];
        const double wgt = (2.0 * c.min_dist - sqrt(qx * qx + qy * qy)) / nb;
        double* cr = COMPACT ? Ck + 2 * i : Ck + (4 + i) * nx;
        cr[0] = ax;
        cr[1] = ay;
        hk[4 + i] = -c.min_dist / 2 - bb;
        px = px + c.wq * wgt * ax;
        py = py + c.wq * wgt * ay;
    }
    pk[0] += px;
    pk[1] += py;
}

}  // namespace cmpc
