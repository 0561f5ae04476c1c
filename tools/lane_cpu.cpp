// Host build of the lane-per-agent solver body (colaborativempc-_amd/csrc/lane_body.h): the exact
// code every lane of mpc_lane_kernel runs, executed on the CPU for one agent after another, so the
// kernel's arithmetic can be checked against the C restatement (oracle/cmpc_oracle.c) without a
// GPU.  Diagnostic only (tools/lane_cpu.py builds and drives it).
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lane_body.h"

extern "C" int lane_cpu_solve(int nx, int nu, int N, int ns, int mc, int batch, const double* Q, const double* R,
                              const double* dR, const double* Qs, const double* u_ub, const double* u_lb,
                              const int* row_slack, const int* row_sign, const double* A, const double* B,
                              const double* x0, const double* up, const double* p, const double* C, const double* h,
                              double tol, int max_iter, int mixed, double* z, double* kkt, int* iters, int* status) {
    using namespace cmpc;
    MpcConst c{};
    c.nx = nx; c.nu = nu; c.N = N; c.ns = ns; c.mc = mc;
    c.n = N * nu; c.ms = N * mc; c.m = c.ms + 2 * nu * N;
    c.max_iter = max_iter; c.tol = tol; c.lane = mixed ? 2 : 1;
    double qs = 1.0;
    for (int i = 0; i < nx * nx; ++i) c.Q[i] = Q[i];
    for (int i = 0; i < nu * nu; ++i) { c.R[i] = R[i]; c.dR[i] = dR[i]; }
    for (int j = 0; j < ns; ++j) { c.Qs[j] = Qs[j]; qs = qs > 2 * Qs[j] ? qs : 2 * Qs[j]; }
    c.qs_max = qs;
    for (int i = 0; i < nu; ++i) { c.u_ub[i] = u_ub[i]; c.u_lb[i] = u_lb[i]; }
    for (int r = 0; r < mc; ++r) { c.row_slack[r] = row_slack[r]; c.row_sign[r] = row_sign[r] >= 0 ? 1 : -1; }
    const LaneLayout L = lane_layout(c);
    std::vector<double> ws(L.total * (size_t)batch);
    auto pack = [&](const double* src, size_t off, int T) {  // lane_pack_kernel on the host
        for (int b = 0; b < batch; ++b)
            for (int e = 0; e < T; ++e) ws[off * batch + ((size_t)(e >> 1) * batch + b) * 2 + (e & 1)] = src[(size_t)b * T + e];
    };
    pack(A, L.iA, N * nx * nx);
    pack(B, L.iB, N * nx * nu);
    pack(C, L.iC, N * mc * nx);
    pack(h, L.ih, N * mc);
    pack(p, L.ip, (N + 1) * nx);
    MpcPtrs P{};
    P.A = A; P.B = B; P.x0 = x0; P.up = up; P.p = p; P.C = C; P.h = h;
    P.z = z; P.kkt = kkt; P.iters = iters; P.status = status; P.ws = ws.data();
    for (int b = 0; b < batch; ++b) {
        if (nx == 6 && nu == 3 && mc == 6 && ns == 3) {
            if (mixed) lane_agent<6, 3, 6, 3, true>(c, P, batch, b, nullptr);
            else lane_agent<6, 3, 6, 3, false>(c, P, batch, b, nullptr);
        } else if (nx == 4 && nu == 2 && mc == 6 && ns == 3) {
            if (mixed) lane_agent<4, 2, 6, 3, true>(c, P, batch, b, nullptr);
            else lane_agent<4, 2, 6, 3, false>(c, P, batch, b, nullptr);
        } else {
            return -1;
        }
    }
    return 0;
}
