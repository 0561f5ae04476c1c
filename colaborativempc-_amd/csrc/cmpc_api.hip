// C ABI of libcmpc (include/cmpc.h): context management, host<->device staging
// and dispatch of the batched kernels.  No CPU solver exists behind this ABI:
// without a gfx950 device every entry point fails with CMPC_ERR_DEVICE.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "ctx.h"

namespace {

// Ensure the device arena holds `bytes`; returns base pointer or nullptr.
char* arena(cmpc_ctx* ctx, size_t bytes) {
    if (ctx->ws_bytes >= bytes) return ctx->ws;
    if (ctx->ws) {
        // the arena may be in use by work queued on caller streams (the *_dev entry points)
        (void)hipDeviceSynchronize();
        (void)hipFree(ctx->ws);
        ctx->ws = nullptr;
        ctx->ws_bytes = 0;
    }
    size_t want = bytes + bytes / 4 + (1 << 20);
    if (hipMalloc(&ctx->ws, want) != hipSuccess) return nullptr;
    ctx->ws_bytes = want;
    return ctx->ws;
}

struct Carve {
    char* base;
    size_t off = 0;
    template <class T>
    T* take(size_t count) {
        off = (off + 255) & ~size_t(255);
        T* p = reinterpret_cast<T*>(base + off);
        off += count * sizeof(T);
        return p;
    }
};

size_t mpc_nz(const cmpc_mpc_dims& d) { return (size_t)(d.nx + d.ns) * (d.N + 1) + 2 * (size_t)d.nu * d.N; }

int set_device(cmpc_ctx* ctx) {
    hipError_t e = hipSetDevice(ctx->device);
    return e == hipSuccess ? CMPC_OK : hip_fail(ctx, e, "hipSetDevice");
}

int build_lpv_const(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* tr, const cmpc_lpv_dims* d,
                    cmpc::LpvConst* c) {
    if (!prm || !tr || !d) return fail(ctx, CMPC_ERR_ARG, "null argument");
    if (tr->nseg < 1 || tr->nseg > CMPC_MAX_SEG) return fail(ctx, CMPC_ERR_UNSUPPORTED, "track has 1..32 segments");
    if (d->N < 1 || d->nb < 0 || 4 + d->nb > CMPC_MAX_MC || (d->last_rows != d->N && d->last_rows != d->N + 1) ||
        d->batch < 0)
        return fail(ctx, CMPC_ERR_ARG, "bad LPV dimensions (last_rows must be N or N+1, nb <= 12)");
    *c = cmpc::LpvConst{};
    c->N = d->N;
    c->nb = d->nb;
    c->last_rows = d->last_rows;
    c->nseg = tr->nseg;
    c->mc = 4 + d->nb;
    c->lf = prm->lf; c->lr = prm->lr; c->m = prm->m; c->I = prm->I;
    c->Cf = prm->Cf; c->Cr = prm->Cr; c->mu = prm->mu;
    c->vx_ref = prm->vx_ref; c->min_dist = prm->min_dist; c->max_vel = prm->max_vel; c->min_vel = prm->min_vel;
    c->max_rs = prm->max_rs; c->max_ls = prm->max_ls; c->max_ac = prm->max_ac; c->max_dc = prm->max_dc;
    c->dt = prm->dt; c->wq = prm->wq; c->Q00 = prm->Q[0];
    for (int i = 0; i < tr->nseg; ++i) {
        c->s0[i] = tr->s0[i];
        c->len[i] = tr->len[i];
        c->curv[i] = tr->curv[i];
        c->hw[i] = tr->half_width[i];
    }
    // TrackLength = PointAndTangent[-1, 3] + PointAndTangent[-1, 4]  (utilities/misc.py:85)
    c->track_len = tr->s0[tr->nseg - 1] + tr->len[tr->nseg - 1];
    return CMPC_OK;
}

int lpv_solver_const(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_lpv_dims* d, const cmpc_opts* o,
                     cmpc::MpcConst* mc) {
    // checked here as well as in build_lpv_const: this runs first in both LPV entry points and
    // fills fixed-size row tables
    if (!prm || !d) return fail(ctx, CMPC_ERR_ARG, "null argument");
    if (d->N < 1 || d->nb < 0 || 4 + d->nb > CMPC_MAX_MC || d->batch < 0)
        return fail(ctx, CMPC_ERR_ARG, "bad LPV dimensions (N >= 1, 0 <= nb <= 12)");
    cmpc_mpc_dims md{9, 2, d->N, 3, 4 + d->nb, d->batch};
    int slack[CMPC_MAX_MC], sign[CMPC_MAX_MC];
    const int base_slack[4] = {-1, 0, 1, 1};
    for (int r = 0; r < md.mc && r < CMPC_MAX_MC; ++r) {
        slack[r] = r < 4 ? base_slack[r] : 2;
        sign[r] = r < 4 ? 1 : -1;
    }
    double Qsd[3] = {prm->Qs[0], prm->Qs[1], prm->Qs[2]};
    // input rows [delta <= max_rs; -delta <= max_ls; a <= max_ac; -a <= max_dc]  (LPV_Planner.py:331-339)
    double ub[2] = {prm->max_rs, prm->max_ac}, lb[2] = {-prm->max_ls, -prm->max_dc};
    cmpc_mpc_weights w{prm->Q, prm->R, prm->dR, Qsd, ub, lb, slack, sign};
    const char* msg = nullptr;
    int rc = cmpc::mpc_prepare(&md, &w, o, mc, &msg);
    if (rc != CMPC_OK) return fail(ctx, rc, msg);
    // the structure lpv_build.hip writes (A_k = I + dt A_c on columns 0..2, B_k rows 0..2, rows on
    // vx / ey / (X, Y)) lets the v3 kernel keep compact images when Q is also diagonal
    bool qdiag = true;
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j)
            if (i != j && prm->Q[i * 9 + j] != 0.0) qdiag = false;
    // 2: Q also zero on states 1, 2, 5, 6 (the reference's config_LPV.py:7): the v3 kernel's L5 contraction
    const bool q5 = prm->Q[1 * 9 + 1] == 0.0 && prm->Q[2 * 9 + 2] == 0.0 && prm->Q[5 * 9 + 5] == 0.0 &&
                    prm->Q[6 * 9 + 6] == 0.0;
    mc->lpv = (qdiag && !(o && (o->flags & CMPC_FLAG_GENERIC))) ? (q5 ? 2 : 1) : 0;
    return CMPC_OK;
}

}  // namespace

extern "C" {

int cmpc_abi_version(void) { return CMPC_ABI_VERSION; }

int cmpc_create(cmpc_ctx** out, int device) {
    if (!out) return CMPC_ERR_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return CMPC_ERR_DEVICE;
    if (device < 0 || device >= count) return CMPC_ERR_ARG;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return CMPC_ERR_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CMPC_ERR_DEVICE;
    auto* c = new cmpc_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return CMPC_ERR_DEVICE;
    }
    *out = c;
    return CMPC_OK;
}

int cmpc_destroy(cmpc_ctx* ctx) {
    if (!ctx) return CMPC_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return CMPC_OK;
}

// ---- multi-GPU exchange over RCCL (cmpc.h) ----
static_assert(sizeof(ncclUniqueId) == CMPC_COMM_ID_BYTES, "ncclUniqueId size");

int cmpc_comm_id(unsigned char id[CMPC_COMM_ID_BYTES]) {
    if (!id) return CMPC_ERR_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return CMPC_ERR_DEVICE;
    std::memcpy(id, &u, sizeof u);
    return CMPC_OK;
}

int cmpc_comm_init(cmpc_ctx* ctx, int nranks, int rank, const unsigned char id[CMPC_COMM_ID_BYTES]) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(ctx, CMPC_ERR_ARG, "bad communicator arguments");
    if (ctx->comm) return fail(ctx, CMPC_ERR_ARG, "context already joined a communicator");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    const ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        ctx->comm = nullptr;
        return fail(ctx, CMPC_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    ctx->nranks = nranks;
    ctx->rank = rank;
    return CMPC_OK;
}

int cmpc_allgather_trajectories(cmpc_ctx* ctx, const double* traj_local, double* traj_all, unsigned long long count,
                                void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!ctx->comm) return fail(ctx, CMPC_ERR_ARG, "cmpc_comm_init has not been called on this context");
    if (count && (!traj_local || !traj_all)) return fail(ctx, CMPC_ERR_ARG, "null trajectory buffer");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    const ncclResult_t r = ncclAllGather(traj_local, traj_all, (size_t)count, ncclDouble, ctx->comm, (hipStream_t)stream);
    if (r != ncclSuccess) return fail(ctx, CMPC_ERR_DEVICE, std::string("ncclAllGather: ") + ncclGetErrorString(r));
    return CMPC_OK;
}

int cmpc_comm_sum_i32(cmpc_ctx* ctx, int* buf, unsigned long long count, void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (count && !buf) return fail(ctx, CMPC_ERR_ARG, "null buffer");
    if (!ctx->comm || !count) return CMPC_OK;  // one rank: the local count is the node's
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, ncclInt32, ncclSum, ctx->comm, (hipStream_t)stream);
    if (r != ncclSuccess) return fail(ctx, CMPC_ERR_DEVICE, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    return CMPC_OK;
}

int cmpc_comm_destroy(cmpc_ctx* ctx) {
    if (!ctx) return CMPC_ERR_ARG;
    if (ctx->comm) {
        (void)set_device(ctx);
        (void)ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
        ctx->nranks = 1;
        ctx->rank = 0;
    }
    return CMPC_OK;
}

const char* cmpc_last_error(const cmpc_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int cmpc_solve_mpc_batch_dev(cmpc_ctx* ctx, const cmpc_mpc_dims* dims, const cmpc_mpc_weights* w,
                             const cmpc_mpc_data* in, const cmpc_mpc_out* out, const cmpc_opts* opts,
                             void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!in || !out || !out->z) return fail(ctx, CMPC_ERR_ARG, "null data / output");
    cmpc::MpcConst c;
    const char* msg = nullptr;
    int rc = cmpc::mpc_prepare(dims, w, opts, &c, &msg);
    if (rc != CMPC_OK) return fail(ctx, rc, msg);
    if ((rc = set_device(ctx)) != CMPC_OK) return rc;
    double* ws = nullptr;
    int* plist = nullptr;
    if (const size_t wsd = cmpc::mpc_ws_doubles(c) * (size_t)dims->batch) {
        // (+ the polish launch's compacted agent list: batch + 1 ints after the scratch)
        ws = reinterpret_cast<double*>(arena(ctx, 8 * wsd + 4 * ((size_t)dims->batch + 1)));
        if (!ws) return fail(ctx, CMPC_ERR_NOMEM, "device scratch allocation failed");
        plist = reinterpret_cast<int*>(ws + wsd);
    }
    cmpc::MpcPtrs p{in->A, in->B, in->x0, in->u_prev, in->qlin, in->C, in->h, out->z, out->kkt, out->iters, out->status,
                    opts ? (unsigned long long*)opts->stamps : nullptr, ws};
    p.order = opts ? opts->order : nullptr;
    p.plist = plist;
    HIP_TRY(cmpc::mpc_launch(c, p, dims->batch, (hipStream_t)stream, opts ? opts->flags : 0));
    return CMPC_OK;
}

int cmpc_plan_mpc(const cmpc_mpc_dims* dims, const cmpc_mpc_weights* w, const cmpc_opts* opts, cmpc_plan_info* out) {
    if (!dims || !w || !out) return CMPC_ERR_ARG;
    cmpc::MpcConst c;
    const char* msg = nullptr;
    const int rc = cmpc::mpc_prepare(dims, w, opts, &c, &msg);
    if (rc != CMPC_OK) return rc;
    // the choice of mpc_launch: lane, Riccati, the specialised condensed kernel, the generic one
    size_t lds;
    out->agents_per_wg = 1;
    if (c.lane) {
        out->solver = CMPC_SOLVER_LANE;
        lds = cmpc::mpc_lane_lds_bytes(c);
        out->agents_per_wg = 32;
    } else if (c.riccati) {
        out->solver = CMPC_SOLVER_RICCATI;
        lds = cmpc::mpc_riccati_lds_bytes(c);
    } else if (!(opts && (opts->flags & CMPC_FLAG_GENERIC)) && (lds = cmpc::mpc3_lds_bytes(c)) != 0) {
        out->solver = CMPC_SOLVER_CONDENSED_V3;
    } else {
        out->solver = CMPC_SOLVER_CONDENSED;
        lds = cmpc::mpc_lds_bytes(c);
    }
    out->lds_bytes = (int)lds;
    const size_t wg = lds ? cmpc::kMaxLdsBytes / lds : 4;
    out->wg_per_cu = (int)(wg < 4 ? wg : 4);
    out->waves_per_agent = (c.riccati && !c.lane && cmpc::mpc_riccati_mw(c)) ? 4 : 1;  // (the Riccati latency mode)
    out->polish_lds_bytes = c.polish ? (int)cmpc::mpc_polish_lds_bytes(c) : 0;
    out->polish_max_active = c.polish ? cmpc::mpc_polish_max_active(c) : 0;
    return CMPC_OK;
}

int cmpc_solve_mpc_batch(cmpc_ctx* ctx, const cmpc_mpc_dims* d, const cmpc_mpc_weights* w,
                         const cmpc_mpc_data* in, const cmpc_mpc_out* out, const cmpc_opts* opts) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!d || !in || !out || !out->z) return fail(ctx, CMPC_ERR_ARG, "null argument");
    cmpc::MpcConst c;
    const char* msg = nullptr;
    int rc = cmpc::mpc_prepare(d, w, opts, &c, &msg);
    if (rc != CMPC_OK) return fail(ctx, rc, msg);
    if ((rc = set_device(ctx)) != CMPC_OK) return rc;
    const size_t B = d->batch, N = d->N, nx = d->nx, nu = d->nu, mc = d->mc;
    const size_t sA = B * N * nx * nx, sB = B * N * nx * nu, sx = B * nx, su = B * nu, sp = B * (N + 1) * nx,
                 sC = B * N * mc * nx, sh = B * N * mc, sz = B * mpc_nz(*d);
    const size_t sw = cmpc::mpc_ws_doubles(c) * B;
    const size_t bytes = 8 * (sA + sB + sx + su + sp + sC + sh + sz + B + sw) + 8 * B + 4 * (B + 1) + 16 * 256;
    char* base = arena(ctx, bytes);
    if (!base) return fail(ctx, CMPC_ERR_NOMEM, "device arena allocation failed");
    Carve cv{base};
    double *dA = cv.take<double>(sA), *dB = cv.take<double>(sB), *dx0 = cv.take<double>(sx),
           *du = cv.take<double>(su), *dp = cv.take<double>(sp), *dC = cv.take<double>(sC),
           *dh = cv.take<double>(sh), *dz = cv.take<double>(sz), *dk = cv.take<double>(B);
    int *di = cv.take<int>(B), *ds = cv.take<int>(B);
    double* dw = sw ? cv.take<double>(sw) : nullptr;
    int* dpl = sw ? cv.take<int>(B + 1) : nullptr;  // the polish launch's compacted agent list
    hipStream_t s = ctx->stream;
    HIP_TRY(hipMemcpyAsync(dA, in->A, 8 * sA, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dB, in->B, 8 * sB, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dx0, in->x0, 8 * sx, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(du, in->u_prev, 8 * su, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dp, in->qlin, 8 * sp, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dC, in->C, 8 * sC, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dh, in->h, 8 * sh, hipMemcpyHostToDevice, s));
    cmpc::MpcPtrs p{dA, dB, dx0, du, dp, dC, dh, dz, dk, di, ds,
                    opts ? (unsigned long long*)opts->stamps : nullptr, dw};  // stamps: device memory
    p.plist = dpl;
    HIP_TRY(cmpc::mpc_launch(c, p, d->batch, s, opts ? opts->flags : 0));
    HIP_TRY(hipMemcpyAsync(out->z, dz, 8 * sz, hipMemcpyDeviceToHost, s));
    if (out->kkt) HIP_TRY(hipMemcpyAsync(out->kkt, dk, 8 * B, hipMemcpyDeviceToHost, s));
    if (out->iters) HIP_TRY(hipMemcpyAsync(out->iters, di, 4 * B, hipMemcpyDeviceToHost, s));
    if (out->status) HIP_TRY(hipMemcpyAsync(out->status, ds, 4 * B, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return CMPC_OK;
}

// Workspace layout of the LPV path (device): structured problem + error flags + solver scratch.
static size_t lpv_ws_bytes(const cmpc_lpv_dims* d, size_t solver_ws_doubles) {
    const size_t B = d->batch, N = d->N, mc = 4 + d->nb;
    return 8 * (B * N * 81 + B * N * 18 + B * (N + 1) * 9 + B * N * mc * 9 + B * N * mc + B * solver_ws_doubles) +
           4 * B + 4 * (B + 1) + 11 * 256;  // (B + 1 ints: the polish launch's compacted agent list)
}

static int lpv_run(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* tr, const cmpc_lpv_dims* d,
                   const cmpc_lpv_data* in, const cmpc_lpv_out* out, const cmpc_opts* opts, hipStream_t s,
                   Carve& cv) {
    cmpc::LpvConst lc;
    int rc = build_lpv_const(ctx, prm, tr, d, &lc);
    if (rc != CMPC_OK) return rc;
    cmpc::MpcConst mc;
    if ((rc = lpv_solver_const(ctx, prm, d, opts, &mc)) != CMPC_OK) return rc;
    const size_t B = d->batch, N = d->N, m = 4 + d->nb;
    double *A = cv.take<double>(B * N * 81), *Bm = cv.take<double>(B * N * 18), *p = cv.take<double>(B * (N + 1) * 9),
           *C = cv.take<double>(B * N * m * 9), *h = cv.take<double>(B * N * m);
    int* err = cv.take<int>(B);
    const size_t sw = cmpc::mpc_ws_doubles(mc) * B;
    double* ws = sw ? cv.take<double>(sw) : nullptr;
    int* plist = sw ? cv.take<int>(B + 1) : nullptr;  // the polish launch's compacted agent list
    HIP_TRY(hipMemsetAsync(err, 0, 4 * B, s));
    cmpc::LpvPtrs lp{in->x_last, in->u_last, in->x_agents, in->pose, A, Bm, p, C, h, out->planes, err};
    HIP_TRY(cmpc::lpv_build_launch(lc, lp, d->batch, s));
    cmpc::MpcPtrs mp{A, Bm, in->x0, in->u_old, p, C, h, out->z, out->kkt, out->iters, out->status,
                    opts ? (unsigned long long*)opts->stamps : nullptr, ws};  // stamps: device memory
    mp.plist = plist;
    HIP_TRY(cmpc::mpc_launch(mc, mp, d->batch, s, opts ? opts->flags : 0));
    HIP_TRY(cmpc::lpv_mark_launch(err, out->status, out->z, (int)(12 * (N + 1) + 4 * N), d->batch, s));
    return CMPC_OK;
}

int cmpc_solve_lpv_batch_dev(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* tr, const cmpc_lpv_dims* d,
                             const cmpc_lpv_data* in, const cmpc_lpv_out* out, const cmpc_opts* opts, void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!d || !in || !out || !out->z || !in->x0 || !in->x_last || !in->u_last || !in->u_old || !in->pose)
        return fail(ctx, CMPC_ERR_ARG, "null argument");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    cmpc::MpcConst mc;
    if ((rc = lpv_solver_const(ctx, prm, d, opts, &mc)) != CMPC_OK) return rc;
    char* base = arena(ctx, lpv_ws_bytes(d, cmpc::mpc_ws_doubles(mc)));
    if (!base) return fail(ctx, CMPC_ERR_NOMEM, "device arena allocation failed");
    Carve cv{base};
    return lpv_run(ctx, prm, tr, d, in, out, opts, (hipStream_t)stream, cv);
}

int cmpc_lpv_gather_dev(cmpc_ctx* ctx, const cmpc_di_dims* d, const int* nbr, const double* traj_all,
                        double* x_agents, double* pose, void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!d || !traj_all || !pose || (d->nb > 0 && (!nbr || !x_agents)))
        return fail(ctx, CMPC_ERR_ARG, "null argument");
    if (d->N < 1 || d->nb < 0 || d->batch < 0 || d->self_offset < 0) return fail(ctx, CMPC_ERR_ARG, "bad dimensions");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    HIP_TRY(cmpc::lpv_gather_launch(d->N, d->nb, d->self_offset, nbr, traj_all, d->nb ? x_agents : nullptr, pose,
                                    d->batch, (hipStream_t)stream));
    return CMPC_OK;
}

int cmpc_lpv_advance_dev(cmpc_ctx* ctx, const cmpc_di_dims* d, const double* z, double* x0, double* x_last,
                         double* u_last, double* u_old, double* traj_local, const int* status, int* infeasible,
                         void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!d || !z || !x0 || !x_last || !u_last || !u_old || !traj_local) return fail(ctx, CMPC_ERR_ARG, "null argument");
    if (d->N < 1 || d->batch < 0) return fail(ctx, CMPC_ERR_ARG, "bad dimensions");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    HIP_TRY(cmpc::lpv_advance_launch(d->N, z, x0, x_last, u_last, u_old, traj_local, d->batch, (hipStream_t)stream,
                                     status, infeasible));
    return CMPC_OK;
}

int cmpc_lpv_build_dev(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* tr, const cmpc_lpv_dims* d,
                       const cmpc_lpv_data* in, const cmpc_lpv_build_out* out, void* stream) {
    if (!ctx || !in || !out || !d) return fail(ctx, CMPC_ERR_ARG, "null argument");
    if (!out->A || !out->B || !out->qlin || !out->C || !out->h || !out->err)
        return fail(ctx, CMPC_ERR_ARG, "null builder output");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    cmpc::LpvConst lc;
    if ((rc = build_lpv_const(ctx, prm, tr, d, &lc)) != CMPC_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(out->err, 0, 4 * (size_t)d->batch, s));
    cmpc::LpvPtrs lp{in->x_last, in->u_last, in->x_agents, in->pose, out->A, out->B, out->qlin, out->C, out->h,
                     out->planes, out->err};
    HIP_TRY(cmpc::lpv_build_launch(lc, lp, d->batch, s));
    return CMPC_OK;
}

int cmpc_solve_lpv_batch(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* tr, const cmpc_lpv_dims* d,
                         const cmpc_lpv_data* in, const cmpc_lpv_out* out, const cmpc_opts* opts) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!d || !in || !out || !out->z || !in->x0 || !in->x_last || !in->u_last || !in->u_old || !in->pose)
        return fail(ctx, CMPC_ERR_ARG, "null argument");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    const size_t B = d->batch, N = d->N, nb = d->nb, nz = 12 * (N + 1) + 4 * N;
    const size_t sx0 = B * 9, sxl = B * d->last_rows * 9, sul = B * N * 2, suo = B * 2,
                 sxa = in->x_agents ? B * (N + 1) * nb * 2 : 0, spo = B * (N + 1) * 2, sz = B * nz,
                 spl = out->planes ? B * N * 3 * nb : 0;
    cmpc::MpcConst mc;
    if ((rc = lpv_solver_const(ctx, prm, d, opts, &mc)) != CMPC_OK) return rc;
    const size_t bytes = lpv_ws_bytes(d, cmpc::mpc_ws_doubles(mc)) +
                         8 * (sx0 + sxl + sul + suo + sxa + spo + sz + spl + B) + 8 * B + 16 * 256;
    char* base = arena(ctx, bytes);
    if (!base) return fail(ctx, CMPC_ERR_NOMEM, "device arena allocation failed");
    Carve cv{base};
    double *x0 = cv.take<double>(sx0), *xl = cv.take<double>(sxl), *ul = cv.take<double>(sul),
           *uo = cv.take<double>(suo), *xa = sxa ? cv.take<double>(sxa) : nullptr, *po = cv.take<double>(spo),
           *z = cv.take<double>(sz), *pl = spl ? cv.take<double>(spl) : nullptr, *kk = cv.take<double>(B);
    int *it = cv.take<int>(B), *st = cv.take<int>(B);
    hipStream_t s = ctx->stream;
    HIP_TRY(hipMemcpyAsync(x0, in->x0, 8 * sx0, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(xl, in->x_last, 8 * sxl, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ul, in->u_last, 8 * sul, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(uo, in->u_old, 8 * suo, hipMemcpyHostToDevice, s));
    if (sxa) HIP_TRY(hipMemcpyAsync(xa, in->x_agents, 8 * sxa, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(po, in->pose, 8 * spo, hipMemcpyHostToDevice, s));
    cmpc_lpv_data din{x0, xl, ul, uo, xa, po};
    cmpc_lpv_out dout{z, pl, kk, it, st};
    rc = lpv_run(ctx, prm, tr, d, &din, &dout, opts, s, cv);
    if (rc != CMPC_OK) return rc;
    HIP_TRY(hipMemcpyAsync(out->z, z, 8 * sz, hipMemcpyDeviceToHost, s));
    if (out->planes) HIP_TRY(hipMemcpyAsync(out->planes, pl, 8 * spl, hipMemcpyDeviceToHost, s));
    if (out->kkt) HIP_TRY(hipMemcpyAsync(out->kkt, kk, 8 * B, hipMemcpyDeviceToHost, s));
    if (out->iters) HIP_TRY(hipMemcpyAsync(out->iters, it, 4 * B, hipMemcpyDeviceToHost, s));
    if (out->status) HIP_TRY(hipMemcpyAsync(out->status, st, 4 * B, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return CMPC_OK;
}

static int di_const(cmpc_ctx* ctx, const cmpc_di_params* prm, const cmpc_di_dims* d, cmpc::DiConst* c) {
    if (!prm || !d) return fail(ctx, CMPC_ERR_ARG, "null argument");
    if ((prm->dim != 2 && prm->dim != 3) || d->N < 1 || d->nb < 0 || 4 + d->nb > CMPC_MAX_MC || d->batch < 0 ||
        d->self_offset < 0)
        return fail(ctx, CMPC_ERR_ARG, "bad double-integrator dimensions");
    *c = cmpc::DiConst{d->N, d->nb, 2 * prm->dim, prm->dim, 3, prm->dim, d->self_offset, prm->v_ref, prm->q_v,
                       prm->q_lane, prm->hw, prm->min_vel, prm->max_vel, prm->min_dist, prm->wq};
    return set_device(ctx);
}

int cmpc_di_build_dev(cmpc_ctx* ctx, const cmpc_di_params* prm, const cmpc_di_dims* d, const int* nbr,
                      const double* lane, const double* traj_all, double* qlin, double* C, double* h, void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!lane || !traj_all || !qlin || !C || !h || (d && d->nb > 0 && !nbr))
        return fail(ctx, CMPC_ERR_ARG, "null argument");
    cmpc::DiConst c;
    int rc = di_const(ctx, prm, d, &c);
    if (rc != CMPC_OK) return rc;
    cmpc::DiPtrs p{nbr, lane, traj_all, qlin, C, h};
    HIP_TRY(cmpc::di_build_launch(c, p, d->batch, (hipStream_t)stream));
    return CMPC_OK;
}

int cmpc_di_solve_dev(cmpc_ctx* ctx, const cmpc_di_params* prm, const cmpc_di_dims* dd, const int* nbr,
                      const double* lane, const double* traj_all, const cmpc_mpc_dims* dims,
                      const cmpc_mpc_weights* w, const cmpc_mpc_data* in, const cmpc_mpc_out* out,
                      const cmpc_opts* opts, void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!lane || !traj_all || !dims || !in || !out || !out->z || (dd && dd->nb > 0 && !nbr))
        return fail(ctx, CMPC_ERR_ARG, "null argument");
    cmpc::DiConst dc;
    int rc = di_const(ctx, prm, dd, &dc);
    if (rc != CMPC_OK) return rc;
    cmpc::MpcConst c;
    const char* msg = nullptr;
    rc = cmpc::mpc_prepare(dims, w, opts, &c, &msg);
    if (rc != CMPC_OK) return fail(ctx, rc, msg);
    if (dims->batch != dd->batch || dims->N != dd->N || dims->nx != dc.nx || dims->nu != dc.nu ||
        dims->mc != 4 + dd->nb)
        return fail(ctx, CMPC_ERR_ARG, "double-integrator and solver dimensions differ");
    if (dims->batch == 0) return CMPC_OK;
    const int flags = opts ? opts->flags : 0;
    hipStream_t s = (hipStream_t)stream;
    if (!c.lane && !c.riccati && !c.rescue && !(flags & CMPC_FLAG_GENERIC)) {  // rescue needs materialised rows
        cmpc::MpcPtrs p{in->A, in->B, in->x0, in->u_prev, nullptr, nullptr, nullptr, out->z, out->kkt, out->iters,
                        out->status, opts ? (unsigned long long*)opts->stamps : nullptr, nullptr};
        p.fuse = cmpc::DiFuse{nbr, lane, traj_all, dc, 1};
        hipError_t e = hipSuccess;
        if (cmpc::mpc3_try_launch(c, p, dims->batch, s, &e)) {
            HIP_TRY(e);
            return CMPC_OK;
        }
    }
    // no fused instantiation for these dimensions: build into data's qlin / C / h, then solve
    if (!in->qlin || !in->C || !in->h) return fail(ctx, CMPC_ERR_ARG, "unfused round needs qlin / C / h buffers");
    cmpc::DiPtrs dp{nbr, lane, traj_all, const_cast<double*>(in->qlin), const_cast<double*>(in->C),
                    const_cast<double*>(in->h)};
    HIP_TRY(cmpc::di_build_launch(dc, dp, dd->batch, s));
    return cmpc_solve_mpc_batch_dev(ctx, dims, w, in, out, opts, stream);
}

int cmpc_di_advance_dev(cmpc_ctx* ctx, const cmpc_di_params* prm, const cmpc_di_dims* d, const double* z,
                        double* x0, double* u_prev, double* traj_local, void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!z || !x0 || !u_prev || !traj_local) return fail(ctx, CMPC_ERR_ARG, "null argument");
    cmpc::DiConst c;
    int rc = di_const(ctx, prm, d, &c);
    if (rc != CMPC_OK) return rc;
    HIP_TRY(cmpc::di_advance_launch(c, z, x0, u_prev, traj_local, d->batch, (hipStream_t)stream));
    return CMPC_OK;
}

int cmpc_solve_qp_batch(cmpc_ctx* ctx, const cmpc_qp_dims* d, const cmpc_qp_data* in, const cmpc_qp_out* out,
                        const cmpc_opts* opts) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!d || !in || !out || !out->x) return fail(ctx, CMPC_ERR_ARG, "null argument");
    if (d->n < 1 || d->m_ineq < 0 || d->m_eq < 0 || d->batch < 0)
        return fail(ctx, CMPC_ERR_ARG, "bad QP dimensions");
    if (!in->H || !in->f) return fail(ctx, CMPC_ERR_ARG, "H and f are required");
    if (d->m_ineq > 0 && (!in->A || !in->b)) return fail(ctx, CMPC_ERR_ARG, "m_ineq > 0 needs A and b");
    if (d->m_eq > 0 && (!in->Aeq || !in->beq)) return fail(ctx, CMPC_ERR_ARG, "m_eq > 0 needs Aeq and beq");
    if ((double)(d->n + d->m_eq) * (d->n + d->m_eq) > 2.0e8) return fail(ctx, CMPC_ERR_UNSUPPORTED, "QP too large");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    if (d->batch == 0) return CMPC_OK;
    const size_t B = d->batch, n = d->n, mi = d->m_ineq, me = d->m_eq;
    const size_t sH = B * n * n, sf = B * n, sA = B * mi * n, sb = B * mi, sE = B * me * n, se = B * me,
                 sl = in->lb ? B * n : 0, su = in->ub ? B * n : 0, ws = B * cmpc::qp_ws_doubles(d->n, d->m_ineq, d->m_eq);
    const size_t bytes = 8 * (sH + sf + sA + sb + sE + se + sl + su + ws + B * n + B * mi + B * me + 2 * B * n + 2 * B) +
                         8 * B + 24 * 256;
    char* base = arena(ctx, bytes);
    if (!base) return fail(ctx, CMPC_ERR_NOMEM, "device arena allocation failed");
    Carve cv{base};
    double *dH = cv.take<double>(sH), *df = cv.take<double>(sf), *dA = mi ? cv.take<double>(sA) : nullptr,
           *db = mi ? cv.take<double>(sb) : nullptr, *dE = me ? cv.take<double>(sE) : nullptr,
           *de = me ? cv.take<double>(se) : nullptr, *dl = sl ? cv.take<double>(sl) : nullptr,
           *du = su ? cv.take<double>(su) : nullptr, *dws = cv.take<double>(ws), *dx = cv.take<double>(B * n),
           *dli = cv.take<double>(B * mi + 1), *dle = cv.take<double>(B * me + 1), *dlo = cv.take<double>(B * n),
           *dup = cv.take<double>(B * n), *dfv = cv.take<double>(B), *dmr = cv.take<double>(B);
    int *dfl = cv.take<int>(B), *dit = cv.take<int>(B);
    hipStream_t s = ctx->stream;
    HIP_TRY(hipMemcpyAsync(dH, in->H, 8 * sH, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(df, in->f, 8 * sf, hipMemcpyHostToDevice, s));
    if (mi) HIP_TRY(hipMemcpyAsync(dA, in->A, 8 * sA, hipMemcpyHostToDevice, s));
    if (mi) HIP_TRY(hipMemcpyAsync(db, in->b, 8 * sb, hipMemcpyHostToDevice, s));
    if (me) HIP_TRY(hipMemcpyAsync(dE, in->Aeq, 8 * sE, hipMemcpyHostToDevice, s));
    if (me) HIP_TRY(hipMemcpyAsync(de, in->beq, 8 * se, hipMemcpyHostToDevice, s));
    if (sl) HIP_TRY(hipMemcpyAsync(dl, in->lb, 8 * sl, hipMemcpyHostToDevice, s));
    if (su) HIP_TRY(hipMemcpyAsync(du, in->ub, 8 * su, hipMemcpyHostToDevice, s));
    cmpc::QpConst qc{d->n, d->m_ineq, d->m_eq, d->col_major ? 1 : 0,
                     (opts && opts->max_iter > 0) ? opts->max_iter : 100, 8,
                     (opts && opts->tol > 0) ? opts->tol : 1e-9, 1e-8};
    cmpc::QpPtrs qp{dH, df, dA, db, dE, de, dl, du, dx, dfv, dli, dle, dlo, dup, dmr, dfl, dit, dws};
    HIP_TRY(cmpc::qp_launch(qc, qp, d->batch, s));
    HIP_TRY(hipMemcpyAsync(out->x, dx, 8 * B * n, hipMemcpyDeviceToHost, s));
    if (out->fval) HIP_TRY(hipMemcpyAsync(out->fval, dfv, 8 * B, hipMemcpyDeviceToHost, s));
    if (out->exitflag) HIP_TRY(hipMemcpyAsync(out->exitflag, dfl, 4 * B, hipMemcpyDeviceToHost, s));
    if (out->iters) HIP_TRY(hipMemcpyAsync(out->iters, dit, 4 * B, hipMemcpyDeviceToHost, s));
    if (out->residual) HIP_TRY(hipMemcpyAsync(out->residual, dmr, 8 * B, hipMemcpyDeviceToHost, s));
    if (out->lambda_ineqlin && mi) HIP_TRY(hipMemcpyAsync(out->lambda_ineqlin, dli, 8 * B * mi, hipMemcpyDeviceToHost, s));
    if (out->lambda_eqlin && me) HIP_TRY(hipMemcpyAsync(out->lambda_eqlin, dle, 8 * B * me, hipMemcpyDeviceToHost, s));
    if (out->lambda_lower) HIP_TRY(hipMemcpyAsync(out->lambda_lower, dlo, 8 * B * n, hipMemcpyDeviceToHost, s));
    if (out->lambda_upper) HIP_TRY(hipMemcpyAsync(out->lambda_upper, dup, 8 * B * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return CMPC_OK;
}

int cmpc_ocd_update_dev(cmpc_ctx* ctx, const cmpc_ocd_dims* d, double alpha, double dth, const int* nbr,
                        const double* traj_all, double* lam, void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!d || d->batch < 0 || d->N < 1 || d->nb < 0 || d->self_offset < 0) return fail(ctx, CMPC_ERR_ARG, "bad OCD dims");
    if (d->batch && d->nb && (!nbr || !traj_all || !lam)) return fail(ctx, CMPC_ERR_ARG, "null argument");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    cmpc::OcdConst c{d->batch, d->N, d->nb, d->self_offset, alpha, dth};
    HIP_TRY(cmpc::ocd_update_launch(c, nbr, traj_all, lam, (hipStream_t)stream));
    return CMPC_OK;
}

int cmpc_ocd_converged_dev(cmpc_ctx* ctx, int batch, int per, double atol, double rtol, const double* x_old,
                           const double* x_pred, int* close, void* stream) {
    if (!ctx) return CMPC_ERR_ARG;
    if (batch < 0 || per < 0) return fail(ctx, CMPC_ERR_ARG, "bad sizes");
    if (batch && (!x_old || !x_pred || !close)) return fail(ctx, CMPC_ERR_ARG, "null argument");
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    HIP_TRY(cmpc::ocd_close_launch(batch, per, atol, rtol, x_old, x_pred, close, (hipStream_t)stream));
    return CMPC_OK;
}

int cmpc_selftest_mfma(cmpc_ctx* ctx, const double* A, const double* B, double* D) {
    if (!ctx || !A || !B || !D) return CMPC_ERR_ARG;
    int rc = set_device(ctx);
    if (rc != CMPC_OK) return rc;
    char* base = arena(ctx, 8 * (64 + 64 + 256) + 1024);
    if (!base) return fail(ctx, CMPC_ERR_NOMEM, "arena");
    Carve cv{base};
    double *dA = cv.take<double>(64), *dB = cv.take<double>(64), *dD = cv.take<double>(256);
    hipStream_t s = ctx->stream;
    HIP_TRY(hipMemcpyAsync(dA, A, 8 * 64, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dB, B, 8 * 64, hipMemcpyHostToDevice, s));
    HIP_TRY(cmpc::selftest_mfma_launch(dA, dB, dD, s));
    HIP_TRY(hipMemcpyAsync(D, dD, 8 * 256, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return CMPC_OK;
}

}  // extern "C"
