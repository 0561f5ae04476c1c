// Consensus rounds behind a handle (include/cmpc.h, cmpc_lpv_rounds_*): the device-resident loop of
// LPV_HP_N_main.py:96-117 for hosts that own no device memory (MATLAB through the MEX gateway, C).
// The handle owns this rank's agent state and the node-global exchange buffer in one device
// allocation; a round chains the C-ABI device entry points on the context's stream:
//   cmpc_lpv_gather_dev -> cmpc_solve_lpv_batch_dev -> cmpc_lpv_advance_dev -> exchange
// where the exchange is a device copy (one rank), the RCCL all-gather of the context's
// communicator (cmpc_allgather_trajectories), or the host's (CMPC_ROUNDS_HOST_EXCHANGE).
#include <cstring>

#include "ctx.h"

struct cmpc_lpv_rounds {
    cmpc_ctx* ctx = nullptr;
    cmpc_lpv_params prm{};
    double seg[4][CMPC_MAX_SEG]{};  // copy of the track table: s0, len, curv, half_width
    cmpc_track track{};
    cmpc_lpv_rounds_dims d{};
    cmpc_opts opts{};
    int last_rows = 0;              // N + 1 in the first round, N afterwards (LPV_HP_N_main.py:115)
    char* mem = nullptr;
    double *x0 = nullptr, *x_last = nullptr, *u_last = nullptr, *u_old = nullptr, *traj_all = nullptr,
           *traj_local = nullptr, *pose = nullptr, *x_agents = nullptr, *z = nullptr, *planes = nullptr,
           *kkt = nullptr, *x_dense = nullptr;
    int *nbr = nullptr, *iters = nullptr, *status = nullptr, *infeasible = nullptr;
};

namespace {

size_t nz_lpv(int N) { return 12 * (size_t)(N + 1) + 4 * (size_t)N; }

}  // namespace

extern "C" {

int cmpc_lpv_rounds_create(cmpc_ctx* ctx, const cmpc_lpv_params* prm, const cmpc_track* track,
                           const cmpc_lpv_rounds_dims* dims, const cmpc_lpv_rounds_init* in, const cmpc_opts* opts,
                           cmpc_lpv_rounds** out) {
    if (!ctx) return CMPC_ERR_ARG;
    if (!out || !prm || !track || !dims || !in) return fail(ctx, CMPC_ERR_ARG, "null argument");
    *out = nullptr;
    const cmpc_lpv_rounds_dims& d = *dims;
    if (d.N < 1 || d.nb < 0 || 4 + d.nb > CMPC_MAX_MC || d.batch < 1 || d.n_total < d.batch || d.self_offset < 0 ||
        d.self_offset + d.batch > d.n_total)
        return fail(ctx, CMPC_ERR_ARG, "bad rounds dimensions (1 <= batch, self_offset + batch <= n_total, nb <= 12)");
    if (d.flags & ~(CMPC_ROUNDS_HOST_EXCHANGE | CMPC_ROUNDS_NO_HALT)) return fail(ctx, CMPC_ERR_ARG, "unknown rounds flag");
    if (track->nseg < 1 || track->nseg > CMPC_MAX_SEG) return fail(ctx, CMPC_ERR_UNSUPPORTED, "track has 1..32 segments");
    if (!in->x0 || !in->x_last || !in->u_last || (d.nb > 0 && !in->nbr))
        return fail(ctx, CMPC_ERR_ARG, "null initial state");
    if (!in->traj && d.batch != d.n_total)
        return fail(ctx, CMPC_ERR_ARG, "a sharded population needs the initial exchange buffer (init->traj)");
    if (d.batch != d.n_total && !(d.flags & CMPC_ROUNDS_HOST_EXCHANGE) &&
        (!ctx->comm || (long)ctx->nranks * d.batch != d.n_total || ctx->rank * d.batch != d.self_offset))
        return fail(ctx, CMPC_ERR_ARG,
                    "a sharded population exchanges over the context's communicator (cmpc_comm_init: equal "
                    "contiguous shards in rank order) or the host's (CMPC_ROUNDS_HOST_EXCHANGE)");
    for (int i = 0; in->nbr && i < d.batch * d.nb; ++i)
        if (in->nbr[i] < 0 || in->nbr[i] >= d.n_total) return fail(ctx, CMPC_ERR_ARG, "neighbour index out of range");
    if (opts && (opts->flags & ~CMPC_FLAG_ALL)) return fail(ctx, CMPC_ERR_ARG, "unknown option flag");
    HIP_TRY(hipSetDevice(ctx->device));

    auto* h = new cmpc_lpv_rounds();
    h->ctx = ctx;
    h->prm = *prm;
    h->d = d;
    if (opts) h->opts = *opts;
    h->opts.stamps = nullptr;
    h->opts.order = nullptr;
    h->last_rows = d.N + 1;
    const int ns = track->nseg;
    std::memcpy(h->seg[0], track->s0, sizeof(double) * ns);
    std::memcpy(h->seg[1], track->len, sizeof(double) * ns);
    std::memcpy(h->seg[2], track->curv, sizeof(double) * ns);
    std::memcpy(h->seg[3], track->half_width, sizeof(double) * ns);
    h->track = cmpc_track{ns, h->seg[0], h->seg[1], h->seg[2], h->seg[3]};

    const size_t B = d.batch, N = d.N, nb = d.nb, T = d.n_total, row = (N + 1) * 2;
    const size_t cnt[] = {B * 9, B * (N + 1) * 9, B * N * 2, B * 2, T * row, B * row, B * row,
                          B * row * (nb ? nb : 1), B * nz_lpv(d.N), B * N * 3 * (nb ? nb : 1), B, B * N * 9};
    size_t bytes = 0;
    for (size_t c : cnt) bytes += ((8 * c + 255) & ~size_t(255));
    bytes += 4 * ((B * (nb ? nb : 1) + 63) & ~size_t(63)) + 3 * 4 * ((B + 63) & ~size_t(63)) + 256;
    if (hipMalloc(&h->mem, bytes) != hipSuccess) {
        delete h;
        return fail(ctx, CMPC_ERR_NOMEM, "device allocation of the rounds state failed");
    }
    size_t off = 0;
    auto take = [&](size_t b) {
        char* p = h->mem + off;
        off += (b + 255) & ~size_t(255);
        return p;
    };
    double** dp[] = {&h->x0, &h->x_last, &h->u_last, &h->u_old, &h->traj_all, &h->traj_local, &h->pose,
                     &h->x_agents, &h->z, &h->planes, &h->kkt, &h->x_dense};
    for (int i = 0; i < 12; ++i) *dp[i] = reinterpret_cast<double*>(take(8 * cnt[i]));
    h->nbr = reinterpret_cast<int*>(take(4 * B * (nb ? nb : 1)));
    h->iters = reinterpret_cast<int*>(take(4 * B));
    h->status = reinterpret_cast<int*>(take(4 * B));
    h->infeasible = reinterpret_cast<int*>(take(4 * B));

    hipStream_t s = ctx->stream;
    auto up = [&](void* dst, const void* src, size_t b) { return hipMemcpyAsync(dst, src, b, hipMemcpyHostToDevice, s); };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = up(h->x0, in->x0, 8 * B * 9);
    if (e == hipSuccess) e = up(h->x_last, in->x_last, 8 * B * (N + 1) * 9);
    if (e == hipSuccess) e = up(h->u_last, in->u_last, 8 * B * N * 2);
    if (e == hipSuccess) e = in->u_old ? up(h->u_old, in->u_old, 8 * B * 2) : hipMemsetAsync(h->u_old, 0, 8 * B * 2, s);
    if (e == hipSuccess && nb) e = up(h->nbr, in->nbr, 4 * B * nb);
    if (e == hipSuccess) e = hipMemsetAsync(h->planes, 0, 8 * B * N * 3 * (nb ? nb : 1), s);
    if (e == hipSuccess && in->traj) e = up(h->traj_all, in->traj, 8 * T * row);
    if (e == hipSuccess && !in->traj)  // the reference's initial `agents` = the predictions' X, Y (misc.py:155-165)
        e = hipMemcpy2DAsync(h->traj_all, 16, h->x_last + 7, 72, 16, B * (N + 1), hipMemcpyDeviceToDevice, s);
    // this rank's rows of the exchange buffer: an agent that is not advanced keeps its initial ones
    if (e == hipSuccess)
        e = hipMemcpyAsync(h->traj_local, h->traj_all + (size_t)d.self_offset * row, 8 * B * row,
                           hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        (void)hipFree(h->mem);
        delete h;
        return hip_fail(ctx, e, "cmpc_lpv_rounds_create: upload");
    }
    *out = h;
    return CMPC_OK;
}

int cmpc_lpv_rounds_step(cmpc_lpv_rounds* h, int rounds, int* rounds_done, int* infeasible) {
    if (!h) return CMPC_ERR_ARG;
    cmpc_ctx* ctx = h->ctx;
    if (rounds < 0) return fail(ctx, CMPC_ERR_ARG, "negative round count");
    const bool host_x = h->d.flags & CMPC_ROUNDS_HOST_EXCHANGE, sharded = h->d.batch != h->d.n_total;
    if (host_x && sharded && rounds > 1)
        return fail(ctx, CMPC_ERR_ARG, "host exchange: one round per step (exchange between steps)");
    const bool halt = !(h->d.flags & CMPC_ROUNDS_NO_HALT);
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const cmpc_di_dims rd{h->d.batch, h->d.N, h->d.nb, h->d.self_offset};
    const int nb = h->d.nb;
    int done = 0, bad = 0, rc;
    for (int r = 0; r < rounds; ++r) {
        if ((rc = cmpc_lpv_gather_dev(ctx, &rd, h->nbr, h->traj_all, nb ? h->x_agents : nullptr, h->pose, s)) != CMPC_OK)
            return rc;
        const cmpc_lpv_dims ld{h->d.batch, h->d.N, nb, h->last_rows};
        const cmpc_lpv_data din{h->x0, h->x_last, h->u_last, h->u_old, nb ? h->x_agents : nullptr, h->pose};
        const cmpc_lpv_out dout{h->z, nb ? h->planes : nullptr, h->kkt, h->iters, h->status};
        if ((rc = cmpc_solve_lpv_batch_dev(ctx, &h->prm, &h->track, &ld, &din, &dout, &h->opts, s)) != CMPC_OK) return rc;
        HIP_TRY(hipMemsetAsync(h->infeasible, 0, sizeof(int), s));
        if (h->last_rows == h->d.N + 1) {
            // first round: Last_xPredicted goes from N + 1 rows per agent to N dense ones.  The advance
            // rewrites each agent's dense slot from its solution, but an agent it does not advance
            // (no finite solution) must find its own previous rows there, not bytes of the
            // (N + 1)-row layout: compact the layout first (rows 0..N-1 of each agent)
            const size_t w = 8 * (size_t)h->d.N * 9;
            HIP_TRY(hipMemcpy2DAsync(h->x_dense, w, h->x_last, w + 72, w, h->d.batch, hipMemcpyDeviceToDevice, s));
            HIP_TRY(hipMemcpyAsync(h->x_last, h->x_dense, w * h->d.batch, hipMemcpyDeviceToDevice, s));
        }
        if ((rc = cmpc_lpv_advance_dev(ctx, &rd, h->z, h->x0, h->x_last, h->u_last, h->u_old, h->traj_local, h->status,
                                       h->infeasible, s)) != CMPC_OK)
            return rc;
        h->last_rows = h->d.N;  // x_old = xPred[1:] from now on (LPV_HP_N_main.py:115)
        const size_t row = 2 * (size_t)(h->d.N + 1);
        if (!sharded) {
            HIP_TRY(hipMemcpyAsync(h->traj_all, h->traj_local, 8 * row * h->d.batch, hipMemcpyDeviceToDevice, s));
        } else if (!host_x) {
            if ((rc = cmpc_allgather_trajectories(ctx, h->traj_local, h->traj_all, row * h->d.batch, s)) != CMPC_OK)
                return rc;
        }
        // the node's infeasible count, not this rank's: the reference's loop quits for every agent
        // at once (LPV_HP_N_main.py:102-111), so every rank must take the same halt decision (a
        // rank that broke alone would leave the others waiting in the next round's all-gather).
        // The host exchange runs one round per step: its caller combines the counts it returns.
        if (sharded && !host_x && (rc = cmpc_comm_sum_i32(ctx, h->infeasible, 1, s)) != CMPC_OK) return rc;
        ++done;
        if (halt || r + 1 == rounds) {  // the reference stops the experiment at an infeasible agent
            HIP_TRY(hipMemcpyAsync(&bad, h->infeasible, sizeof(int), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (halt && bad) break;
        }
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (rounds_done) *rounds_done = done;
    if (infeasible) *infeasible = bad;
    return CMPC_OK;
}

int cmpc_lpv_rounds_read(cmpc_lpv_rounds* h, const cmpc_lpv_rounds_out* o) {
    if (!h) return CMPC_ERR_ARG;
    cmpc_ctx* ctx = h->ctx;
    if (!o) return fail(ctx, CMPC_ERR_ARG, "null output");
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t B = h->d.batch;
    auto dn = [&](void* dst, const void* src, size_t b) { return hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, s); };
    if (o->z) HIP_TRY(dn(o->z, h->z, 8 * B * nz_lpv(h->d.N)));
    if (o->kkt) HIP_TRY(dn(o->kkt, h->kkt, 8 * B));
    if (o->iters) HIP_TRY(dn(o->iters, h->iters, 4 * B));
    if (o->status) HIP_TRY(dn(o->status, h->status, 4 * B));
    if (o->x0) HIP_TRY(dn(o->x0, h->x0, 8 * B * 9));
    if (o->planes && h->d.nb) HIP_TRY(dn(o->planes, h->planes, 8 * B * h->d.N * 3 * h->d.nb));
    HIP_TRY(hipStreamSynchronize(s));
    return CMPC_OK;
}

int cmpc_lpv_rounds_get_traj(cmpc_lpv_rounds* h, double* traj_local) {
    if (!h) return CMPC_ERR_ARG;
    cmpc_ctx* ctx = h->ctx;
    if (!traj_local) return fail(ctx, CMPC_ERR_ARG, "null buffer");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpyAsync(traj_local, h->traj_local, 16 * (size_t)(h->d.N + 1) * h->d.batch, hipMemcpyDeviceToHost,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return CMPC_OK;
}

int cmpc_lpv_rounds_set_traj(cmpc_lpv_rounds* h, const double* traj_all) {
    if (!h) return CMPC_ERR_ARG;
    cmpc_ctx* ctx = h->ctx;
    if (!traj_all) return fail(ctx, CMPC_ERR_ARG, "null buffer");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpyAsync(h->traj_all, traj_all, 16 * (size_t)(h->d.N + 1) * h->d.n_total, hipMemcpyHostToDevice,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return CMPC_OK;
}

int cmpc_lpv_rounds_destroy(cmpc_lpv_rounds* h) {
    if (!h) return CMPC_OK;
    (void)hipSetDevice(h->ctx->device);
    (void)hipStreamSynchronize(h->ctx->stream);
    (void)hipFree(h->mem);
    delete h;
    return CMPC_OK;
}

}  // extern "C"
