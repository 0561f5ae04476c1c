"""Device-resident consensus-round driver (the collaborative loop of
planner/scripts/LPV_HP_N_main.py:96-120, and of the one-process-per-agent ROS
variant ROS/src/planner_experiments/src/LPV_ROS_main.py:124-150, re-designed as
one process per GPU).

Each round, on the GPU and on one stream:
  1. build   — every local agent's stage rows / linear cost from the previous
               round's exchanged trajectories            (cmpc_di_build_dev)
  2. solve   — batched condensed IPM, one wavefront per agent  (cmpc_solve_mpc_batch_dev)
  3. advance — x0 <- x_1, u_prev <- u_0, local trajectory <- predicted positions
               (LPV_HP_N_main.py:106-117)                (cmpc_di_advance_dev)
  4. exchange — all-gather of the (N+1) x 2 fp64 predicted positions of every
               agent over RCCL (torch.distributed "nccl" backend) — the
               replacement of the ROS topic exchange / np.swapaxes at :117.

Agents are sharded contiguously across ranks (they are ordered along the road,
so most neighbours are local); every rank holds the full gathered trajectory
buffer, which is what a Jacobi round needs.
"""
from __future__ import annotations

import ctypes as ct

import numpy as np

from . import _lib as L
from .solver import _dims, _tptr, _weights, nz_of


def exchange_positions(traj_all, traj_local, world=1, group=None, comm=None):
    """The per-round exchange of predicted positions (the np.swapaxes "exchange" of
    LPV_HP_N_main.py:117, and the ROS topic publish/subscribe of LPV_ROS_main.py:66-77):
    every rank's contiguous block `traj_local` (B, N+1, 2) is gathered, in rank order,
    into the node-global `traj_all` (world*B, N+1, 2).  One all-gather per round;
    over RCCL/xGMI with the "nccl" backend, gloo on CPU tensors."""
    if comm is not None:   # libcmpc's own RCCL communicator (cmpc.comm.Comm), no torch.distributed
        comm.allgather(traj_local, traj_all)
        return
    if world == 1:
        traj_all.copy_(traj_local)
        return
    import torch.distributed as dist

    if traj_all.shape[0] != world * traj_local.shape[0]:
        raise ValueError("traj_all must hold world x local agents")
    if traj_all.is_cuda and dist.get_backend(group) == "gloo":
        # gloo moves host memory only: stage through the host (multi-process runs sharing one
        # GPU, or hosts without RCCL); the gathered rows are the same bytes in the same order
        host = traj_all.new_empty(traj_all.shape, device="cpu")
        dist.all_gather_into_tensor(host, traj_local.detach().cpu().contiguous(), group=group)
        traj_all.copy_(host)
        return
    dist.all_gather_into_tensor(traj_all, traj_local.contiguous(), group=group)


class DIRounds:
    def __init__(self, scen, rank=0, world=1, device=None, ctx=None, tol=None, max_iter=None, group=None,
                 fp32=False, comm=None, fused=True, lpt=None):
        import torch

        self.torch = torch
        self.scen, self.rank, self.world, self.group, self.comm = scen, rank, world, group, comm
        # step(): rows built inside the solver launch (cmpc_di_solve_dev) instead of build() + solve()
        self.fused = fused
        if scen.n_agents % world:
            raise ValueError("n_agents must be divisible by the number of ranks")
        self.dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.ctx = ctx or L.default_context(self.dev.index)
        sl = scen.shard(rank, world)
        self.off = sl.start
        self.B = sl.stop - sl.start
        self.N, self.nb = scen.N, scen.nb
        sh = scen.shared
        self.shared = sh
        T = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=self.dev)
        self.A = T(scen.A[sl])
        self.Bm = T(scen.B[sl])
        self.x0 = T(scen.x0[sl])
        self.u_prev = T(scen.u_prev[sl])
        self.lane = T(scen.lane[sl])
        self.nbr = T(scen.nbr[sl], torch.int32)
        self.traj_all = T(scen.traj)
        self.traj_local = torch.empty((self.B, self.N + 1, 2), dtype=torch.float64, device=self.dev)
        nx, mc = sh["nx"], sh["mc"]
        self.qlin = torch.empty((self.B, self.N + 1, nx), dtype=torch.float64, device=self.dev)
        self.C = torch.empty((self.B, self.N, mc, nx), dtype=torch.float64, device=self.dev)
        self.h = torch.empty((self.B, self.N, mc), dtype=torch.float64, device=self.dev)
        self.z = torch.empty((self.B, nz_of(sh)), dtype=torch.float64, device=self.dev)
        self.kkt = torch.empty(self.B, dtype=torch.float64, device=self.dev)
        self.iters = torch.empty(self.B, dtype=torch.int32, device=self.dev)
        self.status = torch.empty(self.B, dtype=torch.int32, device=self.dev)
        p = scen.params
        self.dprm = L.cmpc_di_params(int(p["dim"]), *(float(p[k]) for k in ("v_ref", "q_v", "q_lane", "hw",
                                                                              "min_vel", "max_vel", "min_dist",
                                                                              "wq")))
        self.ddims = L.cmpc_di_dims(self.B, self.N, self.nb, self.off)
        self.mdims = _dims(sh, self.B)
        self.w, self._wkeep = _weights(sh)
        from .solver import FP32_TOL

        self.opts = L.opts(tol or (FP32_TOL if fp32 else None), max_iter, L.CMPC_FLAG_FP32 if fp32 else 0)
        # lpt: launch the Riccati solver's agents longest-first, by last round's IPM iterations
        # (cmpc_opts.order; many agents per SIMD there, so the launch otherwise ends with whichever
        # slow agents happened to start last).  Default: on where the stage-wise solver runs (the
        # condensed kernels have one agent per SIMD and ignore the order).  The fp32 lane kernel packs
        # its wavefronts in that order, but at cfg5 all of its 256 wavefronts run at once (one per CU),
        # so its launch still ends with the slowest agent (measured 91.9 -> 99.8 ms): off where fp32
        # runs on it, i.e. on dimensions without the Riccati kernel's fp32 instantiation (6, 3, 6).
        ric32 = (sh["nx"], sh["nu"], sh["mc"]) == (6, 3, 6)
        self.lpt = (self.N * sh["nu"] > 64 and (not fp32 or ric32)) if lpt is None else bool(lpt)
        self._order = None
        self.data = L.cmpc_mpc_data(*[_tptr(t) for t in (self.A, self.Bm, self.x0, self.u_prev, self.qlin,
                                                          self.C, self.h)])
        self.out = L.cmpc_mpc_out(_tptr(self.z), _tptr(self.kkt), _tptr(self.iters), _tptr(self.status))

    def bind_outputs(self, kkt, iters, status):
        """Point the solver's per-agent kkt / iters / status outputs at other (B,) device
        tensors (e.g. one row per round of a preallocated history), without copies."""
        torch = self.torch
        for name, t, dt in (("kkt", kkt, torch.float64), ("iters", iters, torch.int32),
                            ("status", status, torch.int32)):
            if not isinstance(t, torch.Tensor) or t.device != self.dev or t.dtype != dt or \
                    tuple(t.shape) != (self.B,) or not t.is_contiguous():
                raise ValueError(f"{name}: need a contiguous ({self.B},) {dt} tensor on {self.dev}")
        self.kkt, self.iters, self.status = kkt, iters, status
        self.out = L.cmpc_mpc_out(_tptr(self.z), _tptr(kkt), _tptr(iters), _tptr(status))

    def _stream(self):
        return ct.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def build(self):
        lib = self.ctx.lib
        self.ctx.check(lib.cmpc_di_build_dev(self.ctx.h, ct.byref(self.dprm), ct.byref(self.ddims), _tptr(self.nbr),
                                             _tptr(self.lane), _tptr(self.traj_all), _tptr(self.qlin),
                                             _tptr(self.C), _tptr(self.h), self._stream()))

    def _order_in(self):
        self.opts.order = self._order.data_ptr() if (self.lpt and self._order is not None) else None

    def _order_out(self):
        if self.lpt:  # next round's launch order (stream-ordered after this solve)
            self._order = self.torch.argsort(self.iters, descending=True, stable=True).to(self.torch.int32)

    def solve(self):
        self._order_in()
        self.ctx.check(self.ctx.lib.cmpc_solve_mpc_batch_dev(self.ctx.h, ct.byref(self.mdims), ct.byref(self.w),
                                                             ct.byref(self.data), ct.byref(self.out),
                                                             ct.byref(self.opts), self._stream()))
        self._order_out()

    def build_solve(self):
        """build() + solve() as one launch where the v3 kernel covers the problem (the rows go
        from traj_all straight into the solver's LDS, bit-identical to build()); qlin / C / h are
        then left untouched — call build() before snapshot() to materialise them."""
        lib = self.ctx.lib
        self._order_in()
        self.ctx.check(lib.cmpc_di_solve_dev(self.ctx.h, ct.byref(self.dprm), ct.byref(self.ddims), _tptr(self.nbr),
                                             _tptr(self.lane), _tptr(self.traj_all), ct.byref(self.mdims),
                                             ct.byref(self.w), ct.byref(self.data), ct.byref(self.out),
                                             ct.byref(self.opts), self._stream()))
        self._order_out()

    def advance(self):
        self.ctx.check(self.ctx.lib.cmpc_di_advance_dev(self.ctx.h, ct.byref(self.dprm), ct.byref(self.ddims),
                                                        _tptr(self.z), _tptr(self.x0), _tptr(self.u_prev),
                                                        _tptr(self.traj_local), self._stream()))

    def exchange(self):
        exchange_positions(self.traj_all, self.traj_local, self.world, self.group, self.comm)

    def step(self, timer=None):
        """One consensus round.  `timer` (start, stop) events bracket the solve launch (with
        `fused`, the launch that builds and solves)."""
        if not self.fused:
            self.build()
        if timer is not None:
            timer[0].record()
        if self.fused:
            self.build_solve()
        else:
            self.solve()
        if timer is not None:
            timer[1].record()
        self.advance()
        self.exchange()

    def snapshot(self):
        """Host copy of this rank's current structured problem (for checkers)."""
        p = dict(self.shared)
        for k, t in (("A", self.A), ("B", self.Bm), ("x0", self.x0), ("u_prev", self.u_prev), ("qlin", self.qlin),
                     ("C", self.C), ("h", self.h)):
            p[k] = t.detach().cpu().numpy().copy()
        return p


class LPVRounds:
    """Device-resident consensus rounds of the reference's LPV agents (LPV_HP_N_main.py:96-117):
    per round gather (neighbour and own positions from the exchange buffer) -> build + solve
    (cmpc_solve_lpv_batch_dev: scheduling, planes, weights, rows, the QP) -> advance (x0 <-
    xPred[1], Last_xPredicted <- xPred[1:], uPred, [OldSteering, OldAccelera] <- u_0) -> exchange
    (all-gather of the predicted X, Y).  Everything stays in HBM; the host only launches.

    ``bp``: a ``PlannerLPVBatch`` (gains, map, horizon, options, context).  Population arrays
    (all ranks' agents, sharded contiguously): x0 (n, 9), x_last (n, N+1, 9) (the first
    round's Last_xPredicted), u_last (n, N, 2), nbr (n, nb) neighbour indices (the reference: all
    other agents, :82-85), u_old (n, 2) (default 0, PlannerLPV's initial OldSteering /
    OldAccelera), traj (n, N+1, 2) (default x_last[:, :, 7:9], the reference's initial
    ``agents``)."""

    def __init__(self, bp, x0, x_last, u_last, nbr, u_old=None, traj=None, rank=0, world=1, group=None, comm=None):
        import torch

        self.torch, self.bp, self.ctx = torch, bp, bp.ctx
        self.rank, self.world, self.group, self.comm = rank, world, group, comm
        x0 = np.asarray(x0, np.float64)
        n, N = x0.shape[0], bp.N
        if n % world:
            raise ValueError("agents must be divisible by the number of ranks")
        nbr = np.asarray(nbr, np.int32).reshape(n, -1)
        if nbr.size and (nbr.min() < 0 or nbr.max() >= n):
            raise ValueError("nbr: neighbour indices must address the population (0 <= j < n)")
        if np.shape(u_last) != (n, N, 2) or (u_old is not None and np.shape(u_old) != (n, 2)) or \
                (traj is not None and np.shape(traj) != (n, N + 1, 2)) or x0.shape != (n, 9):
            raise ValueError("x0 (n, 9), u_last (n, N, 2), u_old (n, 2), traj (n, N+1, 2) expected")
        self.N, self.nb = N, nbr.shape[1]
        self.B = n // world
        sl = slice(rank * self.B, (rank + 1) * self.B)
        self.off = sl.start
        self.dev = torch.device("cuda", self.ctx.device)
        T = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=self.dev)  # noqa
        x_last = np.asarray(x_last, np.float64)
        if x_last.shape != (n, N + 1, 9):   # the gather / builder kernels trust these extents
            raise ValueError("x_last: the first round's Last_xPredicted, (n, N+1, 9)")
        self.x0 = T(x0[sl])
        self.x_last = T(x_last[sl])
        self.u_last = T(np.asarray(u_last, np.float64)[sl])
        self.u_old = T(np.zeros((n, 2)) if u_old is None else np.asarray(u_old, np.float64))[sl].contiguous()
        self.nbr = T(nbr[sl], torch.int32)
        self.traj_all = T(x_last[:, :, 7:9] if traj is None else traj)
        # this rank's rows of the exchange buffer; an agent that is not advanced (no finite
        # solution) keeps them, so they start as the initial trajectories
        self.traj_local = self.traj_all[sl].clone()
        self.pose = torch.empty((self.B, N + 1, 2), dtype=torch.float64, device=self.dev)
        self.x_agents = torch.empty((self.B, N + 1, max(self.nb, 1), 2), dtype=torch.float64, device=self.dev)
        nz = 12 * (N + 1) + 4 * N
        self.z = torch.empty((self.B, nz), dtype=torch.float64, device=self.dev)
        self.planes = torch.zeros((self.B, N, 3, max(self.nb, 1)), dtype=torch.float64, device=self.dev)
        self.kkt = torch.empty(self.B, dtype=torch.float64, device=self.dev)
        self.iters = torch.empty(self.B, dtype=torch.int32, device=self.dev)
        self.status = torch.empty(self.B, dtype=torch.int32, device=self.dev)
        self.last_rows = N + 1
        self.rdims = L.cmpc_di_dims(self.B, N, self.nb, self.off)
        # agents of the latest round the reference calls infeasible (status not in {1, 2, -2})
        self.n_infeasible = torch.zeros(1, dtype=torch.int32, device=self.dev)

    def _stream(self):
        return ct.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def gather(self):
        lib = self.ctx.lib
        self.ctx.check(lib.cmpc_lpv_gather_dev(self.ctx.h, ct.byref(self.rdims), _tptr(self.nbr), _tptr(self.traj_all),
                                               _tptr(self.x_agents) if self.nb else None, _tptr(self.pose),
                                               self._stream()))

    def solve(self):
        lib, bp = self.ctx.lib, self.bp
        dims = L.cmpc_lpv_dims(self.B, self.N, self.nb, self.last_rows)
        data = L.cmpc_lpv_data(_tptr(self.x0), _tptr(self.x_last), _tptr(self.u_last), _tptr(self.u_old),
                               _tptr(self.x_agents) if self.nb else None, _tptr(self.pose))
        out = L.cmpc_lpv_out(_tptr(self.z), _tptr(self.planes) if self.nb else None, _tptr(self.kkt),
                             ct.cast(self.iters.data_ptr(), L._IP), ct.cast(self.status.data_ptr(), L._IP))
        self.ctx.check(lib.cmpc_solve_lpv_batch_dev(self.ctx.h, ct.byref(bp.prm), ct.byref(bp.track), ct.byref(dims),
                                                    ct.byref(data), ct.byref(out), ct.byref(bp.opts),
                                                    self._stream()))

    def advance(self):
        """x0 <- xPred[1], Last_xPredicted <- xPred[1:], uPred, u_old <- u_0, the exchanged X, Y; an agent
        without a finite solution keeps its state and trajectory; infeasible agents are counted."""
        self.n_infeasible.zero_()
        if self.last_rows == self.N + 1:
            # first round: Last_xPredicted goes from N + 1 rows per agent to N dense rows.  An agent the
            # advance leaves alone (no finite solution) must find its own previous rows in its dense
            # slot, not bytes of the (N + 1)-row layout: compact the layout first (rows 0..N-1)
            dense = self.x_last[:, :self.N, :].contiguous()
            self.x_last.view(-1)[:dense.numel()].copy_(dense.view(-1))
        self.ctx.check(self.ctx.lib.cmpc_lpv_advance_dev(self.ctx.h, ct.byref(self.rdims), _tptr(self.z),
                                                         _tptr(self.x0), _tptr(self.x_last), _tptr(self.u_last),
                                                         _tptr(self.u_old), _tptr(self.traj_local),
                                                         _tptr(self.status), _tptr(self.n_infeasible),
                                                         self._stream()))
        self.last_rows = self.N   # x_old = xPred[1:] from now on (LPV_HP_N_main.py:115)

    def exchange(self):
        exchange_positions(self.traj_all, self.traj_local, self.world, self.group, self.comm)

    def step(self, timer=None, halt=True):
        """One consensus round.  `timer` (start, stop) events bracket the build + solve launch.
        ``halt``: like the reference (LPV_HP_N_main.py:102-111, "QUIT..."), raise InfeasibleRound when an
        agent of this rank is infeasible (reads a device counter: one host synchronisation per round;
        ``halt=False`` leaves the check to the caller, ``infeasible()``)."""
        self.gather()
        if timer is not None:
            timer[0].record()
        self.solve()
        if timer is not None:
            timer[1].record()
        self.advance()
        self.exchange()
        if halt:
            bad = self.infeasible_all()
            if bad:
                raise InfeasibleRound(bad)

    def infeasible(self):
        """Infeasible agents of this rank in the latest round (synchronises)."""
        return int(self.n_infeasible.item())

    def infeasible_all(self):
        """Infeasible agents of every rank in the latest round (synchronises; collective when
        sharded).  The reference's loop quits for every agent at once (LPV_HP_N_main.py:102-111):
        each rank takes the halt decision on the node's count, so no rank breaks out of the loop
        while the others wait for it in the next round's all-gather."""
        if self.world == 1:
            return self.infeasible()
        if self.comm is not None:   # libcmpc's RCCL communicator (cmpc_comm_sum_i32)
            cnt = self.n_infeasible.clone()
            self.comm.sum_i32(cnt, self.torch.cuda.current_stream(self.dev))
            return int(cnt.item())
        import torch.distributed as dist

        cnt = self.n_infeasible.clone()
        if dist.get_backend(self.group) == "gloo":   # gloo reduces host tensors
            cnt = cnt.cpu()
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=self.group)
        return int(cnt.item())


class InfeasibleRound(RuntimeError):
    """A round left agents infeasible (status not in {1, 2, -2}, LPV_Planner.py:243-249); the
    reference stops the experiment there (LPV_HP_N_main.py:102-111)."""

    def __init__(self, count):
        super().__init__(f"{count} agent(s) infeasible in this round: QUIT (LPV_HP_N_main.py:102-111)")
        self.count = count


class LPVRoundsHandle:
    """The same rounds through the C ABI's round handle (cmpc_lpv_rounds_*): the library owns the
    device state; no torch.  What a MATLAB (MEX) or C host drives.  Arguments as LPVRounds;
    ``host_exchange``: the caller exchanges positions between steps (get_traj / set_traj)."""

    def __init__(self, bp, x0, x_last, u_last, nbr, u_old=None, traj=None, rank=0, world=1, host_exchange=False,
                 halt=True):
        self.bp, self.ctx = bp, bp.ctx
        x0 = L.f64(x0)
        n, N = x0.shape[0], bp.N
        nbr = L.i32(np.asarray(nbr).reshape(n, -1))
        if n % world:
            raise ValueError("agents must be divisible by the number of ranks")
        B = n // world
        sl = slice(rank * B, (rank + 1) * B)
        self.N, self.nb, self.B, self.n = N, nbr.shape[1], B, n
        flags = (L.CMPC_ROUNDS_HOST_EXCHANGE if host_exchange else 0) | (0 if halt else L.CMPC_ROUNDS_NO_HALT)
        self.dims = L.cmpc_lpv_rounds_dims(n, B, rank * B, N, self.nb, flags)
        keep = [L.f64(x0[sl]), L.f64(np.asarray(x_last)[sl]), L.f64(np.asarray(u_last)[sl]),
                None if u_old is None else L.f64(np.asarray(u_old)[sl]), L.i32(nbr[sl]),
                None if traj is None else L.f64(traj)]
        init = L.cmpc_lpv_rounds_init(L.dptr(keep[0]), L.dptr(keep[1]), L.dptr(keep[2]), L.dptr(keep[3]),
                                      L.iptr(keep[4]), L.dptr(keep[5]))
        h = ct.c_void_p()
        self.ctx.check(self.ctx.lib.cmpc_lpv_rounds_create(self.ctx.h, ct.byref(bp.prm), ct.byref(bp.track),
                                                           ct.byref(self.dims), ct.byref(init), ct.byref(bp.opts),
                                                           ct.byref(h)))
        self.h = h

    def step(self, rounds=1):
        """Runs up to `rounds` rounds; returns (rounds done, infeasible agents of the last one)."""
        done, bad = ct.c_int(), ct.c_int()
        self.ctx.check(self.ctx.lib.cmpc_lpv_rounds_step(self.h, int(rounds), ct.byref(done), ct.byref(bad)))
        return done.value, bad.value

    def read(self):
        nz = 12 * (self.N + 1) + 4 * self.N
        r = dict(z=np.zeros((self.B, nz)), kkt=np.zeros(self.B), iters=np.zeros(self.B, np.int32),
                 status=np.zeros(self.B, np.int32), x0=np.zeros((self.B, 9)),
                 planes=np.zeros((self.B, self.N, 3, self.nb)))
        o = L.cmpc_lpv_rounds_out(L.dptr(r["z"]), L.dptr(r["kkt"]), L.iptr(r["iters"]), L.iptr(r["status"]),
                                  L.dptr(r["x0"]), L.dptr(r["planes"]) if self.nb else None)
        self.ctx.check(self.ctx.lib.cmpc_lpv_rounds_read(self.h, ct.byref(o)))
        return r

    def get_traj(self):
        t = np.zeros((self.B, self.N + 1, 2))
        self.ctx.check(self.ctx.lib.cmpc_lpv_rounds_get_traj(self.h, L.dptr(t)))
        return t

    def set_traj(self, traj_all):
        t = L.f64(traj_all)
        if t.shape != (self.n, self.N + 1, 2):
            raise ValueError("traj_all: (n_total, N+1, 2)")
        self.ctx.check(self.ctx.lib.cmpc_lpv_rounds_set_traj(self.h, L.dptr(t)))

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.cmpc_lpv_rounds_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
