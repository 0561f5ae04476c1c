"""Reference-interface mirror of the LPV distributed planner.

``PlannerLPV`` has the constructor and ``solve`` signature of the reference's
``plan_lib.distributedPlanner.PlannerLPV`` (planner/lib/plan_lib/
distributedPlanner/LPV_Planner.py:15-182) and sets the same attributes
(xPred, uPred, duPred, sPred, raw_States, planes, weights, dist, OldSteering,
OldAccelera), so
an agent loop written against the reference runs unchanged.  Every call goes
through libcmpc's fused GPU path (cmpc_solve_lpv_batch): LPV scheduling,
hyperplanes, weights, QP build and the condensed interior-point solve all run
on the MI355X; the host only moves the inputs.

``PlannerLPVBatch`` is the hot-path form: one call solves every agent of a
control step (the inner loop of LPV_HP_N_main.py:99-106) in one launch.
"""
from __future__ import annotations

import ctypes as ct
import warnings

import numpy as np

from . import _lib as L

N_S, N_SLACK, N_U = 9, 3, 2
N_EXP = N_S + N_SLACK

# model / limit defaults of PlannerLPV when model_param / sys_lim are None (LPV_Planner.py:34-72)
DEFAULT_MODEL = dict(lf=0.12, lr=0.14, m=2.250, I=0.06, Cf=60.0, Cr=60.0, mu=0.05)
DEFAULT_LIMITS = dict(vx_ref=6.0, min_dist=0.45, max_vel=5.5, min_vel=0.2, max_rs=0.45, max_ls=0.45,
                      max_ac=4.0, max_dc=3.0, sm=0.9)


def lpv_params(Q, Qs, R, dR, dt, wq, model_param=None, sys_lim=None):
    mp = model_param or DEFAULT_MODEL
    sl = sys_lim or DEFAULT_LIMITS
    prm = L.cmpc_lpv_params()
    for k in ("lf", "lr", "m", "I", "Cf", "Cr", "mu"):
        setattr(prm, k, float(mp[k]))
    for k in ("vx_ref", "min_dist", "max_vel", "min_vel", "max_rs", "max_ls", "max_ac", "max_dc"):
        setattr(prm, k, float(sl[k]))
    prm.dt, prm.wq = float(dt), float(wq)
    Qs = np.asarray(Qs, float)
    if np.any(Qs != np.diag(np.diag(Qs))):
        raise ValueError("libcmpc eliminates slacks with a diagonal Schur complement: Qs must be diagonal")
    for i, v in enumerate(np.asarray(Q, float).ravel()):
        prm.Q[i] = v
    for i, v in enumerate(np.diag(Qs)):
        prm.Qs[i] = v
    for i, v in enumerate(np.asarray(R, float).ravel()):
        prm.R[i] = v
    for i, v in enumerate(np.asarray(dR, float).ravel()):
        prm.dR[i] = v
    return prm


def track_of(map_obj):
    """cmpc_track from any object with PointAndTangent (rows, 6, lanes), halfWidth and lane
    (the reference's Map, track_initialization.py:220-300)."""
    lane = int(getattr(map_obj, "lane", 0))
    tab = np.asarray(map_obj.PointAndTangent, float)[:, :, lane]
    keep = [L.f64(tab[:, 3]), L.f64(tab[:, 4]), L.f64(tab[:, 5]),
            L.f64(np.asarray(map_obj.halfWidth, float)[: tab.shape[0]])]
    tr = L.cmpc_track(tab.shape[0], *[L.dptr(a) for a in keep])
    return tr, keep


class PlannerLPVBatch:
    """All agents of one control step in one GPU call (same gains / map / horizon).
    ``riccati``: force the stage-wise Riccati solver (the default only when N*nu > 64);
    ``polish``: CMPC_FLAG_POLISH (default on, as the reference's OSQP polish=True)."""

    def __init__(self, Q, Qs, R, dR, N, dt, map, wq=0, model_param=None, sys_lim=None, ctx=None,
                 tol=None, max_iter=None, riccati=False, polish=True):
        self.N, self.dt, self.map = int(N), float(dt), map
        self.ctx = ctx or L.default_context()
        self.prm = lpv_params(Q, Qs, R, dR, dt, wq, model_param, sys_lim)
        self.track, self._track_keep = track_of(map)
        # rescue pass on: an agent whose condensed factorisation breaks down (theta ~ 1e18 on
        # saturated rows) is re-solved by the Riccati kernel instead of returning its best iterate;
        # polish on (OSQP's polish=True, LPV_Planner.py:233): a breakdown at the rounding floor has its
        # active set solved exactly
        self.opts = L.opts(tol, max_iter, L.CMPC_FLAG_RICCATI if riccati else
                           L.CMPC_FLAG_RESCUE | (L.CMPC_FLAG_POLISH if polish else 0))

    def solve(self, x0, x_last, u_last, u_old, x_agents, pose):
        """x0 (B,9); x_last (B,N or N+1,9); u_last (B,N,2); u_old (B,2);
        x_agents (B,N+1,nb,2) or None; pose (B,N+1,2).
        Returns dict(z (B,nz), planes (B,N,3,nb), kkt, iters, status)."""
        x0 = L.f64(x0)
        B = x0.shape[0]
        x_last, u_last, u_old, pose = L.f64(x_last), L.f64(u_last), L.f64(u_old), L.f64(pose)
        nb = 0 if x_agents is None else np.shape(x_agents)[2]
        xa = None if x_agents is None else L.f64(x_agents)
        N = self.N
        if x_last.shape[1] not in (N, N + 1):
            raise ValueError("Last_xPredicted must have N or N+1 rows")
        nz = N_EXP * (N + 1) + 2 * N_U * N
        z = np.zeros((B, nz))
        planes = np.zeros((B, N, 3, nb))
        kkt = np.zeros(B)
        iters = np.zeros(B, np.int32)
        status = np.zeros(B, np.int32)
        dims = L.cmpc_lpv_dims(B, N, nb, x_last.shape[1])
        data = L.cmpc_lpv_data(L.dptr(x0), L.dptr(x_last), L.dptr(u_last), L.dptr(u_old), L.dptr(xa), L.dptr(pose))
        out = L.cmpc_lpv_out(L.dptr(z), L.dptr(planes) if nb else None, L.dptr(kkt), L.iptr(iters), L.iptr(status))
        self.ctx.check(self.ctx.lib.cmpc_solve_lpv_batch(self.ctx.h, ct.byref(self.prm), ct.byref(self.track),
                                                         ct.byref(dims), ct.byref(data), ct.byref(out),
                                                         ct.byref(self.opts)))
        return dict(z=z, planes=planes, kkt=kkt, iters=iters, status=status)


    def build(self, x_last, u_last, x_agents, pose):
        """The builder alone on the GPU (cmpc_lpv_build_dev): the structured agent-QP the solve
        runs on.  Returns host arrays dict(A, B, qlin, C, h, planes, err)."""
        import torch

        x_last, u_last, pose = L.f64(x_last), L.f64(u_last), L.f64(pose)
        B = x_last.shape[0]
        N = self.N
        nb = 0 if x_agents is None else np.shape(x_agents)[2]
        dev = torch.device("cuda", self.ctx.device)
        T = lambda a: torch.as_tensor(a, device=dev)   # noqa: E731
        ins = dict(x_last=T(x_last), u_last=T(u_last), pose=T(pose),
                   x_agents=None if x_agents is None else T(L.f64(x_agents)))
        mc = 4 + nb
        outs = dict(A=torch.empty((B, N, 9, 9), dtype=torch.float64, device=dev),
                    B=torch.empty((B, N, 9, 2), dtype=torch.float64, device=dev),
                    qlin=torch.empty((B, N + 1, 9), dtype=torch.float64, device=dev),
                    C=torch.empty((B, N, mc, 9), dtype=torch.float64, device=dev),
                    h=torch.empty((B, N, mc), dtype=torch.float64, device=dev),
                    planes=torch.zeros((B, N, 3, max(nb, 1)), dtype=torch.float64, device=dev),
                    err=torch.empty(B, dtype=torch.int32, device=dev))
        dp = lambda t: None if t is None else ct.cast(t.data_ptr(), L._DP)   # noqa: E731
        dims = L.cmpc_lpv_dims(B, N, nb, x_last.shape[1])
        data = L.cmpc_lpv_data(None, dp(ins["x_last"]), dp(ins["u_last"]), None, dp(ins["x_agents"]), dp(ins["pose"]))
        o = L.cmpc_lpv_build_out(*[dp(outs[k]) for k in ("A", "B", "qlin", "C", "h")],
                                 dp(outs["planes"]) if nb else None, ct.cast(outs["err"].data_ptr(), L._IP))
        s = torch.cuda.current_stream(dev)
        self.ctx.check(self.ctx.lib.cmpc_lpv_build_dev(self.ctx.h, ct.byref(self.prm), ct.byref(self.track),
                                                       ct.byref(dims), ct.byref(data), ct.byref(o),
                                                       ct.c_void_p(s.cuda_stream)))
        torch.cuda.synchronize(dev)
        return {k: v.cpu().numpy() for k, v in outs.items()}


def unpack(z, N):
    """Solution unpacking of LPV_Planner.py:164-178 (xPred, uPred, duPred, sPred, raw_States).

    ``duPred`` keeps the reference's index expression verbatim (:175):
    ``n_exp(N+1) + arange(n_u N) + arange(n_u N)`` = base + 2 j, i.e. every other entry of
    the [u | du] block, so it holds the steering components of u_0..u_{N-1} followed by
    those of du_0..du_{N-1} — not the input rates.  Nothing downstream of the reference
    reads it; the true rates are z[base + n_u N : base + 2 n_u N] (``du_of``)."""
    xi = z[: N_EXP * (N + 1)].reshape(N + 1, N_EXP)
    x_pred = xi[:, :N_S].copy()
    s_pred = xi[1:, N_S:].copy()
    base = N_EXP * (N + 1)
    u_pred = z[base: base + N_U * N].reshape(N, N_U).copy()
    j = np.arange(N_U * N)
    du_pred = z[base + j + j].reshape(N, N_U).copy()
    return x_pred, u_pred, du_pred, s_pred, xi.copy()


def du_of(z, N):
    """The input rates du_0..du_{N-1} of a reference-layout solution (N, n_u)."""
    base = N_EXP * (N + 1) + N_U * N
    return z[base: base + N_U * N].reshape(N, N_U).copy()


def weights_of(pose, x_agents, min_dist):
    """compute_weights (utilities/misc.py:10-18): dist[h, i] = ||pose[h+1] - x_agents[h+1, i]||,
    weights = (2 D - dist) / nb, both (N, nb)."""
    pose = np.asarray(pose, float)
    xa = np.asarray(x_agents, float)
    nb = xa.shape[1]
    d = np.sqrt((pose[1:, None, 0] - xa[1:, :, 0]) ** 2 + (pose[1:, None, 1] - xa[1:, :, 1]) ** 2)
    return (2 * min_dist - d) / nb, d


def feasible_of(status):
    """OSQP status_val -> feasible flag exactly as LPV_Planner.py:246-248."""
    return 1 if status in (L.CMPC_SOLVED, L.CMPC_SOLVED_INACCURATE, L.CMPC_MAX_ITER_REACHED) else 0


class PlannerLPV:
    """Drop-in for plan_lib.distributedPlanner.PlannerLPV (one agent per call)."""

    def __init__(self, Q, Qs, R, dR, N, dt, map, id, wq=0, model_param=None, sys_lim=None, ctx=None):
        self.dR, self.n_s, self.slack, self.n_u = dR, N_S, N_SLACK, N_U
        self.n_exp = N_EXP
        self.id, self.dt, self.map, self.N = id, dt, map, N
        self.first_it = True
        self.OldSteering = [0.0]
        self.OldAccelera = [0.0]
        if Q.shape[0] != self.n_s:
            warnings.warn("Q has not the correct shape!, defaulting to identity of 9")
            Q = np.eye(self.n_s)
        if Qs.shape[0] != self.slack:
            warnings.warn("Qs has not the correct shape!, defaulting to identity of 3")
            Qs = np.eye(self.slack)
        if R.shape[0] != self.n_u:
            warnings.warn("R has not the correct shape!, defaulting to identity of 2")
            R = np.eye(self.n_u)
        self.Q, self.Qs, self.R, self.wq = Q, Qs, R, wq
        lim = sys_lim or DEFAULT_LIMITS
        self.min_dist = lim["min_dist"]
        self._batch = PlannerLPVBatch(Q, Qs, R, dR, N, dt, map, wq, model_param, sys_lim, ctx=ctx)

    def solve(self, x0, Last_xPredicted, uPred, x_agents, agents_id, pose):
        self.agent_list = agents_id
        if self.first_it:
            self.first_it = False
            self.n_agents = len(agents_id)
        u_old = [self.OldSteering[0], self.OldAccelera[0]]
        xa = None if x_agents is None else np.asarray(x_agents, float)[None]
        res = self._batch.solve(np.asarray(x0, float)[None], np.asarray(Last_xPredicted, float)[None],
                                np.asarray(uPred, float)[None], np.asarray(u_old, float)[None], xa,
                                np.asarray(pose, float)[None])
        status = int(res["status"][0])
        feasible = feasible_of(status)
        if status != L.CMPC_SOLVED:
            print("OSQP exited with status '%s'" % L.STATUS_TEXT.get(status, str(status)))
        if feasible == 0:
            print("QUIT...")
        Solution = res["z"][0]
        if status == L.CMPC_UNSOLVED and np.isnan(Solution).all():
            # the builder's track-segment lookup failed; the reference raises there (misc.py:97)
            raise ValueError("curvature/get_ey: s of the previous prediction lies on no single track segment")
        if x_agents is None:   # LPV_Planner.py:132-135
            self.planes = np.zeros((self.N, self.n_agents, 3))
            self.weights = np.ones((self.N, self.n_agents))
            self.dist = -self.weights
        else:                  # :137-139
            self.planes = res["planes"][0]
            self.weights, self.dist = weights_of(pose, x_agents, self.min_dist)
        self.xPred, self.uPred, self.duPred, self.sPred, self.raw_States = unpack(Solution, self.N)
        self.OldSteering = [self.uPred[0, 0]]
        self.OldAccelera = [self.uPred[0, 1]]
        self.kkt, self.iters, self.status = float(res["kkt"][0]), int(res["iters"][0]), status
        return feasible, Solution, self.planes
