"""Synthetic agent populations for BASELINE.json configs 1-5.

Double integrator x = [p (dim) | v (dim)], u = a (dim), dt = 0.025 (the
reference's sample time, planner/scripts/config_files/config_LPV.py:22).  Cost
and limits mirror the reference's roles (config_LPV.py:6-11, config/base_class.py:
30-41): 10 on (v_x - v_ref) with v_ref = 3.0, 25 on (p_y - lane), R = 0,
dR = 50 I, Qs = 1e7, accel 5 / decel 10 on a_x and |a| <= 5 on the others,
soft speed cap 5.5, soft lane half-width 0.75 (Highway halfWidth,
mapManager/track_initialization.py:112), soft collision half-planes d = 0.25,
coverage weight wq = 5.

Agents sit on a straight 3-lane road: p_x = 0.5 floor(i/3) + U(-.05,.05),
p_y = {-0.5, 0, 0.5}[i%3] + U(-.05,.05), v_x ~ U(1.0, 1.6), v_y = 0, drawn from
numpy.random.default_rng(20240101) in that order.  Neighbours: the nb nearest
agents by initial position (fixed graph).  Previous predictions: constant-velocity
rollout, as initialise_agents does (utilities/misc.py:155-210).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

DT = 0.025
SEED = 20240101
LANES = (-0.5, 0.0, 0.5)


def di_params(dim=2):
    return dict(dim=dim, v_ref=3.0, q_v=10.0, q_lane=25.0, hw=0.75, min_vel=0.0, max_vel=5.5,
                min_dist=0.25, wq=5.0)


def di_shared(dim, N, nb):
    nx, nu = 2 * dim, dim
    prm = di_params(dim)
    Q = np.zeros((nx, nx))
    Q[1, 1] = prm["q_lane"]
    Q[dim, dim] = prm["q_v"]
    ub = np.full(nu, 5.0)
    lb = np.full(nu, -5.0)
    lb[0] = -10.0
    return dict(nx=nx, nu=nu, N=N, ns=3, mc=4 + nb, Q=Q, R=np.zeros((nu, nu)), dR=50.0 * np.eye(nu),
                Qs=np.full(3, 1e7), u_ub=ub, u_lb=lb,
                row_slack=np.array([-1, 0, 1, 1] + [2] * nb, np.int32),
                row_sign=np.array([1, 1, 1, 1] + [-1] * nb, np.int32))


def di_dynamics(dim, dt=DT):
    I = np.eye(dim)
    A = np.block([[I, dt * I], [np.zeros((dim, dim)), I]])
    B = np.vstack([0.5 * dt * dt * I, dt * I])
    return A, B


@dataclass
class DIScenario:
    dim: int
    N: int
    nb: int
    n_agents: int
    params: dict
    shared: dict
    A: np.ndarray       # (n, N, nx, nx)
    B: np.ndarray       # (n, N, nx, nu)
    x0: np.ndarray      # (n, nx)
    u_prev: np.ndarray  # (n, nu)
    lane: np.ndarray    # (n,)
    nbr: np.ndarray     # (n, nb) int32 global indices
    traj: np.ndarray    # (n, N+1, 2) previous predicted positions
    extra: dict = field(default_factory=dict)

    def shard(self, rank, world):
        """Contiguous block of agents owned by `rank` (agents are ordered along the road,
        so most neighbours live on the same GPU)."""
        per = self.n_agents // world
        return slice(rank * per, (rank + 1) * per)


def nearest_neighbours(pos, nb):
    from scipy.spatial import cKDTree

    n = pos.shape[0]
    if nb == 0:
        return np.zeros((n, 0), np.int32)
    if nb >= n:
        raise ValueError("need more agents than neighbours")
    _, idx = cKDTree(pos).query(pos, k=nb + 1)
    out = np.zeros((n, nb), np.int32)
    for i in range(n):
        row = [j for j in idx[i] if j != i][:nb]
        out[i] = row
    return out


def make_di(n_agents, N, nb=2, dim=2, seed=SEED):
    rng = np.random.default_rng(seed)
    nx, nu = 2 * dim, dim
    i = np.arange(n_agents)
    ds = rng.uniform(-0.05, 0.05, n_agents)
    dl = rng.uniform(-0.05, 0.05, n_agents)
    vx = rng.uniform(1.0, 1.6, n_agents)
    lane = np.array([LANES[k % 3] for k in i])
    x0 = np.zeros((n_agents, nx))
    x0[:, 0] = 0.5 * (i // 3) + ds
    x0[:, 1] = lane + dl
    x0[:, dim] = vx
    Ad, Bd = di_dynamics(dim)
    A = np.broadcast_to(Ad, (n_agents, N, nx, nx)).copy()
    B = np.broadcast_to(Bd, (n_agents, N, nx, nu)).copy()
    k = np.arange(N + 1)[None, :]
    traj = np.stack([x0[:, 0:1] + k * DT * x0[:, dim:dim + 1],
                     x0[:, 1:2] + k * DT * x0[:, dim + 1:dim + 2]], axis=-1)
    nbr = nearest_neighbours(x0[:, :2], nb)
    return DIScenario(dim, N, nb, n_agents, di_params(dim), di_shared(dim, N, nb), A, B, x0,
                      np.zeros((n_agents, nu)), lane, nbr, traj)


def di_alg_bytes(nx, nu, N, nb, word=8):
    """Algorithmic HBM bytes per agent-QP (SURVEY.md §8d formula)."""
    return word * (N * (nx * nx + nx * nu) + (N + 1) * nx + N * nu + nx + nu + (N + 1) + 2 * nb * (N + 1)
                   + N * nu + (N + 1) * nx + 3 * N + 2)


def riccati_flops(nx, nu, N, iters):
    """Algorithmic flops per agent-QP of the stage-wise Riccati method (mpc_riccati.hip): per IPM
    iteration one factorisation, N x (P[A|B] + [A|B]'T + Hvy'K: 2 na nc nx + nc^2 nx + na^2 nu,
    na = nc = nx + nu), and two Newton solves of 2 sweeps each (4 N (2 nx na)), plus the two
    residual adjoints (2 N 2 nx (nx + nu)).  Used for cfg5's roofline instead of the condensed
    count, which would credit the Riccati kernel with work it does not do."""
    na = nx + nu
    per_it = N * (2 * na * na * nx + na * na * nx + na * na * nu) + 4 * N * 2 * nx * na + 2 * N * 2 * nx * na
    return iters * per_it


def alg_flops(nx, nu, N, ncons, iters):
    """Algorithmic flops per agent-QP: condensing + iters x (G'WG + Cholesky + ...)."""
    n = N * nu
    condense = 2 * N * N * nx * nx * nu + N * nx * n * n + 4 * N * nx * n
    per_it = N * nx * n * n + n ** 3 / 3 + 4 * n * n + 2 * ncons * n
    return condense + iters * per_it
