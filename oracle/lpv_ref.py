"""ORACLE (test infrastructure only) — numpy restatement of the reference's
per-agent LPV-DMPC QP assembly and control loop.

Every function cites the reference file:line it restates (paths relative to
``/root/reference/planner/lib/plan_lib`` unless they start with ``planner/``).
All arithmetic is IEEE float64, as in the reference (numpy default).

This module is pinned by ``tests/test_oracle_lpv.py`` against QPs captured from
the reference's own ``PlannerLPV`` (tests/golden/lpv_*.npz, made by
``oracle/gen_fixtures.py``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# --------------------------------------------------------------------------
# Parameters (config/base_class.py:19-41 "SCALED CAR"; scripts config_LPV.py:6-23)
# --------------------------------------------------------------------------

SCALED_CAR_MODEL = dict(lf=0.125, lr=0.125, m=1.98, I=0.09, Cf=70.0, Cr=70.0, mu=0.05)


def scaled_car_limits(vx_ref=3.0):
    """``experiment_utilities.sys_lim`` for model "SCALED CAR" (base_class.py:30-41)."""
    return dict(vx_ref=vx_ref, min_dist=0.25, max_vel=5.5, min_vel=0.0, max_rs=0.3,
                max_ls=0.3, max_ac=5.0, max_dc=10.0, sm=0.9)


def paper_gains():
    """Gains of ``planner/scripts/config_files/config_LPV.py:6-11``."""
    return dict(Q=np.diag([10.0, 0.0, 0.0, 25.0, 10.0, 0.0, 0.0, 0.0, 0.0]),
                Qs=10000000.0 * np.eye(3), R=0.0 * np.eye(2), dR=50.0 * np.eye(2), wq=5.0)


# x0_database (config/__init__.py:3-7): [vx vy psidot ey epsi theta s X Y]
X0_DATABASE = [
    [1.3, -0.16, 0.00, 0.0, 0, 0.0, 0, 0.0, 1.0],
    [1.3, -0.16, 0.00, -0.25, 0, 0.0, 0, 0.0, 1.0],
    [1.3, -0.16, 0.00, 0.45, 0, 0.0, 0, 0.0, 1.45],
    [1.3, -0.16, 0.00, 0.25, 0, 0.0, 0.25, 0.0, 1.5],
]

# --------------------------------------------------------------------------
# Track (mapManager/track_initialization.py:10-300)
# --------------------------------------------------------------------------

_PI = np.pi


def _wrap(a):  # track_initialization.py:566-574
    if a < -_PI:
        return 2 * _PI + a
    if a > _PI:
        return a - 2 * _PI
    return a


def _sgn(a):  # track_initialization.py:577-582 (0 counts as positive)
    return 1 if a >= 0 else -1


def _track_spec(name):
    """(segments[len, radius] per lane, halfWidth, open) — track_initialization.py:23-215."""
    if name == "Highway":  # :98-113
        seg = 2 * np.array([[0.0, 0], [1.0, 0], [4.5, 4.5 / (0.5 * _PI)], [2.0, 0],
                            [2.5, -2.5 / (0.5 * _PI)], [2.0, 0], [4.5, 4.5 / _PI], [2.0, 0],
                            [5.0, 0], [0.0, 0]])
        return [seg], 0.75 * np.ones(10), True
    if name == "oval":  # :41-50
        seg = np.array([[2.0, 0], [5.85, 5.85 / _PI], [4.0, 0], [5.85, 5.85 / _PI], [2.0, 0]])
        return [seg], np.full(6, 0.55), False
    if name == "Oval2":  # :63-79 (two lanes; the reference's "3110" spec is 2-D and fails at :221)
        seg0 = 2 * np.array([[1.0, 0], [4.5, 4.5 / _PI], [2.0, 0], [4.5, 4.5 / _PI], [1.0, 0]])
        seg1 = np.array([[2.0, 0], [5.85, 5.85 / _PI], [4.0, 0], [5.85, 5.85 / _PI], [2.0, 0]])
        return [seg0, seg1], 0.5 * np.ones(5), False
    if name == "SL":  # :115-133
        seg = 2 * np.array([[0.0, 0], [3.0, 0], [1.0, 0], [1.0, 0], [1.0, 0], [1.0, 0], [1.0, 0],
                            [1.0, 0], [1.0, 0], [1.0, 0], [2.0, 0], [3.0, 0]])
        hw = np.asarray([0.75, 0.75, 0.65, 0.65, 0.55, 0.35, 0.35, 0.55, 0.65, 0.65, 0.75, 0.75])
        return [seg], hw, True
    raise KeyError(name)


@dataclass
class Track:
    """Restatement of ``Map`` (track_initialization.py:10-300): only what the QP reads.

    ``PointAndTangent[i] = [x_end, y_end, psi_end, s_start, length, curvature]``.
    """
    name: str
    PointAndTangent: np.ndarray          # (rows, 6, lanes)
    halfWidth: np.ndarray
    open: bool
    TrackLength: np.ndarray
    lane: int = 0

    @classmethod
    def build(cls, name):
        lanes, hw, is_open = _track_spec(name)
        y_start = [2 * hw[0], 4 * hw[0]]                       # :227
        nseg = lanes[0].shape[0]
        tab = np.zeros((nseg + (0 if is_open else 1), 6, len(lanes)))
        tlen = np.zeros(len(lanes))
        for k, seg in enumerate(lanes):
            for i in range(nseg):
                length, radius = seg[i]
                s0 = 0.0 if i == 0 else tab[i - 1, 3, k] + tab[i - 1, 4, k]
                ang = 0.0 if i == 0 else tab[i - 1, 2, k]
                if radius == 0.0:                              # straight, :231-248
                    xs, ys = (0.0, y_start[k]) if i == 0 else (tab[i - 1, 0, k], tab[i - 1, 1, k])
                    tab[i, :, k] = [xs + length * np.cos(ang), ys + length * np.sin(ang), ang,
                                    s0, length, 0.0]
                else:                                          # arc, :249-285
                    d = 1 if radius >= 0 else -1
                    # quirk: the first-segment arc centre is taken from (0, 0), :259-263
                    bx, by = (0.0, 0.0) if i == 0 else (tab[i - 1, 0, k], tab[i - 1, 1, k])
                    cx = bx + np.abs(radius) * np.cos(ang + d * _PI / 2)
                    cy = by + np.abs(radius) * np.sin(ang + d * _PI / 2)
                    span = length / np.abs(radius)
                    psi = _wrap(ang + span * np.sign(radius))
                    nrm = _wrap(d * _PI / 2 + ang)
                    a0 = -(_PI - np.abs(nrm)) * _sgn(nrm)
                    tab[i, :, k] = [cx + np.abs(radius) * np.cos(a0 + d * span),
                                    cy + np.abs(radius) * np.sin(a0 + d * span), psi,
                                    s0, length, 1 / radius]
            if not is_open:                                    # closing segment, :287-297
                xs, ys = tab[-2, 0, k], tab[-2, 1, k]
                tab[-1, :, k] = [0.0, y_start[k], 0.0, tab[-2, 3, k] + tab[-2, 4, k],
                                 np.sqrt((0.0 - xs) ** 2 + (y_start[k] - ys) ** 2), 0.0]
            tlen[k] = tab[-1, 3, k] + tab[-1, 4, k]
        return cls(name, tab, hw, is_open, tlen)

    # -- track_initialization.py:305-317
    def wrap_s(self, s):
        if not self.open:
            while s >= self.TrackLength[self.lane]:
                s = s - self.TrackLength[self.lane]
        elif s >= self.TrackLength[self.lane]:
            s = s - self.TrackLength[self.lane]
        return 0 if s < 0 else s

    def segment(self, s):
        """Index of the segment containing s, or raise like the reference does
        (``int(np.where(...)[0])`` on an empty/multiple match, misc.py:97,123)."""
        t = self.PointAndTangent[:, :, self.lane]
        hit = np.nonzero((s >= t[:, 3]) & (s < t[:, 3] + t[:, 4]))[0]
        if hit.size != 1:
            raise ValueError(f"s={s} matches {hit.size} segments")
        return int(hit[0])

    def getGlobalPosition(self, s, ey):
        """(s, ey) -> (X, Y, theta) — track_initialization.py:325-399 (plotting=False)."""
        s = self.wrap_s(s)
        t = self.PointAndTangent[:, :, self.lane]
        i = self.segment(s)
        if t[i, 5] == 0.0:
            xf, yf, psi = t[i, 0], t[i, 1], t[i, 2]
            xs, ys = t[i - 1, 0], t[i - 1, 1]
            frac = (s - t[i, 3]) / t[i, 4]
            x = (1 - frac) * xs + frac * xf + ey * np.cos(psi + _PI / 2)
            y = (1 - frac) * ys + frac * yf + ey * np.sin(psi + _PI / 2)
            return x, y, psi
        r = 1 / t[i, 5]
        ang = t[i - 1, 2]
        d = 1 if r >= 0 else -1
        cx = t[i - 1, 0] + np.abs(r) * np.cos(ang + d * _PI / 2)
        cy = t[i - 1, 1] + np.abs(r) * np.sin(ang + d * _PI / 2)
        span = (s - t[i, 3]) / (_PI * np.abs(r)) * _PI
        nrm = _wrap(d * _PI / 2 + ang)
        a0 = -(_PI - np.abs(nrm)) * _sgn(nrm)
        x = cx + (np.abs(r) - d * ey) * np.cos(a0 + d * span)
        y = cy + (np.abs(r) - d * ey) * np.sin(a0 + d * span)
        return x, y, ang + d * span


def _wrap_lap(s, tab):
    """misc.py:84-91 / 114-119: subtract whole laps, clamp negatives."""
    L = tab[-1, 3] + tab[-1, 4]
    while s > L:
        s = s - L
    return 0 if s < 0 else s


def curvature(s, track):
    """misc.py:78-101."""
    tab = track.PointAndTangent[:, :, track.lane]
    s = _wrap_lap(s, tab)
    hit = np.nonzero((s >= tab[:, 3]) & (s < tab[:, 3] + tab[:, 4]))[0]
    if hit.size != 1:
        raise ValueError(f"curvature: s={s} matches {hit.size} segments")
    return tab[hit[0], 5]


def get_ey(s_vec, track, sm=1.0):
    """misc.py:105-126 (half-width of the segment containing each s, times sm)."""
    tab = track.PointAndTangent[:, :, track.lane]
    out = np.zeros(len(s_vec))
    for j, s in enumerate(s_vec):
        s = _wrap_lap(s, tab)
        hit = np.nonzero((s >= tab[:, 3]) & (s < tab[:, 3] + tab[:, 4]))[0]
        if hit.size != 1:
            raise ValueError(f"get_ey: s={s} matches {hit.size} segments")
        out[j] = track.halfWidth[hit[0]] * sm
    return out


# --------------------------------------------------------------------------
# Hyperplanes and coverage weights
# --------------------------------------------------------------------------

def compute_hyperplane(agents, pose, horizon, ego_id=0, agents_id=None, keep_sign=True):
    """planes[h, :, n] = sign*[a_x, a_y, b] with a = unit(p_n - p_ego),
    b = -0.5 a.(p_ego + p_n) — planes/compute_plane.py:41-68."""
    nb = agents.shape[1]
    out = np.zeros((horizon, 3, nb))
    for h in range(horizon):
        for n in range(nb):
            pe = pose[h, :]
            pn = agents[h, n, :]
            a = pn - pe
            a = a / np.sqrt(a[0] ** 2 + a[1] ** 2)
            b = -0.5 * a @ (pe + pn).T
            sgn = 1 if (keep_sign or ego_id < agents_id[n]) else -1
            out[h, 0, n] = sgn * a[0]
            out[h, 1, n] = sgn * a[1]
            out[h, 2, n] = sgn * b
    return out


def compute_weights(pose, neigh, D):
    """misc.py:10-18 (+ EuDistance :21-25): rows 1..N of the trajectories."""
    nb = neigh.shape[1]
    dist = np.empty((pose.shape[0] - 1, nb))
    w = np.empty_like(dist)
    for i in range(nb):
        p1 = pose[1:]
        p2 = neigh[1:, i, :]
        dist[:, i] = np.sqrt((p1[:, 0] - p2[:, 0]) ** 2 + (p1[:, 1] - p2[:, 1]) ** 2)
        w[:, i] = (2 * D - dist[:, i]) / nb
    return w, dist


# --------------------------------------------------------------------------
# LPV scheduling (distributedPlanner/LPV_Planner.py:477-591)
# --------------------------------------------------------------------------

def estimate_abc(states, u, N, dt, prm, track):
    """Returns A (N,9,9), B (N,9,2), ey_hor (len(states))."""
    lf, lr, m, I, Cf, Cr, mu = (prm[k] for k in ("lf", "lr", "m", "I", "Cf", "Cr", "mu"))
    ey_hor = get_ey(states[:, 6], track)                      # :491 (sm = 1)
    A = np.zeros((N, 9, 9))
    B = np.zeros((N, 9, 2))
    for i in range(N):
        vx, vy, ey, epsi, theta, s = (states[i, j] for j in (0, 1, 3, 4, 5, 6))
        cur = curvature(s, track)
        delta = u[i, 0]
        if vx < 0.2:                                           # :505-517
            A12 = A13 = A22 = A23 = A32 = A33 = B11 = 0.0
        else:                                                  # :521-531
            A12 = (np.sin(delta) * Cf) / (m * vx)
            A13 = (np.sin(delta) * Cf * lf) / (m * vx) + vy
            A22 = -(Cr + Cf * np.cos(delta)) / (m * vx)
            A23 = -(lf * Cf * np.cos(delta) - lr * Cr) / (m * vx) - vx
            A32 = -(lf * Cf * np.cos(delta) - lr * Cr) / (I * vx)
            A33 = -(lf * lf * Cf * np.cos(delta) + lr * lr * Cr) / (I * vx)
            B11 = -(np.sin(delta) * Cf) / m
        den = 1 - ey * cur
        Ac = np.zeros((9, 9))
        Ac[0, 0], Ac[0, 1], Ac[0, 2] = -mu, A12, A13
        Ac[1, 1], Ac[1, 2] = A22, A23
        Ac[2, 1], Ac[2, 2] = A32, A33
        Ac[3, 0], Ac[3, 1] = np.sin(epsi), np.cos(epsi)
        Ac[4, 0] = (1 / den) * (-np.cos(epsi) * cur)
        Ac[4, 1] = (1 / den) * (np.sin(epsi) * cur)
        Ac[4, 2] = 1.0
        Ac[5, 2] = 1.0
        Ac[6, 0], Ac[6, 1] = np.cos(epsi) / den, -np.sin(epsi) / den
        Ac[7, 0], Ac[7, 1] = np.cos(theta), -np.sin(theta)
        Ac[8, 0], Ac[8, 1] = np.sin(theta), np.cos(theta)
        Bc = np.zeros((9, 2))
        Bc[0, 0], Bc[0, 1] = B11, 1.0
        Bc[1, 0] = (np.cos(delta) * Cf) / m
        Bc[2, 0] = (lf * Cf * np.cos(delta)) / I
        A[i] = np.eye(9) + dt * Ac                             # :583
        B[i] = dt * Bc                                         # :584
    return A, B, ey_hor


# --------------------------------------------------------------------------
# QP assembly (LPV_Planner.py:251-475) — reference form
#   z = [xi_0 .. xi_N | u_0 .. u_{N-1} | du_0 .. du_{N-1}],  xi_k = [x_k(9) | sigma_k(3)]
# --------------------------------------------------------------------------

NS, NSL, NU = 9, 3, 2
NEXP = NS + NSL


def build_ineq(N, lim, planes, ey):
    """F z <= b — LPV_Planner.py:279-380 with GenerateColisionAvoidanceConstraints :251-276."""
    nb = planes.shape[2]
    ey = np.append(ey, ey[-1]) if ey.shape[0] < N else ey[:N]        # :310-313
    nz = NEXP * (N + 1) + 2 * NU * N
    rows_x = 4 + nb
    F = np.zeros((N * rows_x + 4 * N, nz))
    b = np.zeros(N * rows_x + 4 * N)
    for k in range(1, N + 1):
        r0 = (k - 1) * rows_x
        c0 = k * NEXP
        F[r0 + 0, c0 + 0] = -1.0;                b[r0 + 0] = -lim["min_vel"]
        F[r0 + 1, c0 + 0] = 1.0; F[r0 + 1, c0 + 9] = 1.0;  b[r0 + 1] = lim["max_vel"]
        F[r0 + 2, c0 + 3] = 1.0; F[r0 + 2, c0 + 10] = 1.0; b[r0 + 2] = ey[k - 1]
        F[r0 + 3, c0 + 3] = -1.0; F[r0 + 3, c0 + 10] = 1.0; b[r0 + 3] = ey[k - 1]
        for i in range(nb):
            F[r0 + 4 + i, c0 + 7] = planes[k - 1, 0, i]
            F[r0 + 4 + i, c0 + 8] = planes[k - 1, 1, i]
            F[r0 + 4 + i, c0 + 11] = -1.0
            b[r0 + 4 + i] = -lim["min_dist"] / 2 - planes[k - 1, 2, i]
    cu = NEXP * (N + 1)
    for k in range(N):
        r0 = N * rows_x + 4 * k
        F[r0 + 0, cu + 2 * k] = 1.0;  b[r0 + 0] = lim["max_rs"]
        F[r0 + 1, cu + 2 * k] = -1.0; b[r0 + 1] = lim["max_ls"]
        F[r0 + 2, cu + 2 * k + 1] = 1.0;  b[r0 + 2] = lim["max_ac"]
        F[r0 + 3, cu + 2 * k + 1] = -1.0; b[r0 + 3] = lim["max_dc"]
    return F, b


def build_cost(N, gains, vx_ref, weights, planes):
    """P = 2 blkdiag(Qt^(N+1), R^N, dR^N), q = 2 p — LPV_Planner.py:382-427, _buildQ :107-113."""
    Qt = np.zeros((NEXP, NEXP))
    Qt[:NS, :NS] = gains["Q"]
    Qt[NS:, NS:] = gains["Qs"]
    nz = NEXP * (N + 1) + 2 * NU * N
    M = np.zeros((nz, nz))
    for k in range(N + 1):
        M[k * NEXP:(k + 1) * NEXP, k * NEXP:(k + 1) * NEXP] = Qt
    cu = NEXP * (N + 1)
    for k in range(N):
        M[cu + 2 * k:cu + 2 * k + 2, cu + 2 * k:cu + 2 * k + 2] = gains["R"]
        cd = cu + 2 * N + 2 * k
        M[cd:cd + 2, cd:cd + 2] = gains["dR"]
    p = np.zeros(nz)
    for k in range(N + 1):
        p[k * NEXP] = -vx_ref * gains["Q"][0, 0]
    nb = planes.shape[2]
    for t in range(1, N + 1):
        for i in range(nb):
            p[t * NEXP + 7] += gains["wq"] * weights[t - 1, i] * planes[t - 1, 0, i]
            p[t * NEXP + 8] += gains["wq"] * weights[t - 1, i] * planes[t - 1, 1, i]
    return 2 * M, 2 * p


def build_eq(N, A, B):
    """G z = E x0 + Eu uOld — LPV_Planner.py:429-475 (slack rows are 0 = 0)."""
    nz = NEXP * (N + 1) + 2 * NU * N
    G = np.zeros((NEXP * (N + 1) + NU * N, nz))
    for k in range(N + 1):
        G[k * NEXP:k * NEXP + NS, k * NEXP:k * NEXP + NS] = np.eye(NS)
    cu = NEXP * (N + 1)
    for k in range(1, N + 1):
        G[k * NEXP:k * NEXP + NS, (k - 1) * NEXP:(k - 1) * NEXP + NS] = -A[k - 1]
        G[k * NEXP:k * NEXP + NS, cu + (k - 1) * NU:cu + k * NU] = -B[k - 1]
    r = NEXP * (N + 1)
    cd = cu + NU * N
    G[r:r + 2, cu:cu + 2] = np.eye(2)
    G[r:r + 2, cd:cd + 2] = -np.eye(2)
    for i in range(1, N):
        G[r + 2 * i:r + 2 * i + 2, cu + 2 * (i - 1):cu + 2 * i] = np.eye(2)
        G[r + 2 * i:r + 2 * i + 2, cu + 2 * i:cu + 2 * i + 2] = -np.eye(2)
        G[r + 2 * i:r + 2 * i + 2, cd + 2 * i:cd + 2 * i + 2] = np.eye(2)
    E = np.zeros((G.shape[0], NS))
    E[:NS, :NS] = np.eye(NS)
    Eu = np.zeros((G.shape[0], NU))
    Eu[r:r + 2, :] = np.eye(2)
    return G, E, Eu


@dataclass
class LPVQP:
    """OSQP-form QP as ``osqp_solve_qp`` hands it to OSQP (LPV_Planner.py:222-233):
    min 1/2 z'Pz + q'z  s.t.  l <= A z <= u,  A = [F; G], l = [-inf; beq], u = [b; beq]."""
    P: np.ndarray
    q: np.ndarray
    A: np.ndarray
    l: np.ndarray
    u: np.ndarray
    planes: np.ndarray = None
    Adyn: np.ndarray = None
    Bdyn: np.ndarray = None
    ey: np.ndarray = None
    weights: np.ndarray = None
    extra: dict = field(default_factory=dict)


def assemble(x0, x_last, u_last, x_agents, pose, u_old, N, dt, track, prm, lim, gains):
    """One ``PlannerLPV.solve`` up to the solver call (LPV_Planner.py:115-157)."""
    if x_agents is None:                                        # :132-135
        nb = 0
        planes = np.zeros((N, 3, 0))
        weights = np.ones((N, 0))
    else:
        nb = x_agents.shape[1]
        planes = compute_hyperplane(x_agents, pose, N, keep_sign=True)   # :138
        weights, _ = compute_weights(pose, x_agents, lim["min_dist"])    # :139
    A, B, ey = estimate_abc(np.asarray(x_last, float), np.asarray(u_last, float), N, dt, prm, track)
    F, b = build_ineq(N, lim, planes, ey)
    G, E, Eu = build_eq(N, A, B)
    P, q = build_cost(N, gains, lim["vx_ref"], weights, planes)
    beq = E @ np.asarray(x0, float) + Eu @ np.asarray(u_old, float)
    Aqp = np.vstack([F, G])
    l = np.hstack([-np.inf * np.ones(len(b)), beq])
    u = np.hstack([b, beq])
    return LPVQP(P, q, Aqp, l, u, planes, A, B, ey, weights)


def unpack(z, N):
    """Solution unpacking, LPV_Planner.py:164-180 (duPred bug not reproduced: unused)."""
    xi = z[:NEXP * (N + 1)].reshape(N + 1, NEXP)
    x_pred = xi[:, :NS].copy()
    s_pred = xi[1:, NS:].copy()
    u_pred = z[NEXP * (N + 1):NEXP * (N + 1) + NU * N].reshape(N, NU).copy()
    return x_pred, u_pred, s_pred


# --------------------------------------------------------------------------
# Initialisation + loop (utilities/misc.py:155-210; planner/scripts/LPV_HP_N_main.py:81-117)
# --------------------------------------------------------------------------

def predicted_vectors_generation(Hp, x0, dt, track, accel_rate=0.0):
    """misc.py:168-210 (S[0] = 0; X, Y, theta from the map with a one-sample lag)."""
    xx = np.zeros((Hp + 1, 9))
    xx[0, 0], xx[0, 1], xx[0, 2], xx[0, 3], xx[0, 4] = x0[0], x0[1], x0[2], x0[3], x0[4]
    xx[0, 6] = 0.0
    gx, gy, gth = track.getGlobalPosition(0.0, xx[0, 3])
    xx[0, 5], xx[0, 7], xx[0, 8] = gth, gx, gy
    xx[1:, 1], xx[1:, 2], xx[1:, 3], xx[1:, 4] = x0[1], x0[2], x0[3], x0[4]
    acc = 1.0 + np.array([accel_rate * i for i in range(Hp)])
    for i in range(Hp):
        xx[i + 1, 0] = xx[i, 0] + acc[i] * dt
        xx[i + 1, 6] = xx[i, 6] + xx[i, 0] * dt
        gx, gy, gth = track.getGlobalPosition(xx[i, 6], xx[i, 3])
        xx[i + 1, 7], xx[i + 1, 8], xx[i + 1, 5] = gx, gy, gth
    return xx, np.zeros((Hp, 2))


def initialise_agents(x0s, Hp, dt, track):
    """misc.py:155-165."""
    n = len(x0s)
    agents = np.zeros((Hp + 1, n, 2))
    xs, us = [], []
    for i, x0 in enumerate(x0s):
        xx, uu = predicted_vectors_generation(Hp, x0, dt, track)
        xs.append(xx)
        us.append(uu)
        agents[:, i, :] = xx[:, -2:]
    return agents, xs, us


def neighbour_lists(n):
    """All other agents, LPV_HP_N_main.py:82-85."""
    return [[j for j in range(n) if j != i] for i in range(n)]


# --------------------------------------------------------------------------
# Structured (per-stage) statement of the same QP — the form the condensed
# solvers (oracle/cmpc_oracle.c and the HIP product) consume.  Row order per
# stage and the input-row order follow build_ineq exactly.
# --------------------------------------------------------------------------

def structured(qp, x0, u_old, N, lim, gains):
    nb = qp.planes.shape[2]
    mc = 4 + nb
    ey = qp.ey
    ey = np.append(ey, ey[-1]) if ey.shape[0] < N else ey[:N]
    C = np.zeros((N, mc, NS))
    h = np.zeros((N, mc))
    C[:, 0, 0] = -1.0; h[:, 0] = -lim["min_vel"]
    C[:, 1, 0] = 1.0;  h[:, 1] = lim["max_vel"]
    C[:, 2, 3] = 1.0;  h[:, 2] = ey
    C[:, 3, 3] = -1.0; h[:, 3] = ey
    for i in range(nb):
        C[:, 4 + i, 7] = qp.planes[:, 0, i]
        C[:, 4 + i, 8] = qp.planes[:, 1, i]
        h[:, 4 + i] = -lim["min_dist"] / 2 - qp.planes[:, 2, i]
    p = np.zeros((N + 1, NS))
    p[:, 0] = -lim["vx_ref"] * gains["Q"][0, 0]
    for t in range(1, N + 1):
        for i in range(nb):
            p[t, 7] += gains["wq"] * qp.weights[t - 1, i] * qp.planes[t - 1, 0, i]
            p[t, 8] += gains["wq"] * qp.weights[t - 1, i] * qp.planes[t - 1, 1, i]
    return dict(nx=NS, nu=NU, N=N, ns=NSL, mc=mc,
                Q=np.array(gains["Q"], float), R=np.array(gains["R"], float),
                dR=np.array(gains["dR"], float), Qs=np.diag(gains["Qs"]).astype(float),
                u_ub=np.array([lim["max_rs"], lim["max_ac"]], float),
                u_lb=np.array([-lim["max_ls"], -lim["max_dc"]], float),
                row_slack=np.array([-1, 0, 1, 1] + [2] * nb, np.int32),
                row_sign=np.array([1, 1, 1, 1] + [-1] * nb, np.int32),
                A=qp.Adyn[None].copy(), B=qp.Bdyn[None].copy(),
                x0=np.asarray(x0, float)[None].copy(), u_prev=np.asarray(u_old, float)[None].copy(),
                qlin=p[None], C=C[None], h=h[None])


def stack(problems):
    """Concatenate B=1 structured problems with identical shared data into one batch."""
    out = dict(problems[0])
    for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
        out[k] = np.concatenate([q[k] for q in problems], axis=0)
    return out
