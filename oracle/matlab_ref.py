"""ORACLE — test infrastructure only (never imported by the product package).

Restatement of the reference's MATLAB per-agent QP path:

* the 5-state LPV-MPC problem of Matlab-tests/mrs_LPV_MPC/LPV_MPC_fnc_dt_Vnew.m:1-155 (the
  YALMIP `optimizer` that PLAN_NL_LPV_MPC_dt_WORKS_Oval.m:237-253 calls every control step),
  with its parameters substituted — what YALMIP compiles into `interfacedata`
  (F_struc, K.f, c, Q, lb, ub);
* YALMIP's model transformation for quadprog, Matlab-tests/yalmip/yalmip/YALMIP-master/solvers/
  yalmip2quadprog.m:1-78 (equality-in-bounds rows :27-36, Aeq = -F(1:K.f,2:end),
  beq = F(1:K.f,1), A = -F(K.f+1:end,2:end), b = F(K.f+1:end,1) :38-46, Q <- 2Q :61);
  callquadprog.m:63-69 then calls quadprog(Q, c, A, b, Aeq, beq, lb, ub, x0, ops).

* the planner script's scheduling of those parameters, PLAN_NL_LPV_MPC_dt_WORKS_Oval.m:127-200
  (k = 1 from the NL_vars.mat it loads at :19, later steps from the previous solution), the
  oval track's curvature lookup (MapMod.m "oval", Curvature.m) and the arc-length update
  :259-260, with the script's left/right swap when it builds the inputs list (:237-238 pass
  {..., right_limit, left_limit} to parameters_in's {..., left_limit, right_limit}).

MATLAB, YALMIP and quadprog are absent: PARITY UNPINNED by quadprog outputs.
What pins it: the transformation is restated line by line and checked on hand-built known
answers (tests/test_matlab_ref.py); the first control step's parameters come from the
reference's own data file NL_vars.mat (read by scipy.io.loadmat, data only) through the
restated :127-167; every model's optimum is certified by the KKT residual of the dense IPM
oracle/qp_ipm.py (tests/golden/matlab_lpv_mpc.npz, made by oracle/gen_matlab_fixtures.py).
Steps k >= 2 are scheduled from the certified optimum of step k-1; the reference's optimum has
flat directions (tests/test_mex_gpu.py::_flat_directions), so quadprog could pick another point
of the same face and schedule slightly different parameters from it.

Variable order (YALMIP orders by sdpvar creation; the ones that survive parameter
substitution here are the decision variables, in this restatement's order):
    z = [x(:,2) .. x(:,Hp+1) (5 each) | u(:,1) .. u(:,Hp) (2 each) | sc(1) .. sc(Hp+1)]
Simple bounds: inequality rows with a single nonzero become lb / ub of that variable (the
tightest wins) and leave F_struc — YALMIP's bound extraction for solvers that take bounds.
"""
from __future__ import annotations

import numpy as np

# tuning of LPV_MPC_fnc_dt_Vnew.m:43-53
QQ = -np.diag([0.000000000213635, -0.000000000000088, -9.703658572659423, -0.153591566469547])
LL = -np.array([0.0, 1.00702414775175, 0.187661946033823, -0.0329493219494661])
MAX_A_LAT, MAX_A_LONG, MIN_A_LONG = 1.5, 0.7, -1.7   # :38-40
NX, NU = 5, 2


def yalmip2quadprog(F_struc, Kf, c, Q, lb, ub):
    """yalmip2quadprog.m:1-78 (the parts that shape the QP).  F_struc rows are
    [constant | coefficients]: the first Kf rows mean F1 + F2 z == 0, the rest F1 + F2 z >= 0.
    Returns dict(H, f, A, b, Aeq, beq, lb, ub) — quadprog's min 1/2 z'Hz + f'z."""
    F = np.array(F_struc, float, copy=True)
    lb = np.array(lb, float, copy=True)
    ub = np.array(ub, float, copy=True)
    n = len(c)
    # :27-36  "QUAPROG does not like lb==ub": such bounds become equality rows, bounds widened by 1
    eib = np.flatnonzero((np.abs(lb - ub) < 1e-12) & ~np.isinf(lb))
    m = len(eib)
    if m:
        rows = np.zeros((m, n + 1))
        rows[:, 0] = -lb[eib]
        rows[np.arange(m), 1 + eib] = 1.0
        F = np.vstack([rows, F]) if F.size else rows
        ub[eib] += 1.0
        lb[eib] -= 1.0
        Kf += m
    if F.size:   # :38-46
        Aeq, beq = -F[:Kf, 1:], F[:Kf, 0]
        A, b = -F[Kf:, 1:], F[Kf:, 0]
    else:
        A = b = Aeq = beq = np.zeros((0,))
    return dict(H=2.0 * np.asarray(Q, float), f=np.asarray(c, float), A=A, b=b, Aeq=Aeq, beq=beq, lb=lb, ub=ub)


class _Affine:
    """Affine expressions over the decision vector: rows of [constant | coefficients]."""

    def __init__(self, n):
        self.n = n

    def var(self, i):
        r = np.zeros(self.n + 1)
        r[1 + i] = 1.0
        return r

    def const(self, v):
        r = np.zeros(self.n + 1)
        r[0] = v
        return r


def lpv_mpc_interface(Hp, dt, p, max_vel=3.5):
    """YALMIP interfacedata of LPV_MPC_fnc_dt_Vnew(Hp, dt, max_vel) after substituting the
    optimizer parameters p (dict: x1 (5,), curv (Hp+1,), A1..A10 (Hp,), B1..B4 (Hp,),
    left (Hp+1,), right (Hp+1,)) — the inputs list of :118-119.  Returns
    (F_struc, Kf, c, Q, lb, ub) with objective z'Qz + c'z (+ constant dropped)."""
    nxv, nuv, nsc = NX * Hp, NU * Hp, Hp + 1
    n = nxv + nuv + nsc
    E = _Affine(n)

    def X(i, k):   # x(i,k) of :4, i 1-based state, k 1-based stage; x(:,1) is a parameter
        return E.const(p["x1"][i - 1]) if k == 1 else E.var((k - 2) * NX + (i - 1))

    def U(i, k):
        return E.var(nxv + (k - 1) * NU + (i - 1))

    def SC(k):
        return E.var(nxv + nuv + (k - 1))

    g = lambda name, k: p[name][k - 1]   # noqa: E731  parameter row vectors, 1-based
    Q = np.zeros((n, n))
    c = np.zeros(n)

    def add_sq(w, e):   # w * e^2 for an affine e (constant part dropped from Q, kept in c)
        co, a = e[0], e[1:]
        Q[:, :] += w * np.outer(a, a)
        c[:] += 2.0 * w * co * a

    def add_lin(w, e):
        c[:] += w * e[1:]

    eqs, ineqs = [], []
    for k in range(1, Hp + 1):
        # objective :79-81: [x4;x1;x2;x5]' QQ [..] + LL [..] + 200 sc(k)^2 + 0.05 x3^2
        v = [X(4, k), X(1, k), X(2, k), X(5, k)]
        for a in range(4):
            add_sq(QQ[a, a], v[a])   # QQ is diagonal
            add_lin(LL[a], v[a])
        add_sq(200.0, SC(k))
        add_sq(0.05, X(3, k))
        # dynamics :89-98 (Euler), written as lhs - rhs == 0
        eqs.append(X(1, k + 1) - (X(1, k) + (-1.0 * X(1, k) + g("A5", k) * X(2, k) + g("A6", k) * X(3, k) +
                                               g("B1", k) * U(1, k) + g("B2", k) * U(2, k)) * dt))
        eqs.append(X(2, k + 1) - (X(2, k) + (g("A7", k) * X(2, k) + g("A8", k) * X(3, k) + g("B3", k) * U(1, k)) * dt))
        eqs.append(X(3, k + 1) - (X(3, k) + (g("A9", k) * X(2, k) + g("A10", k) * X(3, k) + g("B4", k) * U(1, k)) * dt))
        eqs.append(X(4, k + 1) - (X(4, k) + (g("A4", k) * X(5, k) + E.const(g("A3", k))) * dt))
        eqs.append(X(5, k + 1) - (X(5, k) + (-g("A1", k) * g("curv", k) * X(1, k) +
                                             g("A1", k) * g("A2", k) * g("curv", k) * X(2, k) + X(3, k)) * dt))
        # :100 left_limit - sc(k) <= x(4,k) <= right_limit + sc(k): left/right are the whole
        # 1 x (Hp+1) parameter rows, so YALMIP emits one row per entry (as written)
        for j in range(1, Hp + 2):
            ineqs.append(X(4, k) + SC(k) - E.const(g("left", j)))       # >= 0
            ineqs.append(E.const(g("right", j)) + SC(k) - X(4, k))      # >= 0
        ineqs.append(X(1, k) - E.const(0.9))                            # :101
        ineqs.append(E.const(max_vel) - X(1, k))
        dvx = (X(1, k + 1) - X(1, k)) * (1.0 / dt)                      # :102
        ineqs.append(dvx - E.const(MIN_A_LONG))
        ineqs.append(E.const(MAX_A_LONG) - dvx)
        dvy = (X(2, k + 1) - X(2, k)) * (1.0 / dt)                      # :103
        ineqs.append(dvy + E.const(MAX_A_LAT))
        ineqs.append(E.const(MAX_A_LAT) - dvy)
        ineqs.append(U(1, k) + E.const(0.3))                            # :104
        ineqs.append(E.const(0.3) - U(1, k))
        ineqs.append(U(2, k) + E.const(10.0))                           # :105
        ineqs.append(E.const(5.0) - U(2, k))
    # terminal :121-128
    add_sq(200.0, SC(Hp + 1))
    add_sq(3.0, X(3, Hp + 1))
    for j in range(1, Hp + 2):
        ineqs.append(X(4, Hp + 1) + SC(Hp + 1) - E.const(g("left", j)))
        ineqs.append(E.const(g("right", j)) + SC(Hp + 1) - X(4, Hp + 1))
    ineqs.append(X(1, Hp + 1) - E.const(0.9))
    ineqs.append(E.const(max_vel) - X(1, Hp + 1))

    lb = np.full(n, -np.inf)
    ub = np.full(n, np.inf)
    rows = []
    for r in ineqs:
        nzc = np.flatnonzero(r[1:])
        if len(nzc) == 0:       # parameter-only constraint (x(:,1) rows): feasible or not, no row
            if r[0] < 0:
                raise ValueError("infeasible parameter-only constraint")
            continue
        if len(nzc) == 1:       # simple bound  a z_i + c0 >= 0
            i, a = nzc[0], r[1 + nzc[0]]
            v = -r[0] / a
            if a > 0:
                lb[i] = max(lb[i], v)
            else:
                ub[i] = min(ub[i], v)
            continue
        rows.append(r)
    F = np.vstack(eqs + rows)
    return F, len(eqs), c, Q, lb, ub


# ---- the planner script's scheduling (PLAN_NL_LPV_MPC_dt_WORKS_Oval.m) ----
# vehicle constants of :46-53 (this script's, not the Python planners' scaled car)
PLAN_LF, PLAN_LR, PLAN_M, PLAN_I, PLAN_CF, PLAN_CR = 0.125, 0.125, 1.98, 0.03, 70.0, 70.0
PLAN_HP, PLAN_TSS = 15, 0.1                      # :44, Tss of NL_vars.mat
PLAN_X0 = np.array([0.97, 0.0, 0.0, 0.0, 0.0])   # :162 [vx, vy, w, ey, etheta]


def oval_segments(side=1):
    """MapMod.m "oval" (spec of lane `side`, scale 2 on lane 1): the Curvature.m-relevant columns
    of PointAndTangent — cumulative s at the segment start (column 4), segment length (5) and
    signed curvature (6) — for the spec rows (Curvature.m loops over all rows but the closing
    one).  Straights have curvature 0, arcs 1/r (MapMod.m: NewLine(6) = 1 / r)."""
    if side == 1:
        spec = 2.0 * np.array([[1.0, 0.0], [4.5, 4.5 / np.pi], [2.0, 0.0], [4.5, 4.5 / np.pi], [1.0, 0.0]])
    else:
        spec = np.array([[2.0, 0.0], [5.85, 5.85 / np.pi], [4.0, 0.0], [5.85, 5.85 / np.pi], [2.0, 0.0]])
    length = spec[:, 0]
    s0 = np.concatenate([[0.0], np.cumsum(length)[:-1]])
    curv = np.where(spec[:, 1] == 0.0, 0.0, 1.0 / np.where(spec[:, 1] == 0.0, 1.0, spec[:, 1]))
    return s0, length, curv


def curvature(s, seg):
    """Curvature.m: wrap s by the track length (end-1 row's s + length), then the LAST segment
    with s0 <= s <= s0 + len wins (both ends inclusive)."""
    s0, length, curv = seg
    track = s0[-1] + length[-1]
    while s > track:
        s = s - track
    idx = None
    for i in range(len(s0)):
        if s >= s0[i] and s <= s0[i] + length[i]:
            idx = i
    if idx is None:
        raise ValueError("s before the start of the track")   # MATLAB: undefined indx
    return curv[idx]


def _lpv_entries(vx, vy, psi_e, ey, delta, curv):
    """:141-160 / :181-197 — A_1..A_10, B_1..B_4 from a scheduling trajectory."""
    lf, lr, m, I, Cf, Cr = PLAN_LF, PLAN_LR, PLAN_M, PLAN_I, PLAN_CF, PLAN_CR
    sd, cd = np.sin(delta), np.cos(delta)
    return dict(A1=1.0 / (1.0 - ey * curv), A2=np.sin(psi_e), A3=np.array(vy, float), A4=np.array(vx, float),
                A5=(sd * Cf) / (m * vx), A6=(sd * Cf * lf) / (m * vx) + vy,
                A7=-(Cr + Cf * cd) / (m * vx), A8=-(lf * Cf * cd - lr * Cr) / (m * vx) - vx,
                A9=-(lf * Cf * cd - lr * Cr) / (I * vx), A10=-(lf * lf * Cf * cd + lr * lr * Cr) / (I * vx),
                B1=-(sd * Cf) / m, B2=np.ones_like(vx), B3=(Cf * cd) / m, B4=(lf * Cf * cd) / I)


def _limits(Hp, counter=0):
    """:227-232 and the swap of :237-238: returns the (left, right) PARAMETERS of the controller."""
    left_limit = (0.5 + counter * 0.1) * np.ones(Hp + 1)
    right_limit = (-0.5 - counter * 0.1) * np.ones(Hp + 1)
    return right_limit, left_limit


def plan_first_step(nl, Hp=PLAN_HP, side=1):
    """Optimizer inputs of control step k = 1 (:127-167) from NL_vars.mat's arrays `nl`
    (ss_NL, ey_NL, etheta_NL, Vy_NL, Vx_NL, delta; each 1 x 26)."""
    g = lambda k: np.asarray(nl[k], float).ravel()   # noqa: E731
    seg = oval_segments(side)
    ss = g("ss_NL")
    curv = np.zeros(Hp + 1)
    for j in range(Hp):                                   # :131-133
        curv[j] = curvature(ss[j], seg)
    s_variation = ss[Hp - 1] - ss[Hp - 2]                 # :136-137
    curv[Hp] = curvature(ss[Hp - 1] + s_variation, seg)
    p = _lpv_entries(g("Vx_NL")[:Hp], g("Vy_NL")[:Hp], g("etheta_NL")[:Hp], g("ey_NL")[:Hp], g("delta")[:Hp],
                     curv[:Hp])
    left, right = _limits(Hp)
    p.update(x1=PLAN_X0.copy(), curv=curv, left=left, right=right)
    return p


def plan_next_step(z, s_hist, k, curv_prev, Hp=PLAN_HP, side=1):
    """After the step-(k-1) solve with decision vector z (this module's variable order): the
    arc-length update :259-260 extends s_hist (0-based list, s_hist[i] = MATLAB s(i+1)), then the
    step-k inputs of :171-199 (x0 = XX_dt(:,1), scheduling on XX_dt / UU_dt).  Returns p."""
    XX = z[: NX * Hp].reshape(Hp, NX).T                   # XX_dt = x(:, 2:end), 5 x Hp
    UU = z[NX * Hp: (NX + NU) * Hp].reshape(Hp, NU).T     # UU_dt = u, 2 x Hp
    kk = k - 1                                            # the step just solved
    for j in range(1, Hp + 1):                            # :259-260, s(kk+j)
        vx, vy, ey, pe = XX[0, j - 1], XX[1, j - 1], XX[3, j - 1], XX[4, j - 1]
        val = s_hist[kk + j - 2] + ((vx * np.cos(pe) - vy * np.sin(pe)) / (1.0 - ey * curv_prev[j - 1])) * PLAN_TSS
        if len(s_hist) < kk + j:
            s_hist.append(val)
        else:
            s_hist[kk + j - 1] = val
    seg = oval_segments(side)
    curv = np.zeros(Hp + 1)
    for j in range(1, Hp + 1):                            # :171-173, s(k+j-1)
        curv[j - 1] = curvature(s_hist[k + j - 2], seg)
    s_variation = s_hist[k + Hp - 2] - s_hist[k + Hp - 3]
    curv[Hp] = curvature(s_hist[k + Hp - 2] + s_variation, seg)
    p = _lpv_entries(XX[0], XX[1], XX[4], XX[3], UU[0], curv[:Hp])
    left, right = _limits(Hp)
    p.update(x1=XX[:, 0].copy(), curv=curv, left=left, right=right)
    return p


def sample_parameters(Hp, seed, vx=1.5, curv_amp=0.4):
    """A plausible parameter set: LPV entries from a scaled-car linearisation around (vx, 0, 0)
    (signs and magnitudes as the MATLAB planner's scheduling produces), curvature of an oval
    track segment, lane limits +-0.4 (hand-built known-answer cases)."""
    rng = np.random.default_rng(seed)
    lf = lr = 0.125
    m, I, Cf, Cr = 1.98, 0.06, 60.0, 60.0
    v = vx + rng.uniform(-0.2, 0.2, Hp)
    p = dict(x1=np.array([vx, rng.uniform(-0.05, 0.05), rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1),
                          rng.uniform(-0.05, 0.05)]),
             curv=curv_amp * np.sin(np.linspace(0, 1.5, Hp + 1) + rng.uniform(0, 3)),
             A1=1.0 / (1.0 - 0.05 * rng.uniform(-1.0, 1.0, Hp)), A2=rng.uniform(-0.05, 0.05, Hp), A3=rng.uniform(-0.1, 0.1, Hp),
             A4=v.copy(), A5=rng.uniform(0.0, 0.2, Hp), A6=rng.uniform(0.0, 0.1, Hp),
             A7=-(Cf + Cr) / (m * v), A8=-(lf * Cf - lr * Cr) / (m * v) - v,
             A9=-(lf * Cf - lr * Cr) / (I * v), A10=-(lf * lf * Cf + lr * lr * Cr) / (I * v),
             B1=-rng.uniform(0.0, 0.5, Hp), B2=np.ones(Hp), B3=np.full(Hp, Cf / m), B4=np.full(Hp, lf * Cf / I),
             left=np.full(Hp + 1, -0.4), right=np.full(Hp + 1, 0.4))
    return p


def osqp_form(model):
    """quadprog model -> the OSQP form of oracle/qp_ipm.py (l <= [A; Aeq; I] z <= u)."""
    n = len(model["f"])
    blocks, lo, up = [], [], []
    if np.size(model["A"]):
        blocks.append(model["A"]); lo.append(np.full(len(model["b"]), -np.inf)); up.append(model["b"])
    if np.size(model["Aeq"]):
        blocks.append(model["Aeq"]); lo.append(model["beq"]); up.append(model["beq"])
    fin = np.isfinite(model["lb"]) | np.isfinite(model["ub"])
    blocks.append(np.eye(n)[fin]); lo.append(model["lb"][fin]); up.append(model["ub"][fin])
    return model["H"], model["f"], np.vstack(blocks), np.concatenate(lo), np.concatenate(up)
