"""ORACLE (test infrastructure only) — dense fp64 primal-dual interior-point
solver for an OSQP-form QP, used in place of OSQP (absent; ``requirements.txt:5``).

    minimize  1/2 z'Pz + q'z   subject to  l <= A z <= u

is exactly what ``osqp_solve_qp`` (``distributedPlanner/LPV_Planner.py:192-249``)
passes to ``OSQP.setup``.  Rows with l == u are equalities, rows with one
infinite side are one-sided inequalities, all-zero rows (the reference's 0 = 0
slack rows, LPV_Planner.py:445-447) are dropped.

Algorithm: Mehrotra predictor-corrector on the full (non-condensed) KKT system
[[P + C'ΘC, E'], [E, 0]] solved by dense LU with one step of iterative
refinement.  The result is returned with OSQP-convention multipliers
y (A'y enters stationarity, y > 0 at active upper bounds) and a KKT
certificate so a fixture carries its own proof of optimality.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.linalg as sla


@dataclass
class QPResult:
    x: np.ndarray
    y: np.ndarray
    status: str
    status_val: int
    iters: int
    kkt: dict


def kkt_certificate(P, q, A, l, u, x, y):
    """OSQP-style residuals: stationarity ||Px+q+A'y||, primal ||Ax - proj_[l,u](Ax)||,
    complementarity max(|y+|·|u-Ax|, |y-|·|Ax-l|) over finite bounds."""
    Ax = A @ x
    stat = P @ x + q + A.T @ y
    proj = np.clip(Ax, l, u)
    prim = Ax - proj
    ypos = np.maximum(y, 0.0)
    yneg = np.maximum(-y, 0.0)
    with np.errstate(invalid="ignore"):
        cu = np.where(np.isfinite(u), ypos * np.abs(u - Ax), 0.0)
        cl = np.where(np.isfinite(l), yneg * np.abs(Ax - l), 0.0)
    # dual feasibility: y > 0 only where u finite, y < 0 only where l finite
    dfeas = np.where(np.isfinite(u), 0.0, ypos) + np.where(np.isfinite(l), 0.0, yneg)
    scale_d = max(1.0, np.abs(P @ x).max(initial=0), np.abs(q).max(initial=0),
                  np.abs(A.T @ y).max(initial=0))
    return dict(stat=float(np.abs(stat).max(initial=0)),
                stat_rel=float(np.abs(stat).max(initial=0) / scale_d),
                prim=float(np.abs(prim).max(initial=0)),
                comp=float(max(cu.max(initial=0), cl.max(initial=0))),
                dual_sign=float(dfeas.max(initial=0)))


def kkt_of_primal(P, q, A, l, u, x, act_tol=1e-7):
    """Reference-form KKT certificate of a primal point alone (for solvers that return no
    multipliers): the multipliers y minimising the stationarity residual ||Px + q + A'y|| subject to
    OSQP's sign convention (y free on equality rows, y >= 0 on rows with only an upper bound,
    y <= 0 on rows with only a lower bound) and to complementarity (y = 0 on rows farther than
    act_tol from their bound), by bounded least squares; returns (kkt_certificate(...), y)."""
    from scipy.optimize import lsq_linear

    P, A = np.asarray(P, float), np.asarray(A, float)
    x, l, u = np.asarray(x, float), np.asarray(l, float), np.asarray(u, float)
    Ax = A @ x
    nz = np.abs(A).sum(1) > 0
    eq = nz & np.isfinite(l) & np.isfinite(u) & (l == u)
    up = nz & ~eq & np.isfinite(u) & (np.abs(u - Ax) <= act_tol * np.maximum(1.0, np.abs(u)))
    lo = nz & ~eq & np.isfinite(l) & (np.abs(Ax - l) <= act_tol * np.maximum(1.0, np.abs(l)))
    use = eq | up | lo
    idx = np.flatnonzero(use)
    lb = np.where(up[idx] & ~lo[idx], 0.0, -np.inf)
    ub = np.where(lo[idx] & ~up[idx], 0.0, np.inf)
    y = np.zeros(A.shape[0])
    if len(idx):
        r = lsq_linear(A[idx].T, -(P @ x + q), bounds=(lb, ub), method="bvls", tol=1e-14, lsmr_tol="auto")
        y[idx] = r.x
    return kkt_certificate(P, q, A, l, u, x, y), y


def solve_qp(P, q, A, l, u, tol=1e-12, max_iter=200, verbose=False):
    P = np.asarray(P, float)
    A = np.asarray(A, float)
    q = np.asarray(q, float)
    l = np.asarray(l, float)
    u = np.asarray(u, float)
    n = P.shape[0]
    nz_row = np.any(A != 0.0, axis=1)
    eq = nz_row & np.isfinite(l) & np.isfinite(u) & (l == u)
    # all-zero rows must be satisfiable (0 in [l,u]) — they are dropped
    zr = ~nz_row
    if np.any((l[zr] > 0) | (u[zr] < 0)):
        raise ValueError("infeasible zero row")
    up = nz_row & ~eq & np.isfinite(u)
    lo = nz_row & ~eq & np.isfinite(l)
    E = A[eq]
    e = u[eq]
    C = np.vstack([A[up], -A[lo]])
    d = np.hstack([u[up], -l[lo]])
    me, mi = E.shape[0], C.shape[0]

    x = np.zeros(n)
    yv = np.zeros(me)
    s = np.maximum(d - C @ x, 1.0)
    lam = np.ones(mi)
    scale_q = max(1.0, np.abs(q).max(initial=0))
    status, it = "max_iter", 0
    best = (np.inf, x.copy(), yv.copy(), lam.copy())

    def kkt_solve(theta, rhs1, rhs2):
        Kmat = np.zeros((n + me, n + me))
        Kmat[:n, :n] = P + C.T @ (theta[:, None] * C)
        Kmat[:n, n:] = E.T
        Kmat[n:, :n] = E
        lu = sla.lu_factor(Kmat)
        rhs = np.hstack([rhs1, rhs2])
        sol = sla.lu_solve(lu, rhs)
        sol = sol + sla.lu_solve(lu, rhs - Kmat @ sol)      # iterative refinement
        return sol[:n], sol[n:]

    for it in range(1, max_iter + 1):
        rd = P @ x + q + E.T @ yv + C.T @ lam
        re = E @ x - e
        ri = C @ x + s - d
        mu = (s @ lam) / mi if mi else 0.0
        nrd = np.abs(rd).max(initial=0) / max(scale_q, np.abs(P @ x).max(initial=0))
        nrp = max(np.abs(re).max(initial=0), np.abs(ri).max(initial=0))
        if verbose:
            print(f"it {it:3d} rd {nrd:.2e} rp {nrp:.2e} mu {mu:.2e}")
        merit = max(nrd, nrp / max(1.0, np.abs(d).max(initial=0)), mu)
        if merit < best[0]:
            best = (merit, x.copy(), yv.copy(), lam.copy())
        if nrd < tol and nrp < tol * max(1.0, np.abs(d).max(initial=0)) and mu < tol:
            status = "solved"
            break
        theta = lam / s
        # predictor
        rc = -s * lam
        rho = (rc + lam * ri) / s
        dx, dy = kkt_solve(theta, -rd - C.T @ rho, -re)
        dlam = rho + theta * (C @ dx)
        ds = -ri - C @ dx
        a_p = _max_step(s, ds)
        a_d = _max_step(lam, dlam)
        a = min(1.0, a_p, a_d)
        mu_aff = ((s + a * ds) @ (lam + a * dlam)) / mi
        sig = (mu_aff / mu) ** 3 if mu > 0 else 0.0
        # corrector
        rc = -s * lam + sig * mu - ds * dlam
        rho = (rc + lam * ri) / s
        dx, dy = kkt_solve(theta, -rd - C.T @ rho, -re)
        dlam = rho + theta * (C @ dx)
        ds = -ri - C @ dx
        a = min(1.0, 0.995 * min(_max_step(s, ds), _max_step(lam, dlam)))
        x += a * dx
        yv += a * dy
        s += a * ds
        lam += a * dlam

    if status != "solved":   # fall back to the best iterate seen
        _, x, yv, lam = best
        if best[0] < 1e-9:
            status = "solved"
    nup = int(up.sum())

    def osqp_y(yv_, lam_):
        # OSQP-convention multipliers on the original rows
        y_ = np.zeros(A.shape[0])
        y_[eq] = yv_
        y_[up] += lam_[:nup]
        y_[lo] -= lam_[nup:]
        return y_

    y = osqp_y(yv, lam)
    cert = kkt_certificate(P, q, A, l, u, x, y)
    # Polish (as OSQP's polish=True, which the reference sets, LPV_Planner.py:232): re-solve
    # with the rows the IPM found active as equalities.  Interior-point iterates approach a
    # weakly active (degenerate) bound only like sqrt(mu); the polished point sits on it.
    # Kept only when it is primal and dual feasible and its certificate is no worse.
    if mi:
        act = lam > s
        Ca, da = C[act], d[act]
        ka = int(act.sum())
        K = np.zeros((n + me + ka, n + me + ka))
        K[:n, :n] = P
        K[:n, n:n + me] = E.T
        K[:n, n + me:] = Ca.T
        K[n:n + me, :n] = E
        K[n + me:, :n] = Ca
        rhs = np.hstack([-q, e, da])
        try:   # LU (not lstsq: its rank cut-off drops the 1e7-scaled slack directions)
            lu = sla.lu_factor(K)
            sol = sla.lu_solve(lu, rhs)
            sol = sol + sla.lu_solve(lu, rhs - K @ sol)
            if not np.isfinite(sol).all():
                sol = None
        except (np.linalg.LinAlgError, ValueError):
            sol = None
        if sol is not None:
            xp = sol[:n]
            lam_p = np.zeros(mi)
            lam_p[act] = sol[n + me:]
            yp = osqp_y(sol[n:n + me], lam_p)
            feas = (C @ xp <= d + 1e-10 * max(1.0, np.abs(d).max(initial=0))).all() and (lam_p >= -1e-9).all()
            cp = kkt_certificate(P, q, A, l, u, xp, yp)
            if feas and cp["stat_rel"] <= max(cert["stat_rel"], 1e-12) and cp["prim"] <= max(cert["prim"], 1e-12) \
                    and cp["comp"] <= cert["comp"]:
                x, y, cert = xp, yp, cp
    sv = 1 if status == "solved" else -2
    return QPResult(x, y, status, sv, it, cert)


def _max_step(v, dv):
    neg = dv < 0
    if not np.any(neg):
        return np.inf
    return float(np.min(-v[neg] / dv[neg]))
