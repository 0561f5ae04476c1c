"""ORACLE (test infrastructure only) — the synthetic double-integrator family of
BASELINE.json, restated in numpy with the reference's QP structure.

The reference has no double integrator (its model is the LPV bicycle); BASELINE
fixes this synthetic family.  Its QP is built here in two
independent forms:

* ``structured(...)``  — per-stage rows / costs, the layout the condensed
  solvers consume (checks the GPU builder cmpc_di_build_dev element by element);
* ``reference_form(...)`` — the full OSQP-form (P, q, A, l, u) with the exact
  z layout and row order of PlannerLPV (distributedPlanner/LPV_Planner.py:
  279-475), solved by oracle/qp_ipm.py to pin the condensed solvers.

Quirks kept from the reference: plane row k-1 and weight row k serve stage k
(LPV_Planner.py:269-272,421; utilities/misc.py:10-18); p_k on the speed state
for every k including 0 (:412-413).
"""
from __future__ import annotations

import numpy as np


def structured(shared, prm, A, B, x0, u_prev, lane, nbr, traj, self_idx):
    """Build the structured batch for agents `self_idx` (global indices) from the
    gathered trajectories `traj` (n_total, N+1, 2)."""
    N, nx, nb = shared["N"], shared["nx"], nbr.shape[1]
    dim = prm["dim"]
    ivx, ipy = dim, 1
    mc = 4 + nb
    nag = len(self_idx)
    C = np.zeros((nag, N, mc, nx))
    h = np.zeros((nag, N, mc))
    p = np.zeros((nag, N + 1, nx))
    for a, g in enumerate(self_idx):
        own = traj[g]
        p[a, :, ivx] = -prm["v_ref"] * prm["q_v"]
        p[a, :, ipy] = -lane[a] * prm["q_lane"]
        for k in range(1, N + 1):
            r = k - 1
            C[a, r, 0, ivx] = -1.0; h[a, r, 0] = -prm["min_vel"]
            C[a, r, 1, ivx] = 1.0;  h[a, r, 1] = prm["max_vel"]
            C[a, r, 2, ipy] = 1.0;  h[a, r, 2] = prm["hw"] + lane[a]
            C[a, r, 3, ipy] = -1.0; h[a, r, 3] = prm["hw"] - lane[a]
            px = py = 0.0
            for i in range(nb):
                nt = traj[nbr[a, i]]
                pe, pn = own[k - 1], nt[k - 1]
                v = pn - pe
                v = v / np.sqrt(v[0] ** 2 + v[1] ** 2)
                b = -0.5 * v @ (pe + pn)
                dist = np.sqrt((own[k, 0] - nt[k, 0]) ** 2 + (own[k, 1] - nt[k, 1]) ** 2)
                w = (2 * prm["min_dist"] - dist) / nb
                C[a, r, 4 + i, 0] = v[0]
                C[a, r, 4 + i, 1] = v[1]
                h[a, r, 4 + i] = -prm["min_dist"] / 2 - b
                px = px + prm["wq"] * w * v[0]
                py = py + prm["wq"] * w * v[1]
            p[a, k, 0] += px
            p[a, k, 1] += py
    out = dict(shared)
    out.update(A=np.asarray(A, float), B=np.asarray(B, float), x0=np.asarray(x0, float),
               u_prev=np.asarray(u_prev, float), qlin=p, C=C, h=h)
    return out


def reference_form(prob, a):
    """OSQP-form QP of agent `a` of a structured batch, laid out exactly like
    PlannerLPV's (z = [xi_0..xi_N | u | du], xi_k = [x_k | s_k])."""
    nx, nu, N, ns, mc = (prob[k] for k in ("nx", "nu", "N", "ns", "mc"))
    ne = nx + ns
    nz = ne * (N + 1) + 2 * nu * N
    cu, cd = ne * (N + 1), ne * (N + 1) + nu * N
    M = np.zeros((nz, nz))
    Qt = np.zeros((ne, ne))
    Qt[:nx, :nx] = prob["Q"]
    Qt[nx:, nx:] = np.diag(prob["Qs"])
    for k in range(N + 1):
        M[k * ne:(k + 1) * ne, k * ne:(k + 1) * ne] = Qt
    for k in range(N):
        M[cu + k * nu:cu + (k + 1) * nu, cu + k * nu:cu + (k + 1) * nu] = prob["R"]
        M[cd + k * nu:cd + (k + 1) * nu, cd + k * nu:cd + (k + 1) * nu] = prob["dR"]
    pv = np.zeros(nz)
    for k in range(N + 1):
        pv[k * ne:k * ne + nx] = prob["qlin"][a, k]
    # inequalities (stage rows then input rows)
    rows, ub = [], []
    for k in range(1, N + 1):
        for r in range(mc):
            row = np.zeros(nz)
            row[k * ne:k * ne + nx] = prob["C"][a, k - 1, r]
            j = prob["row_slack"][r]
            if j >= 0:
                row[k * ne + nx + j] = prob["row_sign"][r]
            rows.append(row)
            ub.append(prob["h"][a, k - 1, r])
    for k in range(N):
        for i in range(nu):
            for sgn, bnd in ((1.0, prob["u_ub"][i]), (-1.0, -prob["u_lb"][i])):
                row = np.zeros(nz)
                row[cu + k * nu + i] = sgn
                rows.append(row)
                ub.append(bnd)
    F = np.array(rows)
    b = np.array(ub)
    # equalities
    G = np.zeros((ne * (N + 1) + nu * N, nz))
    beq = np.zeros(G.shape[0])
    for k in range(N + 1):
        G[k * ne:k * ne + nx, k * ne:k * ne + nx] = np.eye(nx)
    beq[:nx] = prob["x0"][a]
    for k in range(1, N + 1):
        G[k * ne:k * ne + nx, (k - 1) * ne:(k - 1) * ne + nx] = -prob["A"][a, k - 1]
        G[k * ne:k * ne + nx, cu + (k - 1) * nu:cu + k * nu] = -prob["B"][a, k - 1]
    r0 = ne * (N + 1)
    for i in range(N):
        G[r0 + i * nu:r0 + (i + 1) * nu, cu + i * nu:cu + (i + 1) * nu] = np.eye(nu) if i == 0 else -np.eye(nu)
        if i > 0:
            G[r0 + i * nu:r0 + (i + 1) * nu, cu + (i - 1) * nu:cu + i * nu] = np.eye(nu)
        G[r0 + i * nu:r0 + (i + 1) * nu, cd + i * nu:cd + (i + 1) * nu] = -np.eye(nu) if i == 0 else np.eye(nu)
    beq[r0:r0 + nu] = prob["u_prev"][a]
    Aqp = np.vstack([F, G])
    fin = np.isfinite(b)
    l = np.hstack([-np.inf * np.ones(len(b)), beq])
    u = np.hstack([np.where(fin, b, np.inf), beq])
    return 2 * M, 2 * pv, Aqp, l, u
