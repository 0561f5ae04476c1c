"""Recognition of the PlannerLPV QP structure at the ``osqp_solve_qp`` boundary.

The reference hands OSQP one sparse QP per agent and control step
(planner/lib/plan_lib/distributedPlanner/LPV_Planner.py:156-157 -> :192-249):

    z = [xi_0 .. xi_N | u_0 .. u_{N-1} | du_0 .. du_{N-1}],   xi_k = [x_k (nx) | s_k (ns)]
    P = 2 blkdiag((Q (+) Qs)^(N+1), R^N, dR^N)                                   (:382-427)
    q = 2 [p_0 .. p_N (state part only), 0, 0]
    G z <= h: stage rows C_{k,r} x_k + sign_r s_k[slack_r] <= h_{k,r}, k = 1..N   (:251-380)
              then per stage [u_i <= ub_i; -u_i <= -lb_i] for every input i
    A z = b:  x_0 = x0;  x_k - A_{k-1} x_{k-1} - B_{k-1} u_{k-1} = 0;  0 = 0 on the slack rows;
              u_0 - du_0 = u_prev;  u_{k-1} - u_k + du_k = 0                        (:429-475)

``recognize`` reads every structured quantity (A_k, B_k, x0, u_prev, Q, R, dR, Qs, p_k,
C_k, h_k, input bounds, the slack pattern) out of such a QP, rebuilds the QP from them
(``reference_form``) and accepts only when the rebuilt matrices and vectors are equal to
the given ones entry for entry.  An accepted QP is therefore *identical* to the structured
problem the one-wavefront-per-agent solvers take (cmpc_solve_mpc_batch), and the adapter
solves it there instead of through the generic dense kernel.  Anything else returns None.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

LPV_LAYOUT = (9, 3, 2)   # PlannerLPV: n_s = 9 states, 3 slacks, n_u = 2 inputs (LPV_Planner.py:31-33)


def _csr(a):
    """Canonical csr (sorted indices, no duplicates, no stored zeros) of ``a``; a float64 csr
    input that is canonical already is returned as it is (the reference's scipy matrices)."""
    if sp.issparse(a) and a.format == "csr" and a.dtype == np.float64 and a.has_canonical_format \
            and a.data.all():
        return a
    m = sp.csr_matrix(a, dtype=np.float64)
    m.sum_duplicates()
    m.eliminate_zeros()
    return m


def _canon(rows, cols, vals, shape):
    """Canonical csr arrays (indptr, indices, data) of coordinate triples without duplicates:
    stored zeros dropped, entries ordered by row then column, as _csr gives them."""
    keep = vals != 0.0
    rows, cols, vals = rows[keep], cols[keep], vals[keep]
    o = np.lexsort((cols, rows))
    rows, cols = rows[o], cols[o]
    if rows.size > 1 and ((np.diff(rows) == 0) & (np.diff(cols) == 0)).any():
        raise ValueError("duplicate entries")   # never for the reference form: one entry per slot
    indptr = np.zeros(shape[0] + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=shape[0]), out=indptr[1:])
    return indptr, cols, vals[o], shape


def _matrix(c):
    indptr, indices, data, shape = c
    return sp.csr_matrix((data, indices, indptr), shape=shape)


def _same_canon(X, c):
    """X (canonical csr) equal entry for entry to the canonical arrays c."""
    indptr, indices, data, shape = c
    return X.shape == shape and np.array_equal(X.indptr, indptr) and np.array_equal(X.indices, indices) \
        and np.array_equal(X.data, data)


def _rows_of(X):
    return np.repeat(np.arange(X.shape[0]), np.diff(X.indptr))


def _dense_block(X, r0, r1, c0, c1):
    """X[r0:r1, c0:c1] as a dense array, read from the canonical csr arrays."""
    out = np.zeros((r1 - r0, c1 - c0))
    s, e = X.indptr[r0], X.indptr[r1]
    r = np.repeat(np.arange(r1 - r0), np.diff(X.indptr[r0:r1 + 1]))
    c = X.indices[s:e]
    m = (c >= c0) & (c < c1)
    out[r[m], c[m] - c0] = X.data[s:e][m]
    return out


def dims_of(nz, m_ineq, m_eq, layout=LPV_LAYOUT):
    """(N, mc) of a reference-form QP with layout (nx, ns, nu), or None."""
    nx, ns, nu = layout
    ne = nx + ns
    if (nz - ne) % (ne + 2 * nu):
        return None
    N = (nz - ne) // (ne + 2 * nu)
    if N < 1 or m_eq != ne * (N + 1) + nu * N or (m_ineq - 2 * nu * N) % N:
        return None
    mc = (m_ineq - 2 * nu * N) // N
    return (N, mc) if mc >= 0 else None


_COST_CACHE = {}


def _cost_matrix(N, ne, nu, qt, r, dr):
    """P = 2 blkdiag(Qt^(N+1), R^N, dR^N) (LPV_Planner.py:382-427) as canonical csr, memoised on
    the exact bytes of its blocks (the gains are fixed per planner, the block_diag rebuild was
    the largest part of a recognition)."""
    key = (N, ne, nu, qt, r, dr)
    P = _COST_CACHE.get(key)
    if P is None:
        blocks = [np.frombuffer(qt).reshape(ne, ne)] * (N + 1) + [np.frombuffer(r).reshape(nu, nu)] * N + \
                 [np.frombuffer(dr).reshape(nu, nu)] * N
        m = _csr(sp.block_diag(blocks, format="csr") * 2.0)
        P = (m.indptr.astype(np.int64), m.indices.astype(np.int64), m.data.copy(), m.shape)
        for a_ in P[:3]:
            a_.setflags(write=False)
        if len(_COST_CACHE) > 64:
            _COST_CACHE.clear()
        _COST_CACHE[key] = P
    return P


def reference_form(p, a=0):
    """Sparse reference-form QP (P, q, G, h, Aeq, beq) of agent ``a`` of a structured problem
    dict (the keys of include/cmpc.h; row_slack / row_sign give the slack pattern)."""
    P, q, G, h, Aeq, beq = _reference_canon(p, a)
    return _matrix(P), q, _matrix(G), h, _matrix(Aeq), beq


_PATTERN_CACHE = {}


def _sorted_pattern(rows, cols, shape):
    """The canonical (row, then column) order of a list of entry slots: (order, rows, cols), read-only.
    The slots of the reference form depend on the dimensions and the slack pattern only, so the sort
    is done once per shape and a rebuild only drops the slots whose value is zero (_canon's result)."""
    o = np.lexsort((cols, rows))
    r, c = rows[o], cols[o]
    if r.size > 1 and ((np.diff(r) == 0) & (np.diff(c) == 0)).any():
        raise ValueError("duplicate entries")   # never for the reference form: one entry per slot
    for a_ in (o, r, c):
        a_.setflags(write=False)
    return o, r, c, shape


def _slot_keys(pat):
    """(sorted row * ncols + col keys, slot of each) of a _sorted_pattern: the lookup that maps a
    canonical csr entry to its slot (recognize)."""
    o, r, c, shape = pat
    keys = r.astype(np.int64) * shape[1] + c
    keys.setflags(write=False)
    return keys, o


def _pattern(N, nx, ns, nu, mc, sl):
    """Entry slots of G and Aeq of the reference form (LPV_Planner.py:251-380, :429-475) for these
    dimensions and slack pattern ``sl`` (row_slack), in the order _reference_canon lists their values,
    with their canonical order; plus the constant values of the input / input-rate slots."""
    key = (N, nx, ns, nu, mc, sl.tobytes())
    pat = _PATTERN_CACHE.get(key)
    if pat is not None:
        return pat
    ne = nx + ns
    nz = ne * (N + 1) + 2 * nu * N
    cu, cd = ne * (N + 1), ne * (N + 1) + nu * N
    # inequalities: stage rows C_{k,r} x_k (+ sign s_k[slack]), then per stage [u_i <= ub; -u_i <= -lb]
    k = np.arange(1, N + 1)
    r_st = (k - 1)[:, None, None] * mc + np.arange(mc)[None, :, None]          # (N, mc, 1)
    c_st = k[:, None, None] * ne + np.arange(nx)[None, None, :]               # (N, 1, nx)
    rows = [np.broadcast_to(r_st, (N, mc, nx)).ravel()]
    cols = [np.broadcast_to(c_st, (N, mc, nx)).ravel()]
    has = np.nonzero(sl >= 0)[0]
    if has.size:
        rows.append(((k - 1)[:, None] * mc + has[None, :]).ravel())
        cols.append((k[:, None] * ne + nx + sl[has][None, :]).ravel())
    ms = N * mc
    ku = np.arange(N)[:, None]
    iu = np.arange(nu)[None, :]
    ru = ms + (ku * nu + iu) * 2
    cu_i = cu + ku * nu + iu
    rows += [ru.ravel(), (ru + 1).ravel()]
    cols += [cu_i.ravel(), cu_i.ravel()]
    G = _sorted_pattern(np.concatenate(rows), np.concatenate(cols), (ms + 2 * nu * N, nz))
    g_const = np.concatenate([np.ones(N * nu), -np.ones(N * nu)])
    # equalities: x_k - A_{k-1} x_{k-1} - B_{k-1} u_{k-1} = 0 (x_0 = x0), then the input-rate rows
    ke = np.arange(N + 1)
    rows = [(ke[:, None] * ne + np.arange(nx)).ravel()]
    cols = [(ke[:, None] * ne + np.arange(nx)).ravel()]
    kd = np.arange(1, N + 1)[:, None, None]
    s_ = np.arange(nx)[None, :, None]
    rows.append(np.broadcast_to(kd * ne + s_, (N, nx, nx)).ravel())
    cols.append(np.broadcast_to((kd - 1) * ne + np.arange(nx)[None, None, :], (N, nx, nx)).ravel())
    rows.append(np.broadcast_to(kd * ne + s_, (N, nx, nu)).ravel())
    cols.append(np.broadcast_to(cu + (kd - 1) * nu + np.arange(nu)[None, None, :], (N, nx, nu)).ravel())
    r0 = ne * (N + 1)
    i = np.arange(N)[:, None]
    j = np.arange(nu)[None, :]
    rr = (r0 + i * nu + j).ravel()
    first = (i == 0).repeat(nu, 1).ravel()
    rows += [rr, rr, rr[~first]]
    cols += [(cu + i * nu + j).ravel(), (cd + i * nu + j).ravel(), (cu + (i - 1) * nu + j).ravel()[~first]]
    A = _sorted_pattern(np.concatenate(rows), np.concatenate(cols), (ne * (N + 1) + nu * N, nz))
    a_const = np.concatenate([np.where(first, 1.0, -1.0), np.where(first, -1.0, 1.0), np.ones((~first).sum())])
    for a_ in (g_const, a_const):
        a_.setflags(write=False)
    pat = dict(G=G, g_const=g_const, A=A, a_const=a_const, ones_x=np.ones((N + 1) * nx), G_keys=_slot_keys(G),
               A_keys=_slot_keys(A), nC=N * mc * nx, nS=N * has.size, has=has, nA=N * nx * nx, nB=N * nx * nu)
    if len(_PATTERN_CACHE) > 64:
        _PATTERN_CACHE.clear()
    _PATTERN_CACHE[key] = pat
    return pat


def _fill(pat, vals):
    """Canonical csr arrays of the slots ``pat`` holding ``vals`` (listed in slot order): the slots in
    canonical order, those with a zero value dropped — equal to _canon of the same triples."""
    o, r, c, shape = pat
    v = vals[o]
    keep = v != 0.0
    indptr = np.zeros(shape[0] + 1, np.int64)
    np.cumsum(np.bincount(r[keep], minlength=shape[0]), out=indptr[1:])
    return indptr, c[keep], v[keep], shape


def _reference_canon(p, a=0):
    """reference_form with the three matrices as canonical csr arrays (see _canon)."""
    nx, nu, N, ns, mc = (int(p[k]) for k in ("nx", "nu", "N", "ns", "mc"))
    ne = nx + ns
    nz = ne * (N + 1) + 2 * nu * N
    # cost
    Qt = np.zeros((ne, ne))
    Qt[:nx, :nx] = p["Q"]
    Qt[nx:, nx:] = np.diag(np.asarray(p["Qs"], float))
    R_, dR_ = np.ascontiguousarray(p["R"], float), np.ascontiguousarray(p["dR"], float)
    P = _cost_matrix(N, Qt.shape[0], R_.shape[0], Qt.tobytes(), R_.tobytes(), dR_.tobytes())
    q = np.zeros(nz)
    q[: ne * (N + 1)].reshape(N + 1, ne)[:, :nx] = 2.0 * np.asarray(p["qlin"][a], float)
    sl = np.asarray(p["row_slack"])
    pat = _pattern(N, nx, ns, nu, mc, sl)
    # inequalities: stage rows, then input rows
    has = np.nonzero(sl >= 0)[0]
    sg = np.asarray(p["row_sign"], float)
    G = _fill(pat["G"], np.concatenate([np.asarray(p["C"][a], float).ravel(), np.tile(sg[has], N),
                                        pat["g_const"]]))
    h = np.concatenate([np.asarray(p["h"][a], float).ravel(),
                        np.stack([np.broadcast_to(np.asarray(p["u_ub"], float), (N, nu)),
                                  np.broadcast_to(-np.asarray(p["u_lb"], float), (N, nu))], -1).ravel()])
    # equalities
    Aeq = _fill(pat["A"], np.concatenate([pat["ones_x"], -np.asarray(p["A"][a], float).ravel(),
                                          -np.asarray(p["B"][a], float).ravel(), pat["a_const"]]))
    r0 = ne * (N + 1)
    beq = np.zeros(Aeq[3][0])
    beq[:nx] = p["x0"][a]
    beq[r0:r0 + nu] = p["u_prev"][a]
    return P, q, G, h, Aeq, beq


def _slots_of(X, keys_slots, nslots):
    """Values of the canonical csr X in the slot order of a pattern (absent slots 0), or None when X
    holds an entry outside the pattern."""
    keys, slot = keys_slots
    k = _rows_of(X).astype(np.int64) * X.shape[1] + X.indices
    i = np.searchsorted(keys, k)
    if k.size and (i[-1] >= keys.size or not np.array_equal(keys[np.minimum(i, keys.size - 1)], k)):
        return None
    vals = np.zeros(nslots)
    vals[slot[i]] = X.data
    return vals


def recognize(P, q, G, h, A, b, layout=LPV_LAYOUT):
    """Structured single-agent problem dict (batch axis of 1) if (P, q, G, h, A, b) is exactly
    a reference-form agent QP of the given layout, else None.

    Every entry of G and Aeq is mapped to its slot of the reference form's pattern (cached per
    shape and slack pattern, _pattern); the structured quantities are read from the slots and the
    QP is accepted only when no entry lies outside the pattern and the fixed slots (identities, the
    +-1 input rows, the slack signs of every stage), P, q, h and b are the reference form's — the
    same QPs _recognize_rebuild accepts by rebuilding them (tests/test_structure.py compares the two)."""
    if G is None or A is None or h is None or b is None:
        return None
    nx, ns, nu = layout
    ne = nx + ns
    P, G, A = _csr(P), _csr(G), _csr(A)
    q, h, b = (np.asarray(v, dtype=np.float64).ravel() for v in (q, h, b))
    nz = P.shape[1]
    if P.shape != (nz, nz) or G.shape[1] != nz or A.shape[1] != nz or q.size != nz or \
            h.size != G.shape[0] or b.size != A.shape[0]:
        return None
    d = dims_of(nz, G.shape[0], A.shape[0], layout)
    if d is None:
        return None
    N, mc = d
    cu, cd = ne * (N + 1), ne * (N + 1) + nu * N
    if not (np.isfinite(q).all() and np.isfinite(b).all()) or np.isnan(h).any():
        return None
    # cost (P / 2 and q / 2 are exact in binary floating point)
    Pd = _dense_block(P, 0, ne, 0, ne) / 2.0
    Q, Qs = Pd[:nx, :nx], np.diag(Pd[nx:, nx:]).copy()
    R = _dense_block(P, cu, cu + nu, cu, cu + nu) / 2.0
    dR = _dense_block(P, cd, cd + nu, cd, cd + nu) / 2.0
    if ns and not (Qs > 0).all():
        return None
    Qt = np.zeros((ne, ne))
    Qt[:nx, :nx] = Q
    Qt[nx:, nx:] = np.diag(Qs)
    if not _same_canon(P, _cost_matrix(N, ne, nu, Qt.tobytes(), np.ascontiguousarray(R).tobytes(),
                                       np.ascontiguousarray(dR).tobytes())):
        return None
    qlin = q[: ne * (N + 1)].reshape(N + 1, ne)[:, :nx] / 2.0
    q2 = np.zeros(nz)
    q2[: ne * (N + 1)].reshape(N + 1, ne)[:, :nx] = 2.0 * qlin
    if not np.array_equal(q, q2):
        return None
    # slack pattern from the stage-1 rows (the slots check every stage)
    row_slack = -np.ones(mc, np.int32)
    row_sign = np.ones(mc, np.int32)
    e1 = G.indptr[mc]
    r1, c1, v1 = _rows_of(G)[:e1], G.indices[:e1], G.data[:e1]
    ss = (c1 >= ne + nx) & (c1 < 2 * ne)
    for rr_, cc_, vv_ in zip(r1[ss], c1[ss], v1[ss]):
        if row_slack[rr_] >= 0 or vv_ not in (1.0, -1.0):
            return None
        row_slack[rr_] = cc_ - ne - nx
        row_sign[rr_] = int(vv_)
    pat = _pattern(N, nx, ns, nu, mc, row_slack)
    nC, nS, has = pat["nC"], pat["nS"], pat["has"]
    gv = _slots_of(G, pat["G_keys"], nC + nS + pat["g_const"].size)
    if gv is None or not np.array_equal(gv[nC:nC + nS], np.tile(row_sign[has].astype(np.float64), N)) \
            or not np.array_equal(gv[nC + nS:], pat["g_const"]):
        return None
    n1, nA, nB = pat["ones_x"].size, pat["nA"], pat["nB"]
    av = _slots_of(A, pat["A_keys"], n1 + nA + nB + pat["a_const"].size)
    if av is None or not np.array_equal(av[:n1], pat["ones_x"]) or \
            not np.array_equal(av[n1 + nA + nB:], pat["a_const"]):
        return None
    Cm = gv[:nC].reshape(N, mc, nx)
    Am = (0.0 - av[n1:n1 + nA]).reshape(N, nx, nx)          # 0.0 - v: an absent slot gives +0.0
    Bm = (0.0 - av[n1 + nA:n1 + nA + nB]).reshape(N, nx, nu)
    ms = N * mc
    hu = h[ms:].reshape(N, nu, 2)
    if not np.array_equal(hu, np.broadcast_to(hu[0], hu.shape)):
        return None
    x0 = b[:nx].copy()
    u_prev = b[cu: cu + nu].copy()
    b2 = np.zeros(b.size)
    b2[:nx] = x0
    b2[cu:cu + nu] = u_prev
    if not np.array_equal(b, b2):
        return None
    hh = h[:ms].reshape(N, mc).copy()
    u_ub, u_lb = hu[0, :, 0].copy(), -hu[0, :, 1]
    return dict(nx=nx, nu=nu, N=N, ns=ns, mc=mc, Q=Q, R=R, dR=dR, Qs=Qs, u_ub=u_ub, u_lb=u_lb,
                row_slack=row_slack, row_sign=row_sign, A=Am[None], B=Bm[None], x0=x0[None], u_prev=u_prev[None],
                qlin=qlin[None], C=Cm[None], h=hh[None])


def _recognize_rebuild(P, q, G, h, A, b, layout=LPV_LAYOUT):
    """recognize by extraction and an exact rebuild (the round-5 form, kept as the tests' reference
    for the slot-based recognize)."""
    if G is None or A is None or h is None or b is None:
        return None
    nx, ns, nu = layout
    ne = nx + ns
    P, G, A = _csr(P), _csr(G), _csr(A)
    q, h, b = (np.asarray(v, dtype=np.float64).ravel() for v in (q, h, b))
    nz = P.shape[1]
    if P.shape != (nz, nz) or G.shape[1] != nz or A.shape[1] != nz or q.size != nz or \
            h.size != G.shape[0] or b.size != A.shape[0]:
        return None
    d = dims_of(nz, G.shape[0], A.shape[0], layout)
    if d is None:
        return None
    N, mc = d
    cu, cd = ne * (N + 1), ne * (N + 1) + nu * N
    if not (np.isfinite(q).all() and np.isfinite(b).all()) or np.isnan(h).any():
        return None
    # cost (P / 2 and q / 2 are exact in binary floating point)
    Pd = _dense_block(P, 0, ne, 0, ne) / 2.0
    Q, Qs = Pd[:nx, :nx], np.diag(Pd[nx:, nx:]).copy()
    R = _dense_block(P, cu, cu + nu, cu, cu + nu) / 2.0
    dR = _dense_block(P, cd, cd + nu, cd, cd + nu) / 2.0
    if ns and not (Qs > 0).all():
        return None
    qlin = q[: ne * (N + 1)].reshape(N + 1, ne)[:, :nx] / 2.0
    # dynamics from the equality rows
    r, c, v = _rows_of(A), A.indices, A.data
    kr, sr = r // ne, r % ne
    dyn = (r < ne * (N + 1)) & (kr >= 1) & (sr < nx)
    Am = np.zeros((N, nx, nx))
    Bm = np.zeros((N, nx, nu))
    mx = dyn & (c < ne * (N + 1)) & (c // ne == kr - 1) & (c % ne < nx)
    Am[kr[mx] - 1, sr[mx], c[mx] % ne] = -v[mx]
    mu_ = dyn & (c >= cu) & (c < cd) & ((c - cu) // nu == kr - 1)
    Bm[kr[mu_] - 1, sr[mu_], (c[mu_] - cu) % nu] = -v[mu_]
    x0 = b[:nx].copy()
    u_prev = b[ne * (N + 1): ne * (N + 1) + nu].copy()
    # stage rows and input bounds from the inequality rows
    r, c, v = _rows_of(G), G.indices, G.data
    ms = N * mc
    st = (r < ms) & (c // ne == r // mc + 1) & (c < ne * (N + 1))
    Cm = np.zeros((N, mc, nx))
    sx = st & (c % ne < nx)
    Cm[r[sx] // mc, r[sx] % mc, c[sx] % ne] = v[sx]
    row_slack = -np.ones(mc, np.int32)
    row_sign = np.ones(mc, np.int32)
    ss = st & (c % ne >= nx) & (r < mc)   # slack pattern from stage 1; the rebuild checks all stages
    for rr_, cc_, vv_ in zip(r[ss], c[ss], v[ss]):
        if row_slack[rr_] >= 0 or vv_ not in (1.0, -1.0):
            return None
        row_slack[rr_] = cc_ % ne - nx
        row_sign[rr_] = int(vv_)
    hh = h[:ms].reshape(N, mc).copy()
    hu = h[ms:].reshape(N, nu, 2)
    u_ub, u_lb = hu[0, :, 0].copy(), -hu[0, :, 1]
    prob = dict(nx=nx, nu=nu, N=N, ns=ns, mc=mc, Q=Q, R=R, dR=dR, Qs=Qs, u_ub=u_ub, u_lb=u_lb,
                row_slack=row_slack, row_sign=row_sign, A=Am[None], B=Bm[None], x0=x0[None], u_prev=u_prev[None],
                qlin=qlin[None], C=Cm[None], h=hh[None])
    P2, q2, G2, h2, A2, b2 = _reference_canon(prob, 0)
    if not (_same_canon(P, P2) and _same_canon(G, G2) and _same_canon(A, A2) and np.array_equal(q, q2)
            and np.array_equal(b, b2) and np.array_equal(h, h2)):
        return None
    return prob


def shared_key(p):
    """Hashable key of the batch-shared part of a structured problem (problems with equal keys
    can share one cmpc_solve_mpc_batch launch)."""
    return (p["nx"], p["nu"], p["N"], p["ns"], p["mc"]) + tuple(
        np.asarray(p[k], float).tobytes() for k in ("Q", "R", "dR", "Qs", "u_ub", "u_lb")) + (
        np.asarray(p["row_slack"]).tobytes(), np.asarray(p["row_sign"]).tobytes())


def stack(probs):
    """One structured batch from single-agent problems with equal shared_key."""
    out = {k: probs[0][k] for k in ("nx", "nu", "N", "ns", "mc", "Q", "R", "dR", "Qs", "u_ub", "u_lb",
                                     "row_slack", "row_sign")}
    for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
        out[k] = np.concatenate([p[k] for p in probs])
    return out
