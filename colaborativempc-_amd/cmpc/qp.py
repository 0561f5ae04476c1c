"""Dense standard-form QP batch with MATLAB ``quadprog`` semantics on the GPU
(``cmpc_solve_qp_batch``, include/cmpc.h), and the ``osqp_solve_qp`` adapter.

* ``quadprog(H, f, A, b, Aeq, beq, lb, ub)`` — the call YALMIP makes
  (Matlab-tests/yalmip/yalmip/YALMIP-master/solvers/callquadprog.m:63-69); the MEX
  gateway (mex/cmpc_quadprog_mex.c) binds the same C entry point.
* ``osqp_solve_qp(P, q, G, h, A, b, initvals)`` — same signature, return value
  ``(res, feasible)`` and status rule as the reference's wrapper
  (planner/lib/plan_lib/distributedPlanner/LPV_Planner.py:192-249): ``res.x``,
  ``res.info.status_val`` / ``res.info.status`` with OSQP's codes, and
  ``feasible = status_val in {1, 2, -2}``.

Both accept one problem or a batch (leading batch axis on every array).
"""
from __future__ import annotations

import ctypes as ct
from types import SimpleNamespace

import numpy as np

from . import _lib as L

# quadprog exitflag -> OSQP status_val / status text (the reference prints the text on failure)
_OSQP_OF_FLAG = {L.CMPC_QP_CONVERGED: (1, "solved"), L.CMPC_QP_MAXITER: (-2, "maximum iterations reached"),
                 L.CMPC_QP_INFEASIBLE: (-3, "primal infeasible"), L.CMPC_QP_UNBOUNDED: (-4, "dual infeasible"),
                 L.CMPC_QP_NONCONVEX: (-7, "problem non convex")}


def _dense(a):
    if a is None:
        return None
    if hasattr(a, "toarray"):
        a = a.toarray()
    return np.asarray(a, dtype=np.float64)


def quadprog(H, f, A=None, b=None, Aeq=None, beq=None, lb=None, ub=None, ctx=None, tol=None, max_iter=None):
    """Solve min 1/2 x'Hx + f'x s.t. A x <= b, Aeq x = beq, lb <= x <= ub on the GPU.

    Single problem: H (n,n), f (n,) ...; batch: a leading axis on every given array.
    Returns dict(x, fval, exitflag, iterations, lambda=dict(ineqlin, eqlin, lower, upper), residual)."""
    H = _dense(H)
    single = H.ndim == 2
    if single:
        H = H[None]
    B, n = H.shape[0], H.shape[1]

    def prep(a, shape_tail, name):
        if a is None:
            return None
        a = _dense(a)
        if a.size == 0:
            return None
        a = a[None] if single else a
        a = np.ascontiguousarray(a.reshape((B,) + shape_tail))
        return a

    f = prep(f, (n,), "f")
    if f is None:
        raise ValueError("f is required")
    # emptiness by shape: np.size of a scipy sparse matrix is its nnz, and a sparse G with no
    # stored entries still carries its rows (and their right-hand sides)
    A_ = None if A is None or 0 in np.shape(A) else _dense(A)
    mi = 0 if A_ is None else A_.shape[-2]
    Aeq_ = None if Aeq is None or 0 in np.shape(Aeq) else _dense(Aeq)
    me = 0 if Aeq_ is None else Aeq_.shape[-2]
    A_ = prep(A_, (mi, n), "A")
    b_ = prep(b, (mi,), "b") if mi else None
    E_ = prep(Aeq_, (me, n), "Aeq")
    e_ = prep(beq, (me,), "beq") if me else None
    lb_ = prep(lb, (n,), "lb")
    ub_ = prep(ub, (n,), "ub")
    ctx = ctx or L.default_context()
    keep = [np.ascontiguousarray(H), f, A_, b_, E_, e_, lb_, ub_]
    data = L.cmpc_qp_data(*[L.dptr(a) for a in keep])
    x = np.zeros((B, n))
    fval = np.zeros(B)
    flag = np.zeros(B, np.int32)
    it = np.zeros(B, np.int32)
    li = np.zeros((B, mi))
    le = np.zeros((B, me))
    llo = np.zeros((B, n))
    lup = np.zeros((B, n))
    resid = np.zeros(B)
    out = L.cmpc_qp_out(L.dptr(x), L.dptr(fval), L.iptr(flag), L.iptr(it), L.dptr(li) if mi else None,
                        L.dptr(le) if me else None, L.dptr(llo), L.dptr(lup), L.dptr(resid))
    dims = L.cmpc_qp_dims(n, mi, me, B, 0)
    ctx.check(ctx.lib.cmpc_solve_qp_batch(ctx.h, ct.byref(dims), ct.byref(data), ct.byref(out),
                                          ct.byref(L.opts(tol, max_iter))))
    del keep
    res = dict(x=x, fval=fval, exitflag=flag, iterations=it, residual=resid,
               **{"lambda": dict(ineqlin=li, eqlin=le, lower=llo, upper=lup)})
    if single:
        res = {k: (v[0] if not isinstance(v, dict) else {kk: vv[0] for kk, vv in v.items()}) for k, v in res.items()}
    return res


def _osqp_result(x, status_val, text, iters, obj, kkt, pri_res, path):
    res = SimpleNamespace(x=x, y=None, info=SimpleNamespace(status_val=status_val, status=text, iter=iters,
                                                           obj_val=obj, kkt=kkt, pri_res=pri_res, solver=path))
    feasible = 1 if status_val in (1, 2, -2) else 0   # LPV_Planner.py:243-249
    if status_val != 1:
        print("OSQP exited with status '%s'" % text)
    return res, feasible


def _pri_res(z, G, h, A, b):
    """Reference-form primal residual max(|A z - b|, max(G z - h, 0)) (OSQP's pri_res, inf-norm)."""
    r = 0.0
    if A is not None and b is not None:
        r = max(r, float(np.abs(A @ z - np.asarray(b, float).ravel()).max(initial=0.0)))
    if G is not None and h is not None:
        r = max(r, float(np.maximum(G @ z - np.asarray(h, float).ravel(), 0.0).max(initial=0.0)))
    return r


def osqp_solve_qp_batch(qps, ctx=None, tol=None, max_iter=None, structured=True):
    """Many ``osqp_solve_qp`` calls in as few GPU launches as possible: ``qps`` is a list of
    (P, q, G, h, A, b) tuples.  Every QP that ``structure.recognize`` identifies as a
    reference-form agent QP (LPV_Planner.py:156-157) joins one structured batch per distinct
    shared part (cmpc_solve_mpc_batch: one wavefront per agent); the others go through the
    dense kernel (cmpc_solve_qp_batch; ``structured=False`` sends every QP there).  Returns a
    list of (res, feasible)."""
    from . import structure as St
    from .solver import solve_mpc

    recs = [St.recognize(*qp[:6]) if structured else None for qp in qps]
    out = [None] * len(qps)
    groups = {}
    for i, p in enumerate(recs):
        if p is not None:
            groups.setdefault(St.shared_key(p), []).append(i)
    for idx in groups.values():
        batch = St.stack([recs[i] for i in idx])
        # CMPC_FLAG_RESCUE, as PlannerLPV / PlannerLPVBatch: a condensed factorisation breakdown
        # continues on the stage-wise kernel instead of returning CMPC_UNSOLVED (OSQP's -10)
        z, kkt, it, st = solve_mpc(batch, ctx, tol=tol, max_iter=max_iter, rescue=True, polish=True)
        for a, i in enumerate(idx):
            P, q, G, h, A, b = qps[i][:6]
            x = z[a]
            obj = float(0.5 * x @ (P @ x) + np.asarray(q, float) @ x)
            out[i] = _osqp_result(x, int(st[a]), L.STATUS_TEXT.get(int(st[a]), "unsolved"), int(it[a]), obj,
                                  float(kkt[a]), _pri_res(x, G, h, A, b), "structured")
    for i, p in enumerate(recs):
        if p is not None:
            continue
        P, q, G, h, A, b = qps[i][:6]
        r = quadprog(P, q, G, h, A, b, ctx=ctx, tol=tol, max_iter=max_iter)
        sv, text = _OSQP_OF_FLAG.get(int(r["exitflag"]), (-10, "unsolved"))
        x = r["x"]
        Gs = None if G is None else (G if hasattr(G, "toarray") else np.asarray(G, float))
        As = None if A is None else (A if hasattr(A, "toarray") else np.asarray(A, float))
        out[i] = _osqp_result(x, sv, text, int(r["iterations"]), float(r["fval"]), float(r["residual"]),
                              _pri_res(x, Gs, h, As, b), "dense")
    return out


def osqp_solve_qp(P, q, G=None, h=None, A=None, b=None, initvals=None, ctx=None):
    """Drop-in for the reference's ``osqp_solve_qp`` (LPV_Planner.py:192-249): the same QP
    (min 1/2 x'Px + q'x s.t. G x <= h, A x = b) solved on the GPU, returning (res, feasible)
    with ``res.x``, ``res.info.status_val`` / ``.status`` (OSQP codes), ``.obj_val``, ``.iter``,
    plus ``.pri_res`` (reference-form primal residual), ``.kkt`` (the solver's scaled KKT
    residual) and ``.solver`` ("structured" when the QP is recognised as the PlannerLPV agent
    QP and solved by the structured kernels, "dense" otherwise).  ``initvals`` is accepted
    but unused: the reference passes it to ``osqp.warm_start`` (:237-238), while the
    interior-point method here starts from its own interior point (the caller in the
    reference, PlannerLPV.solve :156-157, never passes it)."""
    return osqp_solve_qp_batch([(P, q, G, h, A, b)], ctx=ctx)[0]
