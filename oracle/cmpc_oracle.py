"""ORACLE (test infrastructure only) — ctypes binding of oracle/libcmpc_oracle.so,
the plain-C condensed IPM restatement (cmpc_oracle.c).
newton: 0 condensed Cholesky, 1 stage-wise Riccati (as csrc/mpc_riccati.hip), 2 Riccati in Joseph form,
3 Riccati with the kernel's double-double mode, 4 / 5 condensed with the hand-over to 3 at a breakdown
(CMPC_FLAG_RESCUE with / without CMPC_FLAG_FINISH).

Problems are plain dicts of numpy arrays (batch-major):
  nx nu N ns mc                 ints
  Q (nx,nx) R (nu,nu) dR (nu,nu) Qs (ns,)  u_ub (nu,) u_lb (nu,)
  row_slack (mc,) int (-1: none)   row_sign (mc,) int (+1/-1)
  A (B,N,nx,nx) B (B,N,nx,nu) x0 (B,nx) u_prev (B,nu)
  qlin (B,N+1,nx)   C (B,N,mc,nx)  h (B,N,mc)
"""
import ctypes as ct
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libcmpc_oracle.so")
        if not os.path.exists(path):
            build()
        _LIB = ct.CDLL(path)
        _LIB.cmpc_oracle_solve.restype = ct.c_int
        _LIB.cmpc_oracle_solve_ex.restype = ct.c_int
    return _LIB


def _d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(ct.POINTER(ct.c_double))


def _i(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(ct.POINTER(ct.c_int))


def nz_of(p):
    return (p["nx"] + p["ns"]) * (p["N"] + 1) + 2 * p["nu"] * p["N"]


def solve_batch_rescue(p, tol=1e-9, max_iter=60, nthreads=0, finish=False, polish=False, polish_amax=None):
    """The product's CMPC_FLAG_RESCUE policy restated: the condensed method; an agent whose
    factorisation breaks down short of the rounding floor (best merit >= 1e3 tol; with ``finish``,
    CMPC_FLAG_FINISH, every breakdown) continues from that iterate with the Riccati method in the
    kernel's double-double mode, its best-iterate bookkeeping restarted (newton 5 / 4, the kernels'
    hand-over); an agent that still ends CMPC_UNSOLVED is re-solved by that Riccati method from a
    cold start (newton 3, the second rescue pass).  ``polish_amax``: the polish kernel's active-set
    capacity for this shape (cmpc.solver.plan(..., rescue=True, polish=True)["polish_max_active"]), so
    both sides polish the same agents.  Required with ``polish``: the kernel lowers its capacity to fit
    LDS (88 for the reference agent at N = 30), and a default would polish different agents than the
    GPU without notice."""
    if polish and not polish_amax:
        raise ValueError("solve_batch_rescue(polish=True) needs polish_amax: the GPU layout's capacity "
                         "(cmpc.solver.plan(P, 1, rescue=True, polish=True)['polish_max_active'])")
    pol = (0x100 | (int(polish_amax) & 0xff) << 16) if polish else 0
    z, kkt, it, st = solve_batch(p, tol, max_iter, nthreads, newton=(4 if finish else 5) | pol)
    bad = np.flatnonzero(st == -10)
    if len(bad):
        q = dict(p)
        for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
            q[k] = p[k][bad]
        z[bad], kkt[bad], it[bad], st[bad] = solve_batch(q, tol, max_iter, nthreads, newton=3 | pol)
    return z, kkt, it, st


def solve_batch(p, tol=1e-9, max_iter=60, nthreads=0, newton=0, refine=0, U0=None):
    nb = p["A"].shape[0]
    keep = []
    args = []
    for k in ("Q", "R", "dR", "Qs", "u_ub", "u_lb"):
        a, ptr = _d(p[k]); keep.append(a); args.append(ptr)
    for k in ("row_slack", "row_sign"):
        a, ptr = _i(p[k]); keep.append(a); args.append(ptr)
    for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
        a, ptr = _d(p[k]); keep.append(a); args.append(ptr)
    if U0 is not None:
        U0 = np.ascontiguousarray(U0, dtype=np.float64)
        keep.append(U0)
    z = np.zeros((nb, nz_of(p)))
    kkt = np.zeros(nb)
    iters = np.zeros(nb, np.int32)
    status = np.zeros(nb, np.int32)
    rc = lib().cmpc_oracle_solve_ex(
        ct.c_int(p["nx"]), ct.c_int(p["nu"]), ct.c_int(p["N"]), ct.c_int(p["ns"]), ct.c_int(p["mc"]),
        ct.c_int(nb), *args, ct.c_double(tol), ct.c_int(max_iter), ct.c_int(nthreads), ct.c_int(newton), ct.c_int(refine),
        None if U0 is None else _d(U0)[1],
        z.ctypes.data_as(ct.POINTER(ct.c_double)), kkt.ctypes.data_as(ct.POINTER(ct.c_double)),
        iters.ctypes.data_as(ct.POINTER(ct.c_int)), status.ctypes.data_as(ct.POINTER(ct.c_int)))
    if rc != 0:
        raise RuntimeError("cmpc_oracle_solve failed")
    return z, kkt, iters, status
