"""Host-side entry points over the libcmpc C ABI.

Problems are dicts of arrays with the keys of include/cmpc.h:

  nx nu N ns mc                     ints (shared)
  Q (nx,nx) R (nu,nu) dR (nu,nu) Qs (ns,) u_ub (nu,) u_lb (nu,) row_slack (mc,) row_sign (mc,)
  A (B,N,nx,nx) B (B,N,nx,nu) x0 (B,nx) u_prev (B,nu) qlin (B,N+1,nx) C (B,N,mc,nx) h (B,N,mc)

``solve_mpc`` takes numpy (host) arrays; ``solve_mpc_dev`` takes torch CUDA
tensors already resident in HBM and launches on the current torch stream.
"""
from __future__ import annotations

import ctypes as ct

import numpy as np

from . import _lib as L

SHARED = ("Q", "R", "dR", "Qs", "u_ub", "u_lb")
PER_AGENT = ("A", "B", "x0", "u_prev", "qlin", "C", "h")


def nz_of(p):
    return (p["nx"] + p["ns"]) * (p["N"] + 1) + 2 * p["nu"] * p["N"]


def _dims(p, batch):
    return L.cmpc_mpc_dims(int(p["nx"]), int(p["nu"]), int(p["N"]), int(p["ns"]), int(p["mc"]), int(batch))


def _weights(p):
    keep = [L.f64(p[k]) for k in SHARED] + [L.i32(p["row_slack"]), L.i32(p["row_sign"])]
    w = L.cmpc_mpc_weights(*[L.dptr(a) for a in keep[:6]], L.iptr(keep[6]), L.iptr(keep[7]))
    return w, keep


def check_shapes(p, batch):
    nx, nu, N, ns, mc = (int(p[k]) for k in ("nx", "nu", "N", "ns", "mc"))
    want = dict(A=(batch, N, nx, nx), B=(batch, N, nx, nu), x0=(batch, nx), u_prev=(batch, nu),
                qlin=(batch, N + 1, nx), C=(batch, N, mc, nx), h=(batch, N, mc))
    for k, shp in want.items():
        if tuple(p[k].shape) != shp:
            raise ValueError(f"{k}: shape {tuple(p[k].shape)} != {shp}")
    for k, shp in dict(Q=(nx, nx), R=(nu, nu), dR=(nu, nu), Qs=(ns,), u_ub=(nu,), u_lb=(nu,),
                       row_slack=(mc,), row_sign=(mc,)).items():
        if tuple(np.shape(p[k])) != shp:
            raise ValueError(f"{k}: shape {np.shape(p[k])} != {shp}")


FP32_TOL = 1e-6   # default tolerance of the fp32 path (BASELINE cfg5; lane kernel, mixed precision)


def _flags(fp32=False, riccati=False, generic=False, rescue=False, lane=False, polish=False):
    return (L.CMPC_FLAG_FP32 if fp32 else 0) | (L.CMPC_FLAG_RICCATI if riccati else 0) | \
        (L.CMPC_FLAG_GENERIC if generic else 0) | (L.CMPC_FLAG_RESCUE if rescue else 0) | \
        (L.CMPC_FLAG_LANE if lane else 0) | (L.CMPC_FLAG_POLISH if polish else 0)


def plan(shared, batch=1, fp32=False, riccati=False, generic=False, lane=False, rescue=False, polish=False, flags=0):
    """Which solver cmpc_solve_mpc_batch would run for this problem shape, and its occupancy
    (cmpc_plan_mpc, host only): dict(solver=name, lds_bytes, wg_per_cu, agents_per_wg, waves_per_agent,
    polish_lds_bytes, polish_max_active) — the last two describe the rescue policy's polish launch (0 without
    ``rescue`` and ``polish``).  ``flags``: further CMPC_FLAG_* bits."""
    w, keep = _weights(shared)
    d = _dims(shared, batch)
    o = L.opts(None, None, _flags(fp32, riccati, generic, rescue, lane, polish) | int(flags))
    info = L.cmpc_plan_info()
    rc = L.load().cmpc_plan_mpc(ct.byref(d), ct.byref(w), ct.byref(o), ct.byref(info))
    if rc != L.CMPC_OK:
        raise L.CmpcError(rc, "cmpc_plan_mpc")
    names = {L.CMPC_SOLVER_CONDENSED_V3: "condensed_v3", L.CMPC_SOLVER_CONDENSED: "condensed",
             L.CMPC_SOLVER_RICCATI: "riccati", L.CMPC_SOLVER_LANE: "lane"}
    del keep
    return dict(solver=names[info.solver], lds_bytes=info.lds_bytes, wg_per_cu=info.wg_per_cu,
                agents_per_wg=info.agents_per_wg, waves_per_agent=info.waves_per_agent,
                polish_lds_bytes=info.polish_lds_bytes, polish_max_active=info.polish_max_active)


def solve_mpc(p, ctx=None, tol=None, max_iter=None, fp32=False, riccati=False, generic=False, rescue=False,
              stamps=None, lane=False, polish=False):
    """Solve a batch of structured agent-QPs on the GPU (host arrays in/out).
    ``fp32``: the fp32 path (BASELINE cfg5): fp32 Riccati factorisation and Newton recursions with
    fp64 iterates — the Riccati kernel's fp32 mode where it is instantiated (nx, nu, mc = 6, 3, 6),
    with ``lane`` (or where only it is instantiated) the lane-per-agent kernel; other dimensions
    raise CmpcError (CMPC_ERR_UNSUPPORTED);
    ``lane``: the lane-per-agent stage-wise kernel (fp64, or fp32 with ``fp32``);
    ``riccati``: force the stage-wise Riccati solver (the default when N*nu > 64);
    ``generic``: force the runtime-dimension condensed kernel;
    ``rescue``: CMPC_FLAG_RESCUE (a condensed solve whose factorisation breaks down continues on
    the stage-wise Riccati kernel; PlannerLPV's default);
    ``polish``: CMPC_FLAG_POLISH with ``rescue`` (OSQP's polish=True for a breakdown at the rounding
    floor: the active set taken as exact, the equality-constrained QP solved; PlannerLPV's default);
    ``stamps``: optional device address of a batch x 16 uint64 buffer (per-section clock counts).

    Returns (z (B,nz), kkt (B,), iters (B,), status (B,))."""
    ctx = ctx or L.default_context()
    batch = int(p["A"].shape[0])
    check_shapes(p, batch)
    w, keep = _weights(p)
    arrs = [L.f64(p[k]) for k in PER_AGENT]
    data = L.cmpc_mpc_data(*[L.dptr(a) for a in arrs])
    z = np.zeros((batch, nz_of(p)))
    kkt = np.zeros(batch)
    iters = np.zeros(batch, np.int32)
    status = np.zeros(batch, np.int32)
    out = L.cmpc_mpc_out(L.dptr(z), L.dptr(kkt), L.iptr(iters), L.iptr(status))
    o = L.opts(tol or (FP32_TOL if fp32 else None), max_iter, _flags(fp32, riccati, generic, rescue, lane, polish),
               stamps)
    ctx.check(ctx.lib.cmpc_solve_mpc_batch(ctx.h, ct.byref(_dims(p, batch)), ct.byref(w), ct.byref(data),
                                           ct.byref(out), ct.byref(o)))
    del keep, arrs
    return z, kkt, iters, status


def _tptr(t):
    import torch

    if t is None:
        return None
    if not (t.is_cuda and t.is_contiguous()):
        raise ValueError("device entry points need contiguous CUDA tensors")
    if t.dtype == torch.float64:
        return ct.cast(ct.c_void_p(t.data_ptr()), L._DP)
    if t.dtype == torch.int32:
        return ct.cast(ct.c_void_p(t.data_ptr()), L._IP)
    raise TypeError(f"unsupported dtype {t.dtype}")


def solve_mpc_dev(shared, dev, out, ctx=None, tol=None, max_iter=None, stream=None, fp32=False, riccati=False,
                  lane=False):
    """Device-resident batch solve.  ``shared``: dict with dims + shared weights (host);
    ``dev``: dict of CUDA float64 tensors (PER_AGENT keys); ``out``: dict with
    'z' (float64) and optional 'kkt' (float64), 'iters', 'status' (int32) tensors.
    Launches asynchronously on ``stream`` (default: torch's current stream)."""
    import torch

    ctx = ctx or L.default_context(dev["A"].device.index or 0)
    batch = int(dev["A"].shape[0])
    w, keep = _weights(shared)
    data = L.cmpc_mpc_data(*[_tptr(dev[k]) for k in PER_AGENT])
    o_ = L.cmpc_mpc_out(_tptr(out["z"]), _tptr(out.get("kkt")), _tptr(out.get("iters")), _tptr(out.get("status")))
    s = stream if stream is not None else torch.cuda.current_stream(dev["A"].device)
    o = L.opts(tol or (FP32_TOL if fp32 else None), max_iter, _flags(fp32, riccati, lane=lane))
    ctx.check(ctx.lib.cmpc_solve_mpc_batch_dev(ctx.h, ct.byref(_dims(shared, batch)), ct.byref(w),
                                               ct.byref(data), ct.byref(o_), ct.byref(o),
                                               ct.c_void_p(s.cuda_stream)))
    del keep


def selftest_mfma(ctx=None, seed=0):
    """D = A*B on one f64 16x16x4 MFMA tile; returns (D_gpu, D_ref)."""
    ctx = ctx or L.default_context()
    rng = np.random.default_rng(seed)
    A = rng.integers(-8, 8, (16, 4)).astype(np.float64)
    B = rng.integers(-8, 8, (4, 16)).astype(np.float64)
    D = np.zeros((16, 16))
    ctx.check(ctx.lib.cmpc_selftest_mfma(ctx.h, L.dptr(A), L.dptr(B), L.dptr(D)))
    return D, A @ B
