"""Diagnostic: iterate-by-iterate comparison of the two kernels on one captured QP
(runs both with max_iter = 1, 2, ... and compares the returned iterate)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa
import cmpc  # noqa
from cmpc import _lib as L  # noqa
from conftest import lpv_qps  # noqa
from oracle import lpv_ref as LR  # noqa

name, which = sys.argv[1], int(sys.argv[2])
ctx = cmpc.Context(0)
g = LR.paper_gains()
tr = LR.Track.build("Highway")
c = [c for j, c in lpv_qps(name)][which]
lim = LR.scaled_car_limits(c["vx_ref"])
qp = LR.assemble(c["x0"], c["x_last"], c["u_last"], c["x_agents"], c["pose"], c["u_old"], c["N"], c["dt"], tr,
                 LR.SCALED_CAR_MODEL, lim, g)
P = LR.structured(qp, c["x0"], c["u_old"], c["N"], lim, g)
from cmpc.solver import solve_mpc  # noqa
import ctypes as ct  # noqa
for it in range(1, 30):
    res = {}
    for flag in (0, 1):
        # solve_mpc has no flags argument: call the ABI directly
        from cmpc.solver import _weights, _dims, PER_AGENT, nz_of
        w, keep = _weights(P)
        arrs = [L.f64(P[k]) for k in PER_AGENT]
        data = L.cmpc_mpc_data(*[L.dptr(a) for a in arrs])
        z = np.zeros((1, nz_of(P))); kkt = np.zeros(1); iters = np.zeros(1, np.int32); st = np.zeros(1, np.int32)
        out = L.cmpc_mpc_out(L.dptr(z), L.dptr(kkt), L.iptr(iters), L.iptr(st))
        o = L.opts(max_iter=it, flags=flag)
        ctx.check(ctx.lib.cmpc_solve_mpc_batch(ctx.h, ct.byref(_dims(P, 1)), ct.byref(w), ct.byref(data),
                                               ct.byref(out), ct.byref(o)))
        res[flag] = (z[0], kkt[0], st[0])
    d = np.abs(res[0][0] - res[1][0]).max()
    print(f"max_iter {it:2d}: |z_v2 - z_gen| {d:.2e}  kkt v2 {res[0][1]:.2e} gen {res[1][1]:.2e}  st {res[0][2]} {res[1][2]}")
