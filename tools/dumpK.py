"""Diagnostic: first-iteration Newton matrix K from both kernels on one captured LPV QP."""
import ctypes as ct
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
from cmpc.solver import _weights, _dims, PER_AGENT, nz_of  # noqa
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
n = P["N"] * P["nu"]
npad = (n + 15) // 16 * 16
Ks = {}
for flag in (2, 3):
    dump = torch.zeros(npad * npad * (2 * c['N'] + 8), dtype=torch.float64, device="cuda")
    w, keep = _weights(P)
    arrs = [L.f64(P[k]) for k in PER_AGENT]
    data = L.cmpc_mpc_data(*[L.dptr(a) for a in arrs])
    z = np.zeros((1, nz_of(P))); kkt = np.zeros(1); iters = np.zeros(1, np.int32); st = np.zeros(1, np.int32)
    out = L.cmpc_mpc_out(L.dptr(z), L.dptr(kkt), L.iptr(iters), L.iptr(st))
    o = L.opts(max_iter=1, flags=flag, stamps=dump.data_ptr())
    ctx.check(ctx.lib.cmpc_solve_mpc_batch(ctx.h, ct.byref(_dims(P, 1)), ct.byref(w), ct.byref(data), ct.byref(out),
                                           ct.byref(o)))
    torch.cuda.synchronize()
    Ks[flag] = np.tril(dump[:npad * npad].cpu().numpy().reshape(npad, npad))[:n, :n]
d = np.abs(Ks[2] - Ks[3])
print("max |K_v2 - K_gen|", d.max(), "rel", d.max() / np.abs(Ks[3]).max())
i, j = np.unravel_index(np.argmax(d), d.shape)
print("worst entry", i, j, Ks[2][i, j], Ks[3][i, j])
bad = np.argwhere(d > 1e-9 * np.abs(Ks[3]).max())
print("bad entries", len(bad), bad[:20].tolist())
for (i, j) in bad:
    a, b = Ks[2][i, j], Ks[3][i, j]
    ia, ib = np.float64(a).view(np.uint64), np.float64(b).view(np.uint64)
    print(i, j, repr(a), repr(b), "diff", a - b, "xor", hex(int(ia) ^ int(ib)))
