"""Diagnostic: specialised vs generic kernel, one IPM iteration, across sizes."""
import ctypes as ct
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa
import cmpc  # noqa
from cmpc import _lib as L  # noqa
from cmpc import scenarios as S  # noqa
from cmpc.solver import _weights, _dims, PER_AGENT, nz_of  # noqa
from oracle import synth  # noqa

ctx = cmpc.Context(0)


def run(P, it, flag):
    B = P["A"].shape[0]
    w, keep = _weights(P)
    arrs = [L.f64(P[k]) for k in PER_AGENT]
    data = L.cmpc_mpc_data(*[L.dptr(a) for a in arrs])
    z = np.zeros((B, nz_of(P))); kkt = np.zeros(B); iters = np.zeros(B, np.int32); st = np.zeros(B, np.int32)
    out = L.cmpc_mpc_out(L.dptr(z), L.dptr(kkt), L.iptr(iters), L.iptr(st))
    o = L.opts(max_iter=it, flags=flag)
    ctx.check(ctx.lib.cmpc_solve_mpc_batch(ctx.h, ct.byref(_dims(P, B)), ct.byref(w), ct.byref(data), ct.byref(out),
                                           ct.byref(o)))
    return z, st, iters


for dim, nb in ((2, 2), (2, 1), (3, 2)):
    for N in (6, 8, 9, 10, 12, 16, 20, 24, 30):
        if N * dim > 64:
            continue
        sc = S.make_di(16, N, nb, dim)
        P = synth.structured(sc.shared, sc.params, sc.A, sc.B, sc.x0, sc.u_prev, sc.lane, sc.nbr, sc.traj, np.arange(16))
        z2, s2, i2 = run(P, 1, 0)
        zg, sg, ig = run(P, 1, 1)
        zf2, sf2, _ = run(P, 60, 0)
        zfg, sfg, _ = run(P, 60, 1)
        print(f"dim {dim} nb {nb} N {N:2d}: iter1 diff {np.abs(z2 - zg).max():.1e}   final diff {np.abs(zf2 - zfg).max():.1e} "
              f"solved v2 {(sf2 == 1).sum()}/16 gen {(sfg == 1).sum()}/16")
