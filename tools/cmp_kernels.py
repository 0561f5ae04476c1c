"""Diagnostic: generic vs specialised kernel on the captured LPV fixtures and a synthetic batch."""
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
from conftest import lpv_qps, LPV_CASES  # noqa
from oracle import lpv_ref as LR  # noqa

ctx = cmpc.Context(0)
g = LR.paper_gains()
tr = LR.Track.build("Highway")
for name in LPV_CASES:
    groups = {}
    for j, c in lpv_qps(name):
        groups.setdefault(c["x_last"].shape[0], []).append(c)
    for rows, cs in groups.items():
        N = cs[0]["N"]
        lim = LR.scaled_car_limits(cs[0]["vx_ref"])
        out = {}
        for flag in (0, 1):
            bp = cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], N, cs[0]["dt"], tr, g["wq"], LR.SCALED_CAR_MODEL,
                                      lim, ctx=ctx)
            bp.opts = L.opts(flags=flag)
            xa = np.stack([c["x_agents"] for c in cs])
            out[flag] = bp.solve(np.stack([c["x0"] for c in cs]), np.stack([c["x_last"] for c in cs]),
                                 np.stack([c["u_last"] for c in cs]), np.stack([c["u_old"] for c in cs]),
                                 xa if xa.shape[2] else None, np.stack([c["pose"] for c in cs]))
        zref = np.stack([c["z"] for c in cs])
        for flag, nm in ((0, "v2"), (1, "generic")):
            r = out[flag]
            print(f"{name} rows{rows} {nm:8s} status {r['status'].tolist()} iters {r['iters'].tolist()} "
                  f"kkt {np.array2string(r['kkt'], precision=1)} err {np.abs(r['z'] - zref).max():.1e}")
