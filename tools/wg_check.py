"""Diagnostic: workgroup-per-agent solver (fp64 N*nu > 64, fp32 cfg5) vs the C restatement."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]
import torch  # noqa: E402,F401

import cmpc  # noqa: E402
from cmpc import scenarios as S  # noqa: E402
from oracle import cmpc_oracle as CO  # noqa: E402
from oracle import synth  # noqa: E402

for (n, N, nb, dim, fp32) in [(48, 40, 2, 2, False), (64, 50, 2, 3, True), (64, 20, 2, 3, True), (64, 30, 2, 2, False)]:
    sc = S.make_di(n, N, nb, dim)
    P = synth.structured(sc.shared, sc.params, sc.A, sc.B, sc.x0, sc.u_prev, sc.lane, sc.nbr, sc.traj, np.arange(n))
    z, kkt, it, st = cmpc.solve_mpc(P, fp32=fp32)
    zc, kc, ic, stc = CO.solve_batch(P, nthreads=16)
    err = np.abs(z - zc) / np.maximum(1.0, np.abs(zc))
    print(f"n{n} N{N} dim{dim} fp32={fp32}: gpu status {dict(zip(*np.unique(st, return_counts=True)))} iters "
          f"{it.mean():.1f}/{it.max()} kkt {np.nanmax(kkt):.1e}; cpu status "
          f"{dict(zip(*np.unique(stc, return_counts=True)))} iters {ic.mean():.1f}; max rel err {np.nanmax(err):.2e}",
          flush=True)
