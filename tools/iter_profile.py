"""Diagnostic: IPM iteration distribution over consecutive cfg3 rounds and its sensitivity to
the termination tolerance (kernel time = slowest wave, so the iteration tail sets it).
Usage: python tools/iter_profile.py [rounds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from cmpc import _lib as L  # noqa: E402
from cmpc import scenarios as S  # noqa: E402
from cmpc.rounds import DIRounds  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
sc = S.make_di(1024, 30, 2, 2)
R = DIRounds(sc)
ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
tols = (1e-9, 1e-8, 1e-7, 1e-6)
for r in range(rounds):
    R.build()
    res = {}
    for tol in tols:
        R.opts = L.opts(tol)
        R.solve()
        ev[0].record()
        R.solve()
        ev[1].record()
        torch.cuda.synchronize()
        res[tol] = (R.z.clone(), R.iters.cpu().numpy().copy(), R.kkt.cpu().numpy().copy(),
                    R.status.cpu().numpy().copy(), ev[0].elapsed_time(ev[1]))
    z0 = res[tols[0]][0]
    it0 = res[tols[0]][1]
    hist = np.bincount(it0, minlength=25)[4:25]
    print(f"round {r}: iters hist[4..24] {hist.tolist()}")
    for tol in tols:
        z, it, kkt, st, ms = res[tol]
        dz = float((z - z0).abs().max())
        print(f"   tol {tol:.0e}: {ms:.3f} ms iters mean {it.mean():.2f} p99 {np.percentile(it, 99):.0f} "
              f"max {it.max()} maxkkt {kkt.max():.1e} max|z-z(1e-9)| {dz:.1e} status "
              f"{dict(zip(*np.unique(st, return_counts=True)))}")
    # slowest agents at the default tolerance
    worst = np.argsort(-it0)[:5]
    print(f"   slowest agents {worst.tolist()} iters {it0[worst].tolist()}")
    R.opts = L.opts()
    R.solve()
    R.advance()
    R.exchange()
