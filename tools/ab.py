"""Diagnostic A/B of the solver kernels (v3 default, generic) on a cfg3-style
device-resident batch: time per launch, iterations, status, max |z - z_v3| and max
|z - z_oracle| on a sample.  Usage: python tools/ab.py [agents] [N] [nb] [dim] [rounds]"""
import ctypes as ct
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import cmpc  # noqa: E402
from cmpc import _lib as L  # noqa: E402
from cmpc import scenarios as S  # noqa: E402
from cmpc.rounds import DIRounds  # noqa: E402
from oracle import cmpc_oracle as CO  # noqa: E402

a = [int(v) for v in sys.argv[1:]] + [None] * 5
n, N, nb, dim, rounds = a[0] or 1024, a[1] or 30, a[2] if a[2] is not None else 2, a[3] or 2, a[4] or 3
sc = S.make_di(n, N, nb, dim)
R = DIRounds(sc)
for rnd in range(rounds):
    R.build()
    prob = R.snapshot()
    res = {}
    for name, flag in (("v3", 0), ("generic", L.CMPC_FLAG_GENERIC)):
        R.opts = L.opts(flags=flag)
        R.solve()
        torch.cuda.synchronize()
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        R.solve()
        ev[1].record()
        torch.cuda.synchronize()
        res[name] = (ev[0].elapsed_time(ev[1]), R.z.cpu().numpy().copy(), R.iters.cpu().numpy().copy(),
                     R.status.cpu().numpy().copy(), R.kkt.cpu().numpy().copy())
    m = min(n, 256)
    p = dict(prob)
    for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
        p[k] = prob[k][:m]
    zc = CO.solve_batch(p, nthreads=16)[0]
    for name, (ms, z, it, st, kk) in res.items():
        print(f"round {rnd} {name:8s} {ms:8.3f} ms  iters mean {it.mean():.2f} max {it.max()}  "
              f"status {dict(zip(*np.unique(st, return_counts=True)))}  max kkt {kk.max():.1e}  "
              f"|z-z_v3| {np.abs(z - res['v3'][1]).max():.1e}  |z-z_cpu|[:{m}] {np.abs(z[:m] - zc).max():.1e}",
              flush=True)
    R.opts = L.opts()
    R.solve()
    R.advance()
    R.exchange()
