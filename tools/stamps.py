"""Diagnostic: per-section shader-clock breakdown of the v3 solver kernel.
Usage: python tools/stamps.py [agents] [N]          cfg3 round-0 problem (double integrator), solved by
                                                    the fused round (rows built in the launch: the
                                                    bench's path); --unfused: build() + solve()
       python tools/stamps.py --lpv [round]         bench.py's lpv_rounds population (nx 9) at that
                                                    round (default 6: the slowest of the line)"""
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

SLOTS = 16
NAMES = {14: "setup", 0: "residual: Q X, C'lam", 1: "residual: 2 adjoints", 2: "residual: rows, norms",
         3: "W_k build", 4: "K: Gamma rec + MFMA", 5: "K: diag adds", 6: "chol: 16x16 factors",
         7: "chol: panel + SYRK", 8: "solve: rho, C'rho", 9: "solve: adjoint", 10: "solve: tri-solves",
         11: "solve: fwd sim", 12: "solve: rows, step", 13: "update"}
UNFUSED = "--unfused" in sys.argv
if UNFUSED:
    sys.argv.remove("--unfused")
WAVES = 0  # --one-wave / --two-waves: CMPC_FLAG_ONE_WAVE / CMPC_FLAG_TWO_WAVES (default: the library's choice)
for a_, f_ in (("--one-wave", L.CMPC_FLAG_ONE_WAVE), ("--two-waves", L.CMPC_FLAG_TWO_WAVES)):
    if a_ in sys.argv:
        sys.argv.remove(a_)
        WAVES = f_
LPV = len(sys.argv) > 1 and sys.argv[1] == "--lpv"
if LPV:
    import bench
    from cmpc.rounds import LPVRounds

    bp, args, kw = bench.lpv_population(None, rescue=False)
    R = LPVRounds(bp, *args, **kw)
    for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 6):
        R.step(halt=False)
    R.gather()
    n, N = R.B, R.N

    class _Opt:   # R.opts -> the planner's options (the LPV solve reads bp.opts)
        def __set__(self, obj, v):
            bp.opts = v

    type(R).opts = _Opt()
else:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    sc = S.make_di(n, N, 2, 2)
    R = DIRounds(sc)
    R.build()
    if not UNFUSED:
        R.solve = R.build_solve
st = torch.zeros((n, SLOTS), dtype=torch.int64, device="cuda")
R.opts = L.opts(stamps=st.data_ptr(), flags=WAVES)
for _ in range(3):
    R.solve()
torch.cuda.synchronize()
ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
ev[0].record()
R.solve()
ev[1].record()
torch.cuda.synchronize()
a = st.cpu().numpy().astype(np.float64)
print("stamped run: status", dict(zip(*np.unique(R.status.cpu().numpy(), return_counts=True))),
      "kkt max", float(R.kkt.max()), "iters", dict(zip(*np.unique(R.iters.cpu().numpy(), return_counts=True))))
it = a[:, SLOTS - 1]
tot = a[:, :SLOTS - 1].sum(1)
print(f"agents {n} N {N}: kernel {ev[0].elapsed_time(ev[1]):.3f} ms (with stamps); iters mean {it.mean():.2f} "
      f"max {it.max():.0f}")
for i in sorted(NAMES, key=lambda i: (i != 14, i)):
    print(f"  {NAMES[i]:24s} {a[:, i].mean() / it.mean():10.0f} clk/iter   {100 * a[:, i].sum() / tot.sum():5.1f} %")
print(f"  total                    {tot.mean() / it.mean():10.0f} clk/iter ; slowest agent {tot.max():.0f} clk")
R.opts = L.opts(flags=WAVES)
ev[0].record()
R.solve()
ev[1].record()
torch.cuda.synchronize()
print(f"kernel without stamps {ev[0].elapsed_time(ev[1]):.3f} ms; status "
      f"{dict(zip(*np.unique(R.status.cpu().numpy(), return_counts=True)))}")
