"""Diagnostic: save the structured problems of the first R cfg3 rounds (as solved on the GPU)
to gpurun_out/snap/round<r>.npz with the GPU iteration counts, for CPU-side analysis.
Usage: python tools/snap_rounds.py [R]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
import torch  # noqa: E402,F401

from cmpc import scenarios as S  # noqa: E402
from cmpc.rounds import DIRounds  # noqa: E402

R_ = int(sys.argv[1]) if len(sys.argv) > 1 else 3
out = os.path.join(ROOT, "gpurun_out", "snap")
os.makedirs(out, exist_ok=True)
R = DIRounds(S.make_di(1024, 30, 2, 2))
for r in range(R_):
    R.build()
    R.solve()
    p = R.snapshot()
    arrs = {k: np.asarray(v) for k, v in p.items() if isinstance(v, (np.ndarray, float, int))}
    arrs["gpu_iters"] = R.iters.cpu().numpy()
    arrs["gpu_z"] = R.z.cpu().numpy()
    np.savez_compressed(os.path.join(out, f"round{r}.npz"), **arrs)
    print(r, sorted(arrs), flush=True)
    R.advance()
    R.exchange()
