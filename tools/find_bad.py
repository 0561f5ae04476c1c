"""Diagnostic: run R consecutive cfg3 rounds on the GPU and save every round's structured
problem in which some agent ends neither solved nor solved-inaccurate to
gpurun_out/bad/round<r>.npz (with the GPU status / iterations / kkt / z), for CPU-side
analysis with the oracle.  Usage: python tools/find_bad.py [R]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
import torch  # noqa: E402

from cmpc import scenarios as S  # noqa: E402
from cmpc.rounds import DIRounds  # noqa: E402

R_ = int(sys.argv[1]) if len(sys.argv) > 1 else 120
out = os.path.join(ROOT, "gpurun_out", "bad")
os.makedirs(out, exist_ok=True)
R = DIRounds(S.make_di(1024, 30, 2, 2))
hist = []
for r in range(R_):
    R.build()
    R.solve()
    st = R.status.cpu().numpy()
    it = R.iters.cpu().numpy()
    hist.append((int(it.max()), float(it.mean())))
    bad = np.nonzero((st != 1) & (st != 2))[0]
    if bad.size:
        p = R.snapshot()
        arrs = {k: np.asarray(v) for k, v in p.items() if isinstance(v, (np.ndarray, float, int))}
        arrs.update(gpu_status=st, gpu_iters=it, gpu_kkt=R.kkt.cpu().numpy(), gpu_z=R.z.cpu().numpy(), bad=bad)
        np.savez_compressed(os.path.join(out, f"round{r}.npz"), **arrs)
        print(f"round {r}: bad agents {bad.tolist()} status {st[bad].tolist()} iters {it[bad].tolist()}", flush=True)
    R.advance()
    R.exchange()
torch.cuda.synchronize()
np.save(os.path.join(out, "iters_hist.npy"), np.array(hist))
print("max iters per round:", [h[0] for h in hist])
