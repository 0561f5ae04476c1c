"""Diagnostic: per-agent IPM iteration counts and per-round solver time over consecutive cfg3
rounds (the bench's workload), saved for the round-scheduling study (tools/dataflow_sim.py).
Usage: python tools/iter_hist.py OUT.npz [rounds] [agents]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from cmpc import scenarios as S  # noqa: E402
from cmpc.rounds import DIRounds  # noqa: E402

out = sys.argv[1]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 200
agents = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
sc = S.make_di(agents, 30, 2, 2)
R = DIRounds(sc)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(rounds)]
it = torch.empty((rounds, R.B), dtype=torch.int32, device=R.dev)
kk = torch.empty((rounds, R.B), dtype=torch.float64, device=R.dev)
st = torch.empty((rounds, R.B), dtype=torch.int32, device=R.dev)
for r in range(rounds):
    R.bind_outputs(kk[r], it[r], st[r])
    R.step(timer=ev[r])
    if r % 50 == 0:
        torch.cuda.synchronize()
        print(f"round {r}", flush=True)
torch.cuda.synchronize()
ms = np.array([a.elapsed_time(b) for a, b in ev])
itn = it.cpu().numpy()
np.savez(out, iters=itn, ms=ms, status=st.cpu().numpy(), kkt=kk.cpu().numpy(), nbr=sc.nbr)
print("mean iters", itn.mean(), "mean max", itn.max(1).mean(), "ms mean", ms[5:].mean())
