"""Lab: fused (cmpc_di_solve_dev) vs build-then-solve rounds of the cfg3 family: per round max |dz|,
agents that differ, iterations.  Usage: python tools/fused_check.py [agents] [rounds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]
import torch  # noqa: E402

from cmpc import scenarios as S  # noqa: E402
from cmpc.rounds import DIRounds  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
sc = S.make_di(n, 30, 2, 2)
F = DIRounds(sc, fused=True)
U = DIRounds(sc, fused=False)
for r in range(rounds):
    F.step()
    U.step()
    torch.cuda.synchronize()
    zf, zu = F.z.cpu().numpy(), U.z.cpu().numpy()
    d = np.abs(zf - zu).max(1)
    bad = np.flatnonzero(d > 0)
    print(f"round {r}: agents differing {len(bad)} max |dz| {d.max():.3e}; iters equal "
          f"{np.mean(F.iters.cpu().numpy() == U.iters.cpu().numpy()):.4f}; first {bad[:8].tolist()} "
          f"iters F {F.iters.cpu().numpy()[bad[:8]].tolist()} U {U.iters.cpu().numpy()[bad[:8]].tolist()}")
    if len(bad):
        a = bad[0]
        j = np.flatnonzero(np.abs(zf[a] - zu[a]) > 0)
        print(f"   agent {a}: {len(j)} entries differ, first {j[:10].tolist()}, values {zf[a][j[:3]].tolist()} vs "
              f"{zu[a][j[:3]].tolist()}")
