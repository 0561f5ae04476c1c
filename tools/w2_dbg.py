"""Lab (GPU): the first interior-point iteration at which the v3 kernel's two-wave mode departs from one
wave — the fused cfg3 round 0 of a small population solved with max_iter = 1, 2, ... under
CMPC_FLAG_ONE_WAVE and CMPC_FLAG_TWO_WAVES; prints z / kkt differences per cap.

  python tools/w2_dbg.py [agents] [max_cap]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def solve(agents, cap, flags):
    import torch

    from cmpc import _lib as L
    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    R = DIRounds(S.make_di(agents, 30, 2, 2), max_iter=cap)
    R.opts = L.opts(max_iter=cap, flags=flags)
    R.build_solve()
    torch.cuda.synchronize()
    return R.z.cpu().numpy(), R.kkt.cpu().numpy(), R.iters.cpu().numpy(), R.status.cpu().numpy()


def main():
    from cmpc import _lib as L

    agents = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    cap = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    for m in range(1, cap + 1):
        z1, k1, i1, s1 = solve(agents, m, L.CMPC_FLAG_ONE_WAVE)
        z2, k2, i2, s2 = solve(agents, m, L.CMPC_FLAG_TWO_WAVES)
        z3, _, _, _ = solve(agents, m, L.CMPC_FLAG_TWO_WAVES)
        z4, _, _, _ = solve(agents, m, L.CMPC_FLAG_ONE_WAVE)
        print(f"   repeat: two waves |dz| {np.abs(z2 - z3).max():.3e}, one wave |dz| {np.abs(z1 - z4).max():.3e}")
        print(f"max_iter {m}: |dz| {np.abs(z1 - z2).max():.3e} |dkkt| {np.abs(k1 - k2).max():.3e} "
              f"iters {np.array_equal(i1, i2)} status {np.array_equal(s1, s2)} kkt1 {k1[:3]} kkt2 {k2[:3]}", flush=True)




def merits(agents, cap, flags):
    """(lab build -DCMPC_DBG_MERIT) the merit of iterations 1..15 per agent"""
    import torch

    from cmpc import _lib as L
    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    R = DIRounds(S.make_di(agents, 30, 2, 2), max_iter=cap)
    st = torch.zeros((agents, 16), dtype=torch.int64, device="cuda")
    R.opts = L.opts(max_iter=cap, flags=flags, stamps=st.data_ptr())
    R.build_solve()
    torch.cuda.synchronize()
    return st.cpu().numpy().view(np.float64)


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "merit":
        from cmpc import _lib as L

        a, m = int(sys.argv[1]), int(sys.argv[2])
        m1, m2 = merits(a, m, L.CMPC_FLAG_ONE_WAVE), merits(a, m, L.CMPC_FLAG_TWO_WAVES)
        for i in range(a):
            print(i, "one", " ".join(f"{v:.6e}" for v in m1[i, 1:m + 1]))
            print(i, "two", " ".join(f"{v:.6e}" for v in m2[i, 1:m + 1]))
    else:
        main()
