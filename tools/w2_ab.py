"""Lab A/B of the v3 kernel's two-wave mode (W2) on the bench's fused cfg3 round (DIRounds): the same
rounds with one wavefront per agent (CMPC_FLAG_ONE_WAVE) and two (CMPC_FLAG_TWO_WAVES); per-round kernel
time (HIP events on the launch stream), and z / iterations / statuses compared bit for bit.

  python tools/w2_ab.py [agents] [rounds]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def run(agents, rounds, flags):
    import torch

    from cmpc import _lib as L
    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    R = DIRounds(S.make_di(agents, 30, 2, 2))
    R.opts = L.opts(flags=flags)
    zs, its, ms = [], [], []
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    for _ in range(rounds):
        ev[0].record()
        R.build_solve()
        ev[1].record()
        torch.cuda.synchronize()
        ms.append(ev[0].elapsed_time(ev[1]))
        zs.append(R.z.cpu().numpy().copy())
        its.append(R.iters.cpu().numpy().copy())
        R.advance()
        R.exchange()
    return np.array(zs), np.array(its), np.array(ms)


def main():
    from cmpc import _lib as L

    agents = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    z1, i1, m1 = run(agents, rounds, L.CMPC_FLAG_ONE_WAVE)
    z2, i2, m2 = run(agents, rounds, L.CMPC_FLAG_TWO_WAVES)
    za, ia, ma = run(agents, rounds, 0)
    w = slice(2, None)
    print(f"agents {agents}, {rounds} rounds: kernel ms (rounds 2..) one wave {m1[w].mean():.4f}, two waves "
          f"{m2[w].mean():.4f} ({m1[w].mean() / m2[w].mean():.3f}x), auto {ma[w].mean():.4f}; "
          f"max iterations per round {i1.max(1)[:10].tolist()}")
    print(f"bit-equal z {np.array_equal(z1, z2)} iterations {np.array_equal(i1, i2)}; auto vs one wave "
          f"{np.array_equal(za, z1)}; max |dz| {np.abs(z1 - z2).max():.2e}")


if __name__ == "__main__":
    main()
