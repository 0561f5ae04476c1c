"""Lab (GPU): the cfg5 fp32 path's closed-loop rounds (bench.py's cfg5 fp32 line: 8192 agents, 2 + 10
rounds); every agent whose solve ends with KKT > 1e-6 is saved with its structured problem (the round's
rows materialised by the builder, bit-identical to the fused launch's) for the CPU lab
(tools/f32_lab.py / oracle RIC_F32).

  python tools/f32_capture.py OUT.npz [rounds]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    import torch

    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    out = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    R = DIRounds(S.make_di(8192, 50, 2, 3), fp32=True)
    keep = {}
    for k in range(rounds):
        R.build()
        P = R.snapshot()
        R.step()
        torch.cuda.synchronize()
        kk, st, it = R.kkt.cpu().numpy(), R.status.cpu().numpy(), R.iters.cpu().numpy()
        bad = np.flatnonzero((kk > 1e-6) | ~np.isin(st, (1, 2)))
        print(f"round {k}: status {dict(zip(*np.unique(st, return_counts=True)))} max kkt {kk.max():.2e} "
              f"iters max {it.max()} bad {bad.tolist()}", flush=True)
        for a in bad:
            for key in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
                keep.setdefault(key, []).append(P[key][a])
            for key, v in (("kkt", kk[a]), ("status", st[a]), ("iters", it[a]), ("round", k), ("agent", a),
                           ("z", R.z.cpu().numpy()[a])):
                keep.setdefault(key, []).append(v)
    shared = {k: np.asarray(v) for k, v in R.shared.items() if isinstance(v, (np.ndarray, int, float))}
    np.savez(out, **{k: np.asarray(v) for k, v in keep.items()}, **{"shared_" + k: v for k, v in shared.items()})
    print("saved", len(keep.get("kkt", [])), "agents to", out)


if __name__ == "__main__":
    main()
