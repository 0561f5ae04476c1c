"""cfg5 diagnostics on the GPU: device-resident rounds of the BASELINE cfg5 population (8192
agents, N=50, nx=6 nu=3, fp64 Riccati kernel), per-round solver time, iteration histogram and
status counts; the problems of agents that end unsolved or in the iteration tail are saved
(host copies, sliced) so the C restatement can replay them on the CPU.

  python tools/cfg5_diag.py [--rounds 6] [--out gpurun_out/cfg5_diag]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=8192)
    ap.add_argument("--horizon", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--tail", type=int, default=8, help="agents saved per round from the iteration tail")
    ap.add_argument("--max-iter", type=int, default=None)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "cfg5_diag"))
    args = ap.parse_args()
    import torch

    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    os.makedirs(args.out, exist_ok=True)
    scen = S.make_di(args.agents, args.horizon, 2, 3)
    R = DIRounds(scen, max_iter=args.max_iter)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    log = []
    for r in range(args.rounds):
        R.build()
        prob = R.snapshot()
        ev[0].record()
        R.solve()
        ev[1].record()
        torch.cuda.synchronize()
        it = R.iters.cpu().numpy()
        st = R.status.cpu().numpy()
        kkt = R.kkt.cpu().numpy()
        bad = np.flatnonzero(st != 1)
        tail = np.argsort(-it, kind="stable")[: args.tail]
        sel = np.unique(np.concatenate([bad, tail]))
        keep = {k: v for k, v in prob.items() if not isinstance(v, np.ndarray)}
        for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
            keep[k] = prob[k][sel]
        for k, v in prob.items():
            if isinstance(v, np.ndarray) and k not in keep:
                keep[k] = v
        np.savez(os.path.join(args.out, f"round{r}.npz"), agents=sel, iters=it[sel], status=st[sel], kkt=kkt[sel],
                 z=R.z.cpu().numpy()[sel], **keep)
        hist = {int(k): int(v) for k, v in zip(*np.unique(it, return_counts=True))}
        rec = {"round": r, "solve_ms": ev[0].elapsed_time(ev[1]), "iters_mean": float(it.mean()),
               "iters_max": int(it.max()), "status": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
               "bad": [(int(a), int(st[a]), int(it[a]), float(kkt[a])) for a in bad], "hist": hist}
        log.append(rec)
        print(json.dumps(rec), flush=True)
        R.advance()
        R.exchange()
    with open(os.path.join(args.out, "log.json"), "w") as f:
        json.dump(log, f, indent=1)


if __name__ == "__main__":
    main()
