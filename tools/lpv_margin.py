"""Diagnostic (round 5): which agents of bench.py's lpv_rounds population sit near the
1e-6 parity bar against the C restatement, and why.

Replays the population's rounds on the GPU (deterministic), re-solves EVERY agent of every round with the C
restatement of the same rescue + polish policy (bench.lpv_check_round), and saves, for each agent whose
|z_gpu - z_cpu| exceeds --thr, its structured problem (the GPU builder's read-back arrays) with both sides'
z, status, iterations and KKT to gpurun_out/<tag>/margin.npz, for CPU analysis with the oracle's lab flags.
Usage: python tools/lpv_margin.py [--rounds 22] [--thr 1e-7] [--tag margin]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=22)
    ap.add_argument("--thr", type=float, default=1e-7)
    ap.add_argument("--tag", default="margin")
    a = ap.parse_args()
    import torch

    import bench
    import cmpc
    from cmpc.rounds import LPVRounds

    ctx = cmpc.Context(0)
    bp, args, kw = bench.lpv_population(ctx)
    R = LPVRounds(bp, *args, **kw)
    B = R.B
    out = os.path.join(ROOT, "gpurun_out", a.tag)
    os.makedirs(out, exist_ok=True)
    keep = {}
    summary = []
    allidx = np.arange(B)
    for r in range(a.rounds):
        R.gather()
        R.solve()
        torch.cuda.synchronize()
        zc, sc, P = bench.lpv_check_round(bp, R, allidx)
        zg = R.z.cpu().numpy()
        sg, ig, kg = R.status.cpu().numpy(), R.iters.cpu().numpy(), R.kkt.cpu().numpy()
        both = (sc == 1) & (sg == 1)
        e = np.abs(zg - zc).max(1)
        bad = np.flatnonzero(both & (e > a.thr))
        summary.append(dict(round=r, both=int(both.sum()), max_err=float(e[both].max()) if both.any() else 0.0,
                            n_over_thr=int(len(bad)), n_over_1e6=int((both & (e > 1e-6)).sum()),
                            status_gpu={int(k): int(v) for k, v in zip(*np.unique(sg, return_counts=True))},
                            status_cpu={int(k): int(v) for k, v in zip(*np.unique(sc, return_counts=True))}))
        print(json.dumps(summary[-1]), flush=True)
        for i in bad:
            tag = f"r{r}_a{i}"
            for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
                keep[f"{tag}_{k}"] = P[k][i]
            keep[f"{tag}_zg"], keep[f"{tag}_zc"] = zg[i], zc[i]
            keep[f"{tag}_info"] = np.array([r, i, sg[i], sc[i], ig[i], kg[i], e[i]])
        R.advance()
        R.exchange()
    for k in ("nx", "nu", "N", "ns", "mc", "Q", "R", "dR", "Qs", "u_ub", "u_lb", "row_slack", "row_sign"):
        keep[k] = np.asarray(P[k])
    np.savez_compressed(os.path.join(out, "margin.npz"), **keep)
    with open(os.path.join(out, "margin.json"), "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
