"""BASELINE cfg5: 8192 agents, N=50, 3-D dynamics (nx=6, nu=3), fp32 path with a tolerance
check against the fp64 reference.  Device-resident consensus rounds (build -> fp32
workgroup solve -> advance -> exchange) on one GPU; prints one JSON line.  The fp64
reference is the C restatement (oracle/cmpc_oracle.c) on a sample of the same round.
Usage: python tools/bench_cfg5.py [--agents 8192 --steps 5 --warmup 2 --sample 128]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=8192)
    ap.add_argument("--horizon", type=int, default=50)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sample", type=int, default=128)
    args = ap.parse_args()
    import torch

    import cmpc
    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds
    from oracle import cmpc_oracle as CO

    scen = S.make_di(args.agents, args.horizon, 2, 3)
    R = DIRounds(scen, fp32=True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for _ in range(args.warmup):
        R.step(timer=ev[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        R.step(timer=ev[k])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kern = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    st = R.status.cpu().numpy()
    # tolerance check of the next round's problem: fp32 GPU vs fp64 CPU restatement
    R.build()
    prob = R.snapshot()
    R.solve()
    torch.cuda.synchronize()
    zg = R.z.cpu().numpy()[: args.sample]
    p = dict(prob)
    for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
        p[k] = prob[k][: args.sample]
    zc, _, _, stc = CO.solve_batch(p, nthreads=min(16, os.cpu_count() or 1))
    err = np.abs(zg - zc) / np.maximum(1.0, np.abs(zc))
    print(json.dumps({
        "metric": "agent-QP solves/sec, BASELINE cfg5 (fp32 path, tolerance vs fp64)",
        "value": args.agents * args.steps / el, "unit": "agent-QP/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "kernel_ms_per_launch": kern, "dtype": "f32",
        "config": {"workload": f"cfg5: {args.agents} agents, N={args.horizon}, nx=6 nu=3, nb=2, fp32 workgroup "
                               f"solver; step = build+solve+advance+exchange"},
        "status_counts": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
        "fp64_check": {"sample": args.sample, "max_rel_err": float(err.max()),
                       "p99_rel_err": float(np.quantile(err.max(1), 0.99)),
                       "cpu_status_solved": int((stc == 1).sum())},
    }))


if __name__ == "__main__":
    main()
