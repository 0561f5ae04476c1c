"""GPU check of the lane-per-agent kernel (mpc_lane.hip) on BASELINE cfg5 problems: statuses,
iterations, launch times and agreement with (a) the fp64 stage-wise Riccati kernel (double-double
near the solution) on every agent and (b) the C restatement (Riccati, newton 1) on a sample.

  python tools/lane_check.py [--agents 8192] [--rounds 3] [--sample 128] [--reps 3]
"""
import argparse
import ctypes as ct
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--sample", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--lanes", action="store_true", help="histogram of unsolved agents over the lane index")
    ap.add_argument("--only", default=None, help="run one solver only: riccati_f64 | lane_f64 | lane_fp32")
    a = ap.parse_args()
    import torch

    import cmpc
    from cmpc import _lib as L
    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    R = DIRounds(S.make_di(a.agents, 50, 2, 3), fused=False)
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        R.step()
    R.build()
    torch.cuda.synchronize()
    print(f"setup: {a.rounds} fp64 Riccati rounds in {time.perf_counter() - t0:.1f} s", flush=True)
    out = {}

    def run(name, flags, tol=None):
        R.opts = L.opts(tol, None, flags)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e in ev:
            e[0].record()
            R.solve()
            e[1].record()
        torch.cuda.synchronize()
        ms = [x.elapsed_time(y) for x, y in ev]
        z = R.z.cpu().numpy().copy()
        st = R.status.cpu().numpy().copy()
        it = R.iters.cpu().numpy().copy()
        kkt = R.kkt.cpu().numpy().copy()
        u, c = np.unique(st, return_counts=True)
        print(f"{name}: ms {['%.2f' % m for m in ms]} -> {a.agents / (min(ms) * 1e-3):.0f} QP/s | status "
              f"{dict(zip(u.tolist(), c.tolist()))} | iters mean {it.mean():.2f} max {it.max()} | kkt max {kkt.max():.2e}",
              flush=True)
        if a.lanes:
            bad = st != 1
            print("   not-solved by lane b%32:", np.bincount(np.flatnonzero(bad) % 32, minlength=32).tolist(), flush=True)
        out[name] = dict(ms=min(ms), qps=a.agents / (min(ms) * 1e-3), status=dict(zip(map(int, u), map(int, c))),
                         iters_mean=float(it.mean()), iters_max=int(it.max()))
        return z, st, it

    if a.only:
        flags = dict(riccati_f64=L.CMPC_FLAG_RICCATI, lane_f64=L.CMPC_FLAG_LANE, lane_fp32=L.CMPC_FLAG_FP32)[a.only]
        run(a.only, flags, 1e-6 if a.only == "lane_fp32" else None)
        return
    zr, sr, _ = run("riccati_f64", L.CMPC_FLAG_RICCATI)
    zl, sl, _ = run("lane_f64", L.CMPC_FLAG_LANE)
    zf, sf, _ = run("lane_fp32", L.CMPC_FLAG_FP32, 1e-6)
    for name, z, st in (("lane_f64", zl, sl), ("lane_fp32", zf, sf)):
        err = np.abs(z - zr) / np.maximum(1.0, np.abs(zr))
        e = err.max(1)
        both = (st == 1) & (sr == 1)
        print(f"{name} vs riccati_f64: rel err max {e.max():.2e} p99 {np.quantile(e, 0.99):.2e} median "
              f"{np.median(e):.2e}; both solved {both.mean():.4f}, max there {e[both].max():.2e}", flush=True)
        out[name]["err_vs_riccati"] = float(e.max())
        out[name]["err_vs_riccati_solved"] = float(e[both].max())
    if not a.no_oracle:
        from oracle import cmpc_oracle as CO

        prob = R.snapshot()
        ns = a.sample
        p = dict(prob)
        for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
            p[k] = prob[k][:ns]
        zc, kc, ic, stc = CO.solve_batch(p, nthreads=min(16, os.cpu_count() or 1), newton=1)
        d = np.abs(zl[:ns] - zc).max(1)
        same = (sl[:ns] == stc)
        print(f"lane_f64 vs oracle newton 1 (sample {ns}): status agree {same.mean():.3f}, max |dz| {d.max():.2e}, "
              f"median {np.median(d):.2e}; oracle status {np.unique(stc, return_counts=True)}", flush=True)
        out["oracle_sample"] = dict(n=ns, status_agree=float(same.mean()), max_dz=float(d.max()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
