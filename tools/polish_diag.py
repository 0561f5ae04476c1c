"""Diagnostic (GPU): bench.py's lpv_rounds population for ROUNDS device-resident rounds with the default
policy (rescue + polish); every round's agents that end at status 2, and sampled agents whose z differs
from the C restatement by more than 1e-7 while both report status 1, are saved as structured problems
(the GPU builder's arrays read back) with the GPU's z / status / kkt, for CPU replays
(oracle/cmpc_oracle.c -DPOLISH_DEBUG).

  python tools/polish_diag.py OUT.npz [rounds]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    import torch

    import bench
    from cmpc import _lib as L
    from cmpc.rounds import LPVRounds
    from cmpc.solver import plan
    from oracle import cmpc_oracle as CO

    out, rounds = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 22
    ctx = L.default_context()
    bp, args, kw = bench.lpv_population(ctx)
    R = LPVRounds(bp, *args, **kw)
    keep = {}
    rng = np.random.default_rng(11)
    for k in range(rounds):
        R.gather()
        R.solve()
        torch.cuda.synchronize()
        st = R.status.cpu().numpy()
        smp = np.sort(rng.choice(R.B, 128, replace=False)) if k >= 2 else np.zeros(0, int)
        sel = np.union1d(np.flatnonzero((st == 2) | (st == -10)), smp)
        if len(sel):
            prm = bp.prm
            rows = R.last_rows
            xl = R.x_last.cpu().numpy().reshape(-1)[: R.B * rows * 9].reshape(R.B, rows, 9)[sel]
            b = bp.build(xl, R.u_last.cpu().numpy()[sel], R.x_agents.cpu().numpy()[sel], R.pose.cpu().numpy()[sel])
            P = dict(nx=9, nu=2, N=bp.N, ns=3, mc=4 + R.nb, Q=np.array(prm.Q[:]).reshape(9, 9),
                     R=np.array(prm.R[:]).reshape(2, 2), dR=np.array(prm.dR[:]).reshape(2, 2), Qs=np.array(prm.Qs[:]),
                     u_ub=np.array([prm.max_rs, prm.max_ac]), u_lb=np.array([-prm.max_ls, -prm.max_dc]),
                     row_slack=np.array([-1, 0, 1, 1] + [2] * R.nb), row_sign=np.array([1, 1, 1, 1] + [-1] * R.nb),
                     A=b["A"], B=b["B"], x0=R.x0.cpu().numpy()[sel], u_prev=R.u_old.cpu().numpy()[sel],
                     qlin=b["qlin"], C=b["C"], h=b["h"])
            amax = plan(P, 1, rescue=True, polish=True)["polish_max_active"]  # the GPU layout's capacity
            zc, kc, ic, sc = CO.solve_batch_rescue(P, nthreads=16, polish=True, polish_amax=amax)
            zg, sg, kg = R.z.cpu().numpy()[sel], st[sel], R.kkt.cpu().numpy()[sel]
            err = np.abs(zg - zc).max(1)
            pick = (sg == 2) | (sg == -10) | ((sg == 1) & (sc == 1) & (err > 1e-7))
            print(f"round {k}: status 2 {int((st == 2).sum())}; C status on them {sc[sg == 2].tolist()}; "
                  f"sample both-solved max err {err[(sg == 1) & (sc == 1)].max() if ((sg == 1) & (sc == 1)).any() else 0:.2e}",
                  flush=True)
            for key in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
                keep.setdefault(key, []).append(P[key][pick])
            for key, v in (("z_gpu", zg), ("st_gpu", sg), ("kkt_gpu", kg), ("z_cpu", zc), ("st_cpu", sc),
                           ("kkt_cpu", kc), ("round", np.full(len(sel), k)), ("agent", sel)):
                keep.setdefault(key, []).append(v[pick])
            shared = {key: P[key] for key in ("nx", "nu", "N", "ns", "mc", "Q", "R", "dR", "Qs", "u_ub", "u_lb",
                                               "row_slack", "row_sign")}
        R.advance()
        R.exchange()
    np.savez_compressed(out, **{k: np.concatenate(v) for k, v in keep.items()}, **shared)


if __name__ == "__main__":
    main()
