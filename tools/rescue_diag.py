"""Diagnostic: the rescue hand-over (CMPC_FLAG_RESCUE) on the GPU against its C restatement, agent
by agent.  bench.py's lpv_rounds population is driven without the rescue to round R; that round's
problems (the GPU builder's, read back) are solved by cmpc.solve_mpc with and without the rescue
and by oracle.cmpc_oracle (newton 0 / the rescue policy); the agents the condensed method leaves
short of convergence are listed with both sides' iterations, statuses and the GPU kernel times.

  python tools/rescue_diag.py [round]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    import torch

    import bench
    import cmpc
    from cmpc.rounds import LPVRounds
    from oracle import cmpc_oracle as CO

    rnd = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ctx = cmpc.Context(0)
    bp, args, kw = bench.lpv_population(ctx, rescue=False)
    R = LPVRounds(bp, *args, **kw)
    for _ in range(rnd):
        R.step(halt=False)
    R.gather()
    torch.cuda.synchronize()
    smp = np.arange(R.B)
    rows = R.last_rows
    xl = R.x_last.cpu().numpy().reshape(-1)[: R.B * rows * 9].reshape(R.B, rows, 9)
    b = bp.build(xl, R.u_last.cpu().numpy(), R.x_agents.cpu().numpy(), R.pose.cpu().numpy())
    prm = bp.prm
    P = dict(nx=9, nu=2, N=bp.N, ns=3, mc=4 + R.nb, Q=np.array(prm.Q[:]).reshape(9, 9),
             R=np.array(prm.R[:]).reshape(2, 2), dR=np.array(prm.dR[:]).reshape(2, 2), Qs=np.array(prm.Qs[:]),
             u_ub=np.array([prm.max_rs, prm.max_ac]), u_lb=np.array([-prm.max_ls, -prm.max_dc]),
             row_slack=np.array([-1, 0, 1, 1] + [2] * R.nb, np.int32), row_sign=np.array([1, 1, 1, 1] + [-1] * R.nb, np.int32),
             A=b["A"], B=b["B"], qlin=b["qlin"], C=b["C"], h=b["h"], x0=R.x0.cpu().numpy()[smp],
             u_prev=R.u_old.cpu().numpy()[smp])
    out = {}
    for name, kw2 in (("plain", {}), ("rescue", {"rescue": True})):
        cmpc.solve_mpc(P, ctx, **kw2)
        t0 = time.perf_counter()
        z, k, it, st = cmpc.solve_mpc(P, ctx, **kw2)
        out[name] = (z, k, it, st, (time.perf_counter() - t0) * 1e3)
    zc0, _, ic0, sc0 = CO.solve_batch(P, nthreads=16)
    zc, kc, ic, sc = CO.solve_batch_rescue(P, nthreads=16)
    st0 = out["plain"][3]
    idx = np.flatnonzero(st0 != 1)
    print(f"round {rnd}: GPU plain {out['plain'][4]:.2f} ms, rescue {out['rescue'][4]:.2f} ms (host call, incl. copies)")
    print(" agent | GPU plain it/st | CPU plain it/st | GPU rescue it/st/kkt | CPU rescue it/st | |dz| rescue")
    for a in idx:
        zr, kr, ir, sr, _ = out["rescue"]
        print(f" {a:5d} | {out['plain'][2][a]:3d} {st0[a]:3d} | {ic0[a]:3d} {sc0[a]:3d} | {ir[a]:3d} {sr[a]:3d} {kr[a]:.1e} | "
              f"{ic[a]:3d} {sc[a]:3d} | {np.abs(zr[a] - zc[a]).max():.1e}")


if __name__ == "__main__":
    main()
