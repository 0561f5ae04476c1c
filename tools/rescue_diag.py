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
    st_buf = torch.zeros((R.B, 16), dtype=torch.int64, device="cuda")
    cmpc.solve_mpc(P, ctx, rescue=True, stamps=st_buf.data_ptr())
    stamps = st_buf.cpu().numpy().astype(np.float64)
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
    # Riccati stamps of the continued agents (they overwrite the condensed kernel's): tools/ric_stamps.py slots
    names = {0: "residuals", 1: "stage weights", 2: "factor", 3: "factor dd", 4: "rhs", 5: "solve", 6: "refinement",
             7: "rows/step", 8: "update", 14: "setup+output"}
    sel = idx[:8]
    print("Riccati clocks (M) of the first continued agents: " + ", ".join(f"{a}" for a in sel))
    for k_, nm in names.items():
        print(f"  {nm:14s} " + " ".join(f"{stamps[a, k_] / 1e6:7.3f}" for a in sel))
    print(f"  {'dd iterations':14s} " + " ".join(f"{stamps[a, 12]:7.0f}" for a in sel))
    print(f"  {'refine steps':14s} " + " ".join(f"{stamps[a, 13]:7.0f}" for a in sel))


if __name__ == "__main__":
    main()
