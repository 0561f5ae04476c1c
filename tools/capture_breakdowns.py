"""Capture agent-QPs on which the condensed factorisation breaks down (status CMPC_UNSOLVED):
closed-loop LPV rounds (cmpc.rounds.LPVRounds, 341 jittered copies of the reference's 3-agent
N = 30 run, rescue off) until a round has such agents; their structured problems (the GPU LPV
builder's A, B, qlin, C, h plus x0, u_old and the shared weights) go to an npz for the CPU lab
(tools/ipm_lab.py-style replays through oracle/cmpc_oracle.c).

  python tools/capture_breakdowns.py OUT.npz [max_rounds]
"""
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    import torch

    import cmpc
    from cmpc import _lib as L
    from cmpc.rounds import LPVRounds

    out, max_rounds = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30
    d = np.load(os.path.join(ROOT, "tests", "golden", "lpv_n30_a3.npz"), allow_pickle=False)
    t = np.load(os.path.join(ROOT, "tests", "golden", "track_highway.npz"), allow_pickle=False)
    track = types.SimpleNamespace(PointAndTangent=t["PointAndTangent"], halfWidth=t["halfWidth"], lane=int(t["lane"]))
    N, dt, reps = int(d["N"]), float(d["dt"]), 341
    sel = sorted([j for j in range(len(d["step"])) if d["step"][j] == 0], key=lambda j: d["agent"][j])
    x0 = np.tile(d["x0"][sel], (reps, 1))
    x0[:, 0] *= np.repeat(1.0 + 0.02 * np.random.default_rng(5).uniform(-1, 1, reps), 3)
    g3 = np.arange(3 * reps) // 3 * 3
    nbr = np.sort(np.stack([g3 + (np.arange(3 * reps) + 1) % 3, g3 + (np.arange(3 * reps) + 2) % 3], 1), 1)
    Q = np.diag([10.0, 0.0, 0.0, 25.0, 10.0, 0.0, 0.0, 0.0, 0.0])
    model = dict(lf=0.125, lr=0.125, m=1.98, I=0.09, Cf=70.0, Cr=70.0, mu=0.05)
    lim = dict(vx_ref=float(d["vx_ref"]), min_dist=0.25, max_vel=5.5, min_vel=0.0, max_rs=0.3, max_ls=0.3,
               max_ac=5.0, max_dc=10.0, sm=0.9)
    bp = cmpc.PlannerLPVBatch(Q, 1e7 * np.eye(3), 0.0 * np.eye(2), 50.0 * np.eye(2), N, dt, track, 5.0, model, lim)
    bp.opts = L.opts()
    R = LPVRounds(bp, x0, np.tile(np.stack([d[f"x_last_{j}"] for j in sel]), (reps, 1, 1)),
                  np.tile(np.stack([d[f"u_last_{j}"] for j in sel]), (reps, 1, 1)), nbr,
                  u_old=np.tile(d["u_old"][sel], (reps, 1)), traj=np.tile(d["pose"][sel], (reps, 1, 1)))
    saved = []
    for rnd in range(max_rounds):
        R.gather()
        R.solve()
        torch.cuda.synchronize()
        st = R.status.cpu().numpy()
        bad = np.flatnonzero(st == cmpc.CMPC_UNSOLVED)
        if len(bad):
            rows = R.last_rows
            xl = R.x_last.cpu().numpy().reshape(-1)[: R.B * rows * 9].reshape(R.B, rows, 9)[bad]
            ul = R.u_last.cpu().numpy()[bad]
            xa = R.x_agents.cpu().numpy()[bad]
            po = R.pose.cpu().numpy()[bad]
            b = bp.build(xl, ul, xa, po)
            saved.append(dict(round=np.full(len(bad), rnd), agent=bad, x0=R.x0.cpu().numpy()[bad],
                              u_prev=R.u_old.cpu().numpy()[bad], A=b["A"], B=b["B"], qlin=b["qlin"], C=b["C"],
                              h=b["h"], z_gpu=R.z.cpu().numpy()[bad], iters=R.iters.cpu().numpy()[bad]))
            print(f"round {rnd}: {len(bad)} breakdowns", flush=True)
        R.advance()
        R.exchange()
    cat = {k: np.concatenate([s[k] for s in saved]) for k in saved[0]} if saved else {}
    shared = dict(nx=9, nu=2, N=N, ns=3, mc=6, Q=Q, R=np.zeros((2, 2)), dR=50.0 * np.eye(2), Qs=1e7 * np.ones(3),
                  u_ub=np.array([0.3, 5.0]), u_lb=np.array([-0.3, -10.0]), row_slack=np.array([-1, 0, 1, 1, 2, 2]),
                  row_sign=np.array([1, 1, 1, 1, -1, -1]))
    np.savez(out, **cat, **{f"s_{k}": np.asarray(v) for k, v in shared.items()})


if __name__ == "__main__":
    main()
