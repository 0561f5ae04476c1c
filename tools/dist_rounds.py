"""Worker of the multi-rank GPU rounds test (tests/test_dist_gpu.py): one rank of the
device-resident consensus rounds (cmpc.rounds.DIRounds — HIP build / solve / advance; round 0
unfused, later rounds the fused build + solve of bench.py) with the
per-round exchange over torch.distributed.  Reads RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
and the backend from the environment (CMPC_DIST_BACKEND, default gloo: on a one-GPU box every
rank shares device 0, and RCCL refuses two ranks on one device).

Usage: python tools/dist_rounds.py OUT.npz N_AGENTS HORIZON ROUNDS SAMPLE
       python tools/dist_rounds.py lpv OUT.npz REPS ROUNDS   (LPVRounds, ring neighbours across ranks)
       python tools/dist_rounds.py lpv_halt OUT.npz REPS ROUNDS   (same, one infeasible agent on rank 0)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def run(n_agents, horizon, rounds, sample, rank=0, world=1, group=None):
    """Returns (traj_all per round, round-0 problem of the first `sample` local agents, their z)."""
    import torch

    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    scen = S.make_di(n_agents, horizon, 2, 2)
    R = DIRounds(scen, rank=rank, world=world, device=0, group=group)
    trajs, snap, z0 = [], None, None
    for r in range(rounds):
        if r == 0:   # build, snapshot, solve (the problems go to the C-restatement check)
            R.build()
            snap = R.snapshot()
            R.solve()
            z0 = R.z[:sample].cpu().numpy().copy()
            st = R.status.cpu().numpy()
            assert np.isin(st, (1, 2)).all(), np.unique(st, return_counts=True)
            R.advance()
            R.exchange()
        else:        # the bench's fused round (cmpc_di_solve_dev; rank > 0 reads traj_all at self_offset)
            R.step()
        torch.cuda.synchronize()
        trajs.append(R.traj_all.cpu().numpy().copy())
    prob = {k: (v[:sample] if isinstance(v, np.ndarray) and k in ("A", "B", "x0", "u_prev", "qlin", "C", "h")
                else v) for k, v in snap.items()}
    return np.stack(trajs), prob, z0


def run_lpv(reps, rounds, rank=0, world=1, group=None, offtrack=False):
    """Device-resident LPV rounds (cmpc.rounds.LPVRounds) of `reps` copies of the reference's
    3-agent N = 30 Highway run (tests/golden/lpv_n30_a3, step 0), ring neighbours (i+1, i+2 mod
    n: the same positions as each copy's own other two agents, but crossing the rank boundary).
    Returns (traj_all per round, this rank's z per round).  ``offtrack``: agent 0 (rank 0's) gets a
    previous prediction off the track (NaN s in one row: infeasible, status -10); every rank's
    LPVRounds.step must then raise InfeasibleRound in the first round with the node's count.
    Returns (raised, count, rounds completed) instead."""
    import types

    import torch

    import cmpc
    from cmpc.rounds import LPVRounds

    d = np.load(os.path.join(ROOT, "tests", "golden", "lpv_n30_a3.npz"), allow_pickle=False)
    t = np.load(os.path.join(ROOT, "tests", "golden", "track_highway.npz"), allow_pickle=False)
    track = types.SimpleNamespace(PointAndTangent=t["PointAndTangent"], halfWidth=t["halfWidth"], lane=int(t["lane"]))
    N, dt, n = int(d["N"]), float(d["dt"]), 3 * reps
    sel = sorted([j for j in range(len(d["step"])) if d["step"][j] == 0], key=lambda j: d["agent"][j])
    i = np.arange(n)
    nbr = np.sort(np.stack([(i + 1) % n, (i + 2) % n], 1), 1)
    Q = np.diag([10.0, 0.0, 0.0, 25.0, 10.0, 0.0, 0.0, 0.0, 0.0])
    model = dict(lf=0.125, lr=0.125, m=1.98, I=0.09, Cf=70.0, Cr=70.0, mu=0.05)
    lim = dict(vx_ref=float(d["vx_ref"]), min_dist=0.25, max_vel=5.5, min_vel=0.0, max_rs=0.3, max_ls=0.3,
               max_ac=5.0, max_dc=10.0, sm=0.9)
    ctx = cmpc.Context(0)
    bp = cmpc.PlannerLPVBatch(Q, 1e7 * np.eye(3), 0.0 * np.eye(2), 50.0 * np.eye(2), N, dt, track, 5.0, model, lim,
                              ctx=ctx)
    x_last = np.tile(np.stack([d[f"x_last_{j}"] for j in sel]), (reps, 1, 1))
    if offtrack:
        x_last[0, 3, 6] = np.nan
    R = LPVRounds(bp, np.tile(d["x0"][sel], (reps, 1)), x_last,
                  np.tile(np.stack([d[f"u_last_{j}"] for j in sel]), (reps, 1, 1)), nbr,
                  u_old=np.tile(d["u_old"][sel], (reps, 1)), traj=np.tile(d["pose"][sel], (reps, 1, 1)),
                  rank=rank, world=world, group=group)
    if offtrack:
        from cmpc.rounds import InfeasibleRound

        for r in range(rounds):
            try:
                R.step()
            except InfeasibleRound as e:
                return True, e.count, r
        return False, 0, rounds
    trajs, zs = [], []
    for _ in range(rounds):
        R.step()
        torch.cuda.synchronize()
        trajs.append(R.traj_all.cpu().numpy().copy())
        zs.append(R.z.cpu().numpy().copy())
    return np.stack(trajs), np.stack(zs)


def main():
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group(os.environ.get("CMPC_DIST_BACKEND", "gloo"), rank=rank, world_size=world)
    try:
        if sys.argv[1] == "lpv_halt":   # dist_rounds.py lpv_halt OUT.npz REPS ROUNDS
            out, reps, rounds = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
            raised, count, done = run_lpv(reps, rounds, rank, world, offtrack=True)
            np.savez(out, raised=raised, count=count, done=done)
            return
        if sys.argv[1] == "lpv":   # dist_rounds.py lpv OUT.npz REPS ROUNDS
            out, reps, rounds = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
            trajs, zs = run_lpv(reps, rounds, rank, world)
            np.savez(out, trajs=trajs, zs=zs)
            return
        out, n, N, rounds, sample = sys.argv[1], *map(int, sys.argv[2:6])
        trajs, prob, z0 = run(n, N, rounds, sample, rank, world)
        arrays = {f"p_{k}": np.asarray(v) for k, v in prob.items()}
        np.savez(out, trajs=trajs, z0=z0, **arrays)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
