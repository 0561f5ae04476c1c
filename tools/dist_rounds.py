"""Worker of the multi-rank GPU rounds test (tests/test_dist_gpu.py): one rank of the
device-resident consensus rounds (cmpc.rounds.DIRounds — HIP build / solve / advance) with the
per-round exchange over torch.distributed.  Reads RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
and the backend from the environment (CMPC_DIST_BACKEND, default gloo: on a one-GPU box every
rank shares device 0, and RCCL refuses two ranks on one device).

Usage: python tools/dist_rounds.py OUT.npz N_AGENTS HORIZON ROUNDS SAMPLE"""
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
        R.build()
        if r == 0:
            snap = R.snapshot()
        R.solve()
        if r == 0:
            z0 = R.z[:sample].cpu().numpy().copy()
            st = R.status.cpu().numpy()
            assert np.isin(st, (1, 2)).all(), np.unique(st, return_counts=True)
        R.advance()
        R.exchange()
        torch.cuda.synchronize()
        trajs.append(R.traj_all.cpu().numpy().copy())
    prob = {k: (v[:sample] if isinstance(v, np.ndarray) and k in ("A", "B", "x0", "u_prev", "qlin", "C", "h")
                else v) for k, v in snap.items()}
    return np.stack(trajs), prob, z0


def main():
    import torch
    import torch.distributed as dist

    out, n, N, rounds, sample = sys.argv[1], *map(int, sys.argv[2:6])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group(os.environ.get("CMPC_DIST_BACKEND", "gloo"), rank=rank, world_size=world)
    try:
        trajs, prob, z0 = run(n, N, rounds, sample, rank, world)
        arrays = {f"p_{k}": np.asarray(v) for k, v in prob.items()}
        np.savez(out, trajs=trajs, z0=z0, **arrays)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
