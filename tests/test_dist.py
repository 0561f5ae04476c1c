"""Multi-rank consensus rounds on CPU (gloo, world size 2): the sharding and the
per-round all-gather of predicted positions used by the one-process-per-GPU path
(cmpc.rounds; the reference's exchange is LPV_HP_N_main.py:117 / the ROS topics of
LPV_ROS_main.py:66-77) reproduce the single-process rounds bit for bit.  The
per-agent solve runs in the oracle here (no GPU); what is under test is the shard
layout and the collective, which are the product's."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cmpc import scenarios as S
from cmpc.rounds import exchange_positions
from oracle import cmpc_oracle as CO
from oracle import synth

N_AG, N, NB, ROUNDS = 24, 10, 2, 3


def _advance(z, nx, nu, ns):
    """Round update of LPV_HP_N_main.py:106-117 (what cmpc_di_advance_dev does)."""
    ne = nx + ns
    x0 = z[:, ne:ne + nx].copy()
    up = z[:, ne * (N + 1):ne * (N + 1) + nu].copy()
    traj = np.stack([z[:, [k * ne for k in range(N + 1)]], z[:, [k * ne + 1 for k in range(N + 1)]]], -1)
    return x0, up, traj


def _rounds(rank, world, group=None):
    sc = S.make_di(N_AG, N, NB, 2)
    sl = sc.shard(rank, world)
    sh = sc.shared
    x0, up = sc.x0[sl].copy(), sc.u_prev[sl].copy()
    traj_all = torch.tensor(sc.traj)
    out = []
    for _ in range(ROUNDS):
        P = synth.structured(sh, sc.params, sc.A[sl], sc.B[sl], x0, up, sc.lane[sl], sc.nbr[sl],
                             traj_all.numpy(), np.arange(sl.start, sl.stop))
        z, _, _, st = CO.solve_batch(P, nthreads=1)
        assert (st == 1).all()
        x0, up, traj_local = _advance(z, sh["nx"], sh["nu"], sh["ns"])
        exchange_positions(traj_all, torch.tensor(traj_local), world, group)
        out.append(traj_all.numpy().copy())
    return np.stack(out)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _rounds(rank, world)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shards_partition_the_population():
    sc = S.make_di(N_AG, N, NB, 2)
    for world in (1, 2, 3, 4, 8):
        idx = np.concatenate([np.arange(N_AG)[sc.shard(r, world)] for r in range(world)])
        assert np.array_equal(idx, np.arange(N_AG))


def test_two_rank_rounds_match_single_process():
    ref = _rounds(0, 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank ends each round holding the same node-global trajectories as one process
    for r in range(2):
        assert np.array_equal(got[r], ref)


def test_exchange_rejects_mismatched_buffers():
    with pytest.raises(ValueError):
        exchange_positions(torch.zeros(5, N + 1, 2, dtype=torch.float64),
                           torch.zeros(2, N + 1, 2, dtype=torch.float64), world=2)
