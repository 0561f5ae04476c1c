"""cfg4 on the HIP path: 4096 agents in two ranks of 2048 (BASELINE.json configs[3]'s
sharding, one process per rank), the real device-resident rounds (cmpc.rounds.DIRounds: HIP
build / solve / advance) and the per-round all-gather of predicted positions.  On a one-GPU box
both ranks share device 0 and the exchange runs over gloo with a host staging copy (RCCL
refuses two ranks on one device); the collective's semantics are the same.

Jacobi semantics of planner/scripts/LPV_HP_N_main.py:96-117: every rank must end every round
holding exactly the node-global trajectories of a single-process run (bit-equal), and the
solved agent-QPs must match the C restatement (oracle/cmpc_oracle.c)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_AGENTS, HORIZON, ROUNDS, SAMPLE = 4096, 30, 3, 256


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_hip_rounds_match_single_process(tmp_path, gpu_ctx):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from dist_rounds import run
    from oracle import cmpc_oracle as CO

    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CMPC_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "dist_rounds.py"),
                                       str(tmp_path / f"rank{r}.npz"), str(N_AGENTS), str(HORIZON), str(ROUNDS),
                                       str(SAMPLE)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    ref, prob, z0 = run(N_AGENTS, HORIZON, ROUNDS, SAMPLE)   # single process, while the ranks run
    for p in procs:
        out, _ = p.communicate(timeout=240)
        assert p.returncode == 0, out.decode()[-3000:]
    for r in range(2):
        d = np.load(tmp_path / f"rank{r}.npz")
        assert d["trajs"].shape == ref.shape
        assert np.array_equal(d["trajs"], ref), f"rank {r}: rounds differ from the single-process run"
        # a sample of this rank's round-0 agent-QPs against the C restatement
        P = {k[2:]: d[k] for k in d.files if k.startswith("p_")}
        for k in ("nx", "nu", "N", "ns", "mc"):
            P[k] = int(P[k])
        zc, _, _, stc = CO.solve_batch(P, nthreads=8)
        assert np.isin(stc, (1, 2)).all()
        assert np.abs(d["z0"] - zc).max() < 1e-6
    # the single-process sample is rank 0's first agents: same problems, same solution bits
    d0 = np.load(tmp_path / "rank0.npz")
    assert np.array_equal(d0["z0"], z0)


def test_two_rank_lpv_rounds_match_single_process(tmp_path, gpu_ctx):
    """The reference's agent model in device-resident rounds (cmpc.rounds.LPVRounds) on two
    ranks: 12 copies of the 3-agent N = 30 Highway run, ring neighbours that cross the rank
    boundary; four rounds of traj_all and every agent's z bit-equal to one process."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from dist_rounds import run_lpv

    reps, rounds = 12, 4
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CMPC_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "dist_rounds.py"), "lpv",
                                       str(tmp_path / f"lpv{r}.npz"), str(reps), str(rounds)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    trajs, zs = run_lpv(reps, rounds)
    for p in procs:
        out, _ = p.communicate(timeout=240)
        assert p.returncode == 0, out.decode()[-3000:]
    half = 3 * reps // 2
    for r in range(2):
        d = np.load(tmp_path / f"lpv{r}.npz")
        assert np.array_equal(d["trajs"], trajs), f"rank {r}: exchanged trajectories differ"
        assert np.array_equal(d["zs"], zs[:, r * half:(r + 1) * half]), f"rank {r}: solutions differ"


def test_two_rank_lpv_rounds_halt_together(tmp_path, gpu_ctx):
    """An infeasible agent on rank 0 only: the reference quits the whole loop in that round
    (LPV_HP_N_main.py:102-111), so BOTH ranks must raise InfeasibleRound in round 0 with the
    node's count (1) — a rank halting alone would leave the other waiting in the next round's
    all-gather (the processes would hang until the timeout)."""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CMPC_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "dist_rounds.py"), "lpv_halt",
                                       str(tmp_path / f"halt{r}.npz"), "4", "3"], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out, _ = p.communicate(timeout=240)
        assert p.returncode == 0, out.decode()[-3000:]
    for r in range(2):
        d = np.load(tmp_path / f"halt{r}.npz")
        assert bool(d["raised"]) and int(d["count"]) == 1 and int(d["done"]) == 0, (r, dict(d))


def test_c_abi_rccl_allgather_single_rank(gpu_ctx):
    """cmpc_comm_init / cmpc_allgather_trajectories (the C-ABI exchange a MATLAB / C host uses
    instead of torch.distributed), one rank: the gather is the identity, and rounds driven
    through it equal the default rounds bit for bit."""
    import torch

    import cmpc
    from cmpc import scenarios as S
    from cmpc.comm import Comm
    from cmpc.rounds import DIRounds

    comm = Comm(gpu_ctx, 1, 0, Comm.new_id())
    try:
        loc = torch.randn(64, 31, 2, dtype=torch.float64, device="cuda")
        out = torch.zeros_like(loc)
        comm.allgather(loc, out)
        torch.cuda.synchronize()
        assert torch.equal(out, loc)
        cnt = torch.tensor([3, 0], dtype=torch.int32, device="cuda")
        comm.sum_i32(cnt)   # one rank: the sum over ranks is the rank's own
        torch.cuda.synchronize()
        assert cnt.tolist() == [3, 0]
        with pytest.raises(ValueError):
            comm.allgather(loc, torch.zeros(65, 31, 2, dtype=torch.float64, device="cuda"))
        sc = S.make_di(256, 30, 2, 2)
        a, b = DIRounds(sc, ctx=gpu_ctx), DIRounds(sc, ctx=gpu_ctx, comm=comm)
        for _ in range(2):
            a.step()
            b.step()
        torch.cuda.synchronize()
        assert torch.equal(a.traj_all, b.traj_all) and torch.equal(a.z, b.z)
    finally:
        comm.close()
    with pytest.raises(cmpc.CmpcError):   # left the communicator: the exchange refuses to run
        gpu_ctx.check(gpu_ctx.lib.cmpc_allgather_trajectories(gpu_ctx.h, None, None, 0, None))


def test_bench_two_ranks_on_one_device_emit_one_line():
    """bench.py's multi-rank path launched as the driver launches it (torch.distributed.run,
    --nproc-per-node 2, RANK / WORLD_SIZE / LOCAL_RANK from the launcher) with both ranks on
    device 0 and the exchange over gloo (CMPC_DIST_BACKEND / CMPC_DEVICE; RCCL refuses two ranks on
    one device): rank 0 prints one JSON line whose value covers both ranks' agents."""
    import json

    env = dict(os.environ, CMPC_DIST_BACKEND="gloo", CMPC_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "5", "--warmup", "1", "--no-cpu", "--no-ref"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["agents_total"] == 2048 and out["steps"] == 5
    assert out["value"] > 0 and out["unsolved"] == 0 and out["max_kkt"] < 1e-6
    assert "gloo" in out["config"]["parallelism"]


def test_bench_two_ranks_strong_scaling_cfg4():
    """bench.py --agents-total (strong scaling, BASELINE cfg4's 4096 agents split over the ranks):
    two ranks of 2048 on device 0 (exchange over gloo), one JSON line for the whole population,
    "scaling": "strong", the workload named cfg4."""
    import json

    env = dict(os.environ, CMPC_DIST_BACKEND="gloo", CMPC_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--agents-total", "4096", "--steps", "3", "--warmup", "1", "--no-cpu", "--no-ref"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["scaling"] == "strong" and out["config"]["agents_total"] == 4096
    assert out["config"]["workload"].startswith("cfg4")
    assert out["value"] > 0 and out["unsolved"] == 0 and out["max_kkt"] < 1e-6
