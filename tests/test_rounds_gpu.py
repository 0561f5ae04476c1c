"""Consensus rounds of the reference's agent model (LPV_HP_N_main.py:96-117) through the C ABI's
round handle (cmpc_lpv_rounds_*, what a MATLAB / C host drives) and the failure semantics of the
loop (LPV_Planner.py:243-249: status outside {1, 2, -2} is infeasible; the reference quits there,
LPV_HP_N_main.py:102-111), on the GPU."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

CASES = ["lpv_n30_a3", "lpv_n10_a1", "lpv_n10_a2", "lpv_n20_a4", "lpv_n10_lowspeed"]


def _case(name, ctx):
    import cmpc
    from oracle import lpv_ref as L

    d = golden(name)
    N, n, dt = int(d["N"]), int(d["n_agents"]), float(d["dt"])
    g = L.paper_gains()
    bp = cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], N, dt, L.Track.build("Highway"), g["wq"],
                              L.SCALED_CAR_MODEL, L.scaled_car_limits(float(d["vx_ref"])), ctx=ctx)
    sel = sorted([j for j in range(len(d["step"])) if d["step"][j] == 0], key=lambda j: d["agent"][j])
    args = (d["x0"][sel].copy(), np.stack([d[f"x_last_{j}"] for j in sel]), np.stack([d[f"u_last_{j}"] for j in sel]),
            np.array(L.neighbour_lists(n), np.int32).reshape(n, n - 1))
    kw = dict(u_old=d["u_old"][sel].copy(), traj=d["pose"][sel].copy())
    return bp, args, kw, int(d["steps"])


def _replicated(ctx, reps):
    """`reps` jittered copies of the reference's 3-agent N = 30 scenario (bench.py lpv_population)."""
    import bench

    return bench.lpv_population(ctx, reps)


@pytest.mark.parametrize("name", CASES)
def test_round_handle_bit_equal_to_lpvrounds(gpu_ctx, name):
    """cmpc_lpv_rounds_create / _step / _read drive the captured reference runs (1-4 agents, 0-3
    neighbours, the vx < 0.2 branch) bit-identically to the torch-driven LPVRounds."""
    import torch

    from cmpc.rounds import LPVRounds, LPVRoundsHandle

    bp, args, kw, steps = _case(name, gpu_ctx)
    R = LPVRounds(bp, *args, **kw)
    H = LPVRoundsHandle(bp, *args, **kw)
    for step in range(steps):
        R.step()
        torch.cuda.synchronize()
        done, bad = H.step(1)
        assert (done, bad) == (1, 0)
        r = H.read()
        assert np.array_equal(r["z"], R.z.cpu().numpy()), step
        assert np.array_equal(r["status"], R.status.cpu().numpy())
        assert np.array_equal(r["x0"], R.x0.cpu().numpy())
        if R.nb:
            assert np.array_equal(r["planes"], R.planes.cpu().numpy())
        assert np.array_equal(H.get_traj(), R.traj_local.cpu().numpy())
    H.close()


def test_round_handle_multi_round_call_and_host_exchange_shards(gpu_ctx):
    """Five rounds of 8 jittered copies (24 agents) in one cmpc_lpv_rounds_step call equal five
    single-round calls; and the same population sharded over two handles (ranks 0 / 1 of 12 agents,
    CMPC_ROUNDS_HOST_EXCHANGE: the host gathers the positions between steps, as an MPI host
    would) is bit-equal to the one-shard run every round."""
    from cmpc.rounds import LPVRoundsHandle

    bp, args, kw = _replicated(gpu_ctx, 8)
    one = LPVRoundsHandle(bp, *args, **kw)
    assert one.step(5) == (5, 0)
    z5 = one.read()["z"]
    ref = LPVRoundsHandle(bp, *args, **kw)
    shards = [LPVRoundsHandle(bp, *args, **kw, rank=r, world=2, host_exchange=True) for r in range(2)]
    for rnd in range(5):
        assert ref.step(1) == (1, 0)
        for h in shards:
            assert h.step(1) == (1, 0)
        gathered = np.concatenate([h.get_traj() for h in shards])
        for h in shards:
            h.set_traj(gathered)
        zr = ref.read()["z"]
        assert np.array_equal(np.concatenate([h.read()["z"] for h in shards]), zr), rnd
    assert np.array_equal(z5, zr)
    with pytest.raises(Exception):
        shards[0].step(2)   # host exchange: one round per step
    for h in [one, ref] + shards:
        h.close()


def _offtrack(ctx):
    """lpv_n10_a2 at step 0 with agent 0's previous prediction off the track (s = NaN in one row:
    no segment holds it, the reference raises in curvature / get_ey, misc.py:97)."""
    bp, args, kw, _ = _case("lpv_n10_a2", ctx)
    x_last = args[1].copy()
    x_last[0, 3, 6] = np.nan
    return bp, (args[0], x_last, args[2], args[3]), kw


def test_infeasible_agent_halts_the_loop_and_is_not_propagated(gpu_ctx):
    """An infeasible agent (status -10) stops LPVRounds.step like the reference's QUIT
    (InfeasibleRound); without the halt the loop goes on, the agent keeps its state and previous
    trajectory and no NaN reaches its neighbour, which stays solved."""
    import torch

    import cmpc
    from cmpc.rounds import InfeasibleRound, LPVRounds

    bp, args, kw = _offtrack(gpu_ctx)
    R = LPVRounds(bp, *args, **kw)
    with pytest.raises(InfeasibleRound) as ei:
        R.step()
    assert ei.value.count == 1
    R = LPVRounds(bp, *args, **kw)
    traj0 = R.traj_all.cpu().numpy().copy()
    N = R.N
    for _ in range(2):
        R.step(halt=False)
        torch.cuda.synchronize()
        # the infeasible agent keeps its previous prediction in its dense N-row slot (rows 0..N-1)
        xl = R.x_last.cpu().numpy().reshape(-1)[: R.B * N * 9].reshape(R.B, N, 9)
        assert np.array_equal(xl[0], args[1][0, :N], equal_nan=True)
        st = R.status.cpu().numpy()
        assert st[0] == cmpc.CMPC_UNSOLVED and st[1] == cmpc.CMPC_SOLVED
        assert R.infeasible() == 1
        assert np.isfinite(R.traj_all.cpu().numpy()).all()
        assert np.array_equal(R.traj_all.cpu().numpy()[0], traj0[0])
        assert np.array_equal(R.x0.cpu().numpy()[0], args[0][0])
        assert np.isfinite(R.z.cpu().numpy()[1]).all()


def test_round_handle_halts_at_an_infeasible_agent(gpu_ctx):
    from cmpc.rounds import LPVRoundsHandle

    bp, args, kw = _offtrack(gpu_ctx)
    H = LPVRoundsHandle(bp, *args, **kw)
    assert H.step(3) == (1, 1)      # stopped after the first round, one infeasible agent
    H.close()
    H = LPVRoundsHandle(bp, *args, **kw, halt=False)
    assert H.step(3) == (3, 1)      # CMPC_ROUNDS_NO_HALT: all rounds run
    assert np.isfinite(H.get_traj()).all()
    H.close()


def test_lpvrounds_rejects_short_initial_prediction(gpu_ctx):
    """x_last must be (n, N+1, 9): the gather and builder kernels index it by the population."""
    from cmpc.rounds import LPVRounds

    bp, args, kw, _ = _case("lpv_n30_a3", gpu_ctx)
    with pytest.raises(ValueError):
        LPVRounds(bp, args[0], args[1][:2], args[2], args[3], **kw)
    with pytest.raises(ValueError):
        LPVRounds(bp, args[0], args[1][:, :-1], args[2], args[3], **kw)


def test_lpv_rounds_at_scale_against_c_restatement(gpu_ctx):
    """The bench's population of the reference's agent model (1023 agents: 341 jittered copies of
    the 3-agent N = 30 Highway scenario), 20 device-resident rounds with the rescue policy: no agent
    unsolved, every agent's KKT residual <= 1e-6, and each round a 128-agent sample re-solved by the
    C restatement with the same rescue policy (oracle.cmpc_oracle.solve_batch_rescue) within 1e-6
    wherever both reach the tolerance."""
    import bench

    out = bench.lpv_rounds(gpu_ctx, replicas=341, rounds=20, warmup=2, check=True, sample=128)
    st = out["status_counts"]
    print({k: v for k, v in out.items() if k in ("agent_qp_per_s", "status_counts", "max_kkt", "oracle_sample")})
    assert out["polish"]   # PlannerLPVBatch's default, as the reference's OSQP polish=True
    assert all(k in (1, 2) for k in st), st
    # the rounding floor (status 2) after the polish: <= 0.5 % of the solves (3.5 % without it)
    assert st.get(2, 0) <= 0.005 * sum(st.values()), st
    assert out["max_kkt"] <= 1e-6
    smp = out["oracle_sample"]
    assert smp["checked"] == 20 * 128, smp
    assert smp["both_solved"] >= 0.99 * smp["checked"], smp
    assert smp["max_abs_err_vs_cpu_non_degenerate"] <= 1e-6, smp
    # both solved but farther apart than 1e-6: an interior-point endpoint against a polished one on a
    # degenerate optimum; the GPU point certifies itself (reference-form KKT, objective not above the
    # C restatement's), and such agents stay rare (<= 0.5 % of the sample; max_abs_err_vs_cpu, over every
    # both-solved agent, includes them)
    dg = smp["degenerate"]
    assert dg["count"] <= 0.005 * smp["checked"], dg
    if dg["count"]:
        assert dg["max_ref_kkt_gpu"] <= 1e-6 and dg["max_obj_gap_rel"] <= 1e-10, dg
