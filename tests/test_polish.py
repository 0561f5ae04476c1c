"""Active-set polish (CMPC_FLAG_POLISH; OSQP's polish=True, LPV_Planner.py:233) on agent-QPs of the
reference's agent model whose condensed factorisation breaks down at the rounding floor
(tests/golden/polish_lpv.npz, made by oracle/gen_polish_fixture.py from bench.py's lpv_rounds
population in the CPU lab)."""
import numpy as np
import pytest

from conftest import golden, polish_amax


def _problems():
    d = golden("polish_lpv")
    P = {k: d[k] for k in d.files if not k.startswith("status_")}
    for k in ("nx", "nu", "N", "ns", "mc"):
        P[k] = int(P[k])
    return P, d["status_plain"], d["status_polish"]


def test_oracle_polish_finishes_floor_breakdowns():
    """The C restatement: without the polish the breakdown agents stop at the rounding floor
    (status 2); with it every agent is solved (merit < tol), the agents that converged are
    untouched (bit-identical), and the polished optimum agrees with the rounding-floor iterate to
    its accuracy and with the Riccati double-double method's solution (newton 3) where that one
    converges."""
    from oracle import cmpc_oracle as CO

    P, st_plain, st_pol = _problems()
    z0, k0, i0, s0 = CO.solve_batch_rescue(P, nthreads=4)
    z1, k1, i1, s1 = CO.solve_batch_rescue(P, nthreads=4, polish=True, polish_amax=polish_amax(P))
    assert np.array_equal(s0, st_plain) and np.array_equal(s1, st_pol)
    assert (s1 == 1).all() and (k1 < 1e-9).all(), k1
    # the agents that converged are untouched, except a degenerate endpoint (a weakly active row,
    # kPolishDegenerate) that the polish improves: then within the endpoint's accuracy and a lower KKT
    same = s0 == 1
    moved = same & np.any(z0 != z1, axis=1)
    assert np.abs(z1[same] - z0[same]).max() < 1e-6
    assert (k1[moved] <= k0[moved]).all(), (k0[moved], k1[moved])
    assert np.abs(z1 - z0).max() < 1e-4
    z3, k3, i3, s3 = CO.solve_batch(P, nthreads=4, newton=3)
    ok = s3 == 1
    assert ok.any()
    assert np.abs(z1[ok] - z3[ok]).max() < 1e-6, np.abs(z1[ok] - z3[ok]).max()


def test_polish_active_set_capacity_is_shared():
    """One active-set capacity on both sides: the kernel's layout reports it
    (cmpc_plan_info.polish_max_active: kPolishMaxActive = 96, lowered in steps of 8 until the LDS image
    fits 160 KB), the C restatement takes it as an argument.  Shapes whose image does not fit at 96 report
    less; with a capacity below the floor agents' active sets the restatement keeps their unpolished
    results (status 2 where the plain policy stops at the floor), as the kernel does."""
    from cmpc import scenarios as S
    from oracle import cmpc_oracle as CO

    P, st_plain, _ = _problems()
    cap_lpv = polish_amax(P)  # the reference's agent at N = 30, nb = 2: 88 (the image at 96 exceeds 160 KB)
    assert 8 <= cap_lpv <= 96 and cap_lpv % 8 == 0, cap_lpv
    big = S.di_shared(2, 32, 3)  # a 64-variable horizon with 7 rows per stage: 96 does not fit
    big.update(nx=9, nu=2)
    big["Q"], big["R"], big["dR"] = np.eye(9), np.eye(2), np.eye(2)
    cap = polish_amax(big)
    assert 8 <= cap < cap_lpv and cap % 8 == 0, cap
    z0, k0, i0, s0 = CO.solve_batch_rescue(P, nthreads=4)
    z8, k8, i8, s8 = CO.solve_batch_rescue(P, nthreads=4, polish=True, polish_amax=8)
    floor = s0 == 2
    assert floor.sum() >= 4 and np.array_equal(s8, s0) and np.array_equal(z8[floor], z0[floor])
    assert np.abs(z8 - z0).max() < 1e-6  # (a converged agent with a small active set may still be polished)


@pytest.mark.gpu
def test_gpu_polish_matches_c_restatement(gpu_ctx):
    """The HIP polish (mpc_polish.hip) on the same agents: every agent solved (status 1), z within
    1e-6 of the C restatement's polished optimum."""
    import cmpc
    from oracle import cmpc_oracle as CO

    P, _, _ = _problems()
    z, kkt, it, st = cmpc.solve_mpc(P, gpu_ctx, rescue=True, polish=True)
    zp, kp, ip, sp = cmpc.solve_mpc(P, gpu_ctx, rescue=True)
    z1, k1, i1, s1 = CO.solve_batch_rescue(P, nthreads=4, polish=True, polish_amax=polish_amax(P))
    print("GPU without polish", sp.tolist(), "with", st.tolist(), "kkt", kkt.max(),
          "|z - z_cpu|", np.abs(z - z1).max())
    assert (st == cmpc.CMPC_SOLVED).all(), st
    assert (kkt < 1e-9).all(), kkt
    assert np.abs(z - z1).max() < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("n,N,nb,dim,tol", [(64, 20, 2, 2, 1e-13), (64, 10, 2, 3, 1e-15)])
def test_gpu_polish_double_integrator_families(gpu_ctx, n, N, nb, dim, tol):
    """The polish kernel's nx = 4 and nx = 6 instantiations (the BASELINE double-integrator families):
    at a tolerance below the rounding floor (1e-13, 1e-15) the solves stop at the floor, so rescue + polish
    runs on them; statuses and z match the C restatement of the same policy (to 1e-6), and the
    polished solves' KKT residuals are no worse than without the polish."""
    import cmpc
    from cmpc import scenarios as S
    from oracle import cmpc_oracle as CO
    from oracle import synth

    sc = S.make_di(n, N, nb, dim)
    P = synth.structured(sc.shared, sc.params, sc.A, sc.B, sc.x0, sc.u_prev, sc.lane, sc.nbr, sc.traj, np.arange(n))
    z0, k0, i0, s0 = cmpc.solve_mpc(P, gpu_ctx, tol=tol, rescue=True)
    z1, k1, i1, s1 = cmpc.solve_mpc(P, gpu_ctx, tol=tol, rescue=True, polish=True)
    zc, kc, ic, sc_ = CO.solve_batch_rescue(P, tol=tol, nthreads=4, polish=True, polish_amax=polish_amax(P))
    print(f"dim {dim}: status without polish {np.unique(s0, return_counts=True)}, with {np.unique(s1, return_counts=True)}, "
          f"C {np.unique(sc_, return_counts=True)}; kkt {k0.max():.1e} -> {k1.max():.1e}; |z - z_cpu| {np.abs(z1 - zc).max():.1e}")
    assert np.isin(s1, (cmpc.CMPC_SOLVED, cmpc.CMPC_SOLVED_INACCURATE)).all()
    assert np.abs(z1 - zc).max() < 1e-6
    assert k1.max() <= max(k0.max(), 1e-12)
