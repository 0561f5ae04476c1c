"""The MEX gateway (colaborativempc-_amd/mex/cmpc_quadprog_mex.c, built against the mock mex.h)
on the GPU, checked against oracles — not against cmpc.quadprog itself:

* sparse arguments as YALMIP passes them (yalmip2quadprog.m:38-70 slices sparse Q / A / Aeq
  out of F_struc) on the MATLAB variant's 5-state LPV-MPC models (LPV_MPC_fnc_dt_Vnew.m,
  oracle/matlab_ref.py) against their KKT-certified optima (tests/golden/matlab_lpv_mpc.npz):
  the planner script's first four control steps scheduled from NL_vars.mat and four hand-built;
* the struct form (cmpc_solve_mpc_batch through MATLAB plumbing) on BASELINE cfg2 — 64 agents,
  N = 20, nb = 2 — against the C restatement oracle/cmpc_oracle.c."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import mex_harness as MX

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "matlab_lpv_mpc.npz")


def _flat_directions(mod, curv=1e-5):
    """Orthonormal basis of the directions in which the objective is (nearly) flat on the
    equality manifold.  The reference's weights make the optimum a face, not a point: the last
    accelerations are unweighted (no terminal vx cost, LPV_MPC_fnc_dt_Vnew.m:121 — curvature
    ~1e-16), and QQ's 8.8e-14 on vx and -2.1e-10 on ey (:45) leave ~8 more directions of
    curvature 1e-7..1e-6 (of a spectrum reaching 400), along which any solver's z is fixed only
    to sqrt(objective tolerance / curvature).  Those are excluded from the 1e-6 z comparison;
    the objective value and feasibility are compared in full."""
    Aeq = mod["Aeq"]
    Z = np.linalg.svd(Aeq)[2][Aeq.shape[0]:].T
    ev, V = np.linalg.eigh(Z.T @ mod["H"] @ Z)
    return Z @ V[:, ev < curv]


@pytest.mark.parametrize("case", range(8))
def test_mex_sparse_yalmip_model_matches_certified_optimum(gpu_ctx, case):
    d = np.load(GOLD, allow_pickle=False)
    mod = {k: d[f"m{case}_{k}"] for k in ("H", "f", "A", "b", "Aeq", "beq", "lb", "ub")}
    zs = d[f"z{case}"]
    ps = [MX.mx_sparse(sp.csc_matrix(mod["H"])), MX.mx(mod["f"]), MX.mx_sparse(sp.csc_matrix(mod["A"])),
          MX.mx(mod["b"]), MX.mx_sparse(sp.csc_matrix(mod["Aeq"])), MX.mx(mod["beq"]), MX.mx(mod["lb"]),
          MX.mx(mod["ub"])]
    out, err = MX.call_raw(ps, 3)
    assert err is None, err
    x, fval, flag = MX.values(out[0]), MX.values(out[1])[0], MX.values(out[2])[0]
    assert flag == 1
    f = lambda z: 0.5 * z @ mod["H"] @ z + mod["f"] @ z   # noqa: E731
    assert abs(fval - f(x)) < 1e-9 * max(1.0, abs(fval))
    assert f(x) - f(zs) < 1e-9 * max(1.0, abs(f(zs)))
    assert np.abs(mod["Aeq"] @ x - mod["beq"]).max() < 1e-8
    assert (mod["A"] @ x - mod["b"]).max() < 1e-8
    assert (x - mod["lb"]).min() > -1e-8 and (mod["ub"] - x).min() > -1e-8
    dz = x - zs
    Nf = _flat_directions(mod)
    dz = dz - Nf @ (Nf.T @ dz)
    # off the flat directions: 1e-6, or — where a bound is weakly active (multiplier ~ 0, the
    # degenerate case in which interior-point iterates approach it only like sqrt(mu), as
    # conftest.assert_matches_optimum allows for the LPV QPs) — a KKT residual <= 1e-6 of x itself
    # in quadprog's form (H, f; A x <= b, Aeq x = beq, lb <= x <= ub), with the value checks above
    err = float(np.abs(dz).max())
    if err >= 1e-6:
        from conftest import KKT_TOL, reference_kkt

        n = x.size
        Aall = np.vstack([mod["A"], mod["Aeq"], np.eye(n)])
        lo = np.concatenate([np.full(mod["A"].shape[0], -np.inf), mod["beq"], mod["lb"]])
        hi = np.concatenate([mod["b"], mod["beq"], mod["ub"]])
        kkt, cert = reference_kkt(mod["H"], mod["f"], Aall, lo, hi, x)
        assert kkt <= KKT_TOL, (err, cert, Nf.shape[1])


def test_mex_sparse_matches_dense(gpu_ctx):
    """The same model passed full and sparse gives the same bits."""
    d = np.load(GOLD, allow_pickle=False)
    mod = {k: d[f"m0_{k}"] for k in ("H", "f", "A", "b", "Aeq", "beq", "lb", "ub")}
    dense, e1 = MX.call([mod[k] for k in ("H", "f", "A", "b", "Aeq", "beq", "lb", "ub")], nlhs=1)
    ps = [MX.mx_sparse(mod["H"]), MX.mx(mod["f"]), MX.mx_sparse(mod["A"]), MX.mx(mod["b"]),
          MX.mx_sparse(mod["Aeq"]), MX.mx(mod["beq"]), MX.mx(mod["lb"]), MX.mx(mod["ub"])]
    sparse, e2 = MX.call_raw(ps, 1)
    assert e1 is None and e2 is None
    assert np.array_equal(MX.values(dense[0]), MX.values(sparse[0]))


def _matlab_struct(P):
    """Structured batch (oracle/synth layout, row-major batch-major) -> the gateway's struct form
    (MATLAB order: A(i,j,k,b) = A_k(i,j) of agent b)."""
    f = {k: np.array([float(P[k])]) for k in ("nx", "nu", "N", "ns")}
    f.update(Q=P["Q"], R=P["R"], dR=P["dR"], Qs=P["Qs"], u_lb=P["u_lb"], u_ub=P["u_ub"],
             row_slack=np.asarray(P["row_slack"], float), row_sign=np.asarray(P["row_sign"], float),
             A=P["A"].transpose(2, 3, 1, 0), B=P["B"].transpose(2, 3, 1, 0), x0=P["x0"].T, u_prev=P["u_prev"].T,
             qlin=P["qlin"].transpose(2, 1, 0), C=P["C"].transpose(2, 3, 1, 0), h=P["h"].transpose(2, 1, 0))
    return f


def test_mex_struct_form_cfg2_batch_matches_c_oracle(gpu_ctx):
    from cmpc import scenarios as S
    from oracle import cmpc_oracle as CO
    from oracle import synth

    sc = S.make_di(64, 20, 2, 2)   # BASELINE cfg2: 64 agents, N = 20
    P = synth.structured(sc.shared, sc.params, sc.A, sc.B, sc.x0, sc.u_prev, sc.lane, sc.nbr, sc.traj,
                         np.arange(64))
    out, err = MX.call_raw([MX.mx_struct(_matlab_struct(P))], 4)
    assert err is None, err
    nz = CO.nz_of(P)
    z = MX.values(out[0]).reshape(64, nz)   # nz x B column-major = agent-major rows
    status = MX.values(out[3])
    zc, _, _, stc = CO.solve_batch(P, nthreads=8)
    assert (status == 1).all() and (stc == 1).all()
    assert np.abs(z - zc).max() < 1e-6
    assert MX.values(out[1]).max() < 1e-6   # kkt


def test_mex_struct_form_rejects_bad_fields(gpu_ctx):
    out, err = MX.call_raw([MX.mx_struct({"nx": np.array([4.0])})], 1)
    assert out is None and err[0] == "cmpc:quadprog:args"


def _lpv_matlab(name):
    """A captured reference run's step-0 inputs in cmpc_lpv's MATLAB order (agents last)."""
    from conftest import golden
    from test_mex import lpv_params

    from oracle import lpv_ref as L

    d = golden(name)
    N, n = int(d["N"]), int(d["n_agents"])
    sel = sorted([j for j in range(len(d["step"])) if d["step"][j] == 0], key=lambda j: d["agent"][j])
    x0, xl = d["x0"][sel], np.stack([d[f"x_last_{j}"] for j in sel])
    ul, uo, pose = np.stack([d[f"u_last_{j}"] for j in sel]), d["u_old"][sel], d["pose"][sel]
    nbr = np.array(L.neighbour_lists(n), np.int32).reshape(n, n - 1)
    xa = np.stack([np.swapaxes(pose[nbr[i]], 0, 1) for i in range(n)])        # (B, N+1, nb, 2)
    P = lpv_params(N)
    P["vx_ref"] = np.array([float(d["vx_ref"])])
    D = dict(x0=x0.T, x_last=xl.transpose(2, 1, 0), u_last=ul.transpose(2, 1, 0), u_old=uo.T,
             pose=pose.transpose(2, 1, 0), x_agents=xa.transpose(3, 2, 1, 0))
    host = dict(x0=x0, x_last=xl, u_last=ul, u_old=uo, pose=pose, nbr=nbr, x_agents=xa, N=N, n=n, vx_ref=float(d["vx_ref"]))
    return P, D, host


def test_mex_lpv_solve_matches_planner_batch(gpu_ctx):
    """cmpc_lpv('solve', P, D) = PlannerLPVBatch.solve on the same captured step (bit-equal)."""
    import cmpc
    from oracle import lpv_ref as L

    P, D, h = _lpv_matlab("lpv_n30_a3")
    out, err = MX.call_lpv([MX.mx_str("solve"), MX.mx_struct(P), MX.mx_struct(D)], 5)
    assert err is None, err
    g = L.paper_gains()
    bp = cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], h["N"], 0.025, L.Track.build("Highway"), g["wq"],
                              L.SCALED_CAR_MODEL, L.scaled_car_limits(h["vx_ref"]), ctx=gpu_ctx)
    res = bp.solve(h["x0"], h["x_last"], h["u_last"], h["u_old"], h["x_agents"], h["pose"])
    nz = 12 * (h["N"] + 1) + 4 * h["N"]
    assert np.array_equal(MX.values(out[0]).reshape(h["n"], nz), res["z"])
    assert np.array_equal(MX.values(out[1]), res["status"])
    assert np.array_equal(MX.values(out[4]).reshape(res["planes"].shape), res["planes"])


@pytest.mark.parametrize("name", ["lpv_n30_a3", "lpv_n20_a4"])
def test_mex_lpv_rounds_handle_bit_equal_to_lpvrounds(gpu_ctx, name):
    """A MATLAB host's consensus loop through the gateway's round handle (rounds_create, five
    rounds_step / rounds_read, rounds_destroy) is bit-equal to LPVRounds every round."""
    import torch

    import cmpc
    from cmpc.rounds import LPVRounds
    from oracle import lpv_ref as L

    P, D, h = _lpv_matlab(name)
    S = dict(nbr=h["nbr"].T.astype(float), traj=h["pose"].transpose(2, 1, 0))
    out, err = MX.call_lpv([MX.mx_str("rounds_create"), MX.mx_struct(P), MX.mx_struct(D), MX.mx_struct(S)], 1)
    assert err is None, err
    hd = MX.values(out[0])
    g = L.paper_gains()
    bp = cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], h["N"], 0.025, L.Track.build("Highway"), g["wq"],
                              L.SCALED_CAR_MODEL, L.scaled_car_limits(h["vx_ref"]), ctx=gpu_ctx)
    R = LPVRounds(bp, h["x0"], h["x_last"], h["u_last"], h["nbr"], u_old=h["u_old"], traj=h["pose"])
    nz = 12 * (h["N"] + 1) + 4 * h["N"]
    for rnd in range(5):
        R.step()
        torch.cuda.synchronize()
        o, err = MX.call_lpv([MX.mx_str("rounds_step"), MX.mx(hd), MX.mx(np.array([1.0]))], 2)
        assert err is None and MX.values(o[0])[0] == 1 and MX.values(o[1])[0] == 0, err
        o, err = MX.call_lpv([MX.mx_str("rounds_read"), MX.mx(hd)], 5)
        assert err is None, err
        assert np.array_equal(MX.values(o[0]).reshape(h["n"], nz), R.z.cpu().numpy()), rnd
        assert np.array_equal(MX.values(o[1]), R.status.cpu().numpy())
        assert np.array_equal(MX.values(o[4]).reshape(h["n"], 9), R.x0.cpu().numpy())
    o, err = MX.call_lpv([MX.mx_str("rounds_get_traj"), MX.mx(hd)], 1)
    assert err is None and np.array_equal(MX.values(o[0]).reshape(h["n"], h["N"] + 1, 2), R.traj_local.cpu().numpy())
    _, err = MX.call_lpv([MX.mx_str("rounds_destroy"), MX.mx(hd)], 0)
    assert err is None
    _, err = MX.call_lpv([MX.mx_str("rounds_read"), MX.mx(hd)], 1)
    assert err[0] == "cmpc:lpv:args"
