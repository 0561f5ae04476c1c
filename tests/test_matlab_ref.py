"""The MATLAB per-agent QP path restated (oracle/matlab_ref.py): YALMIP's quadprog model
transformation (yalmip2quadprog.m) on hand-built known answers, and the 5-state LPV-MPC models
of LPV_MPC_fnc_dt_Vnew.m regenerated bit for bit against the committed, KKT-certified
fixtures (tests/golden/matlab_lpv_mpc.npz, oracle/gen_matlab_fixtures.py), including the planner
script's first control steps scheduled from the reference's NL_vars.mat
(PLAN_NL_LPV_MPC_dt_WORKS_Oval.m:127-200).  MATLAB is absent: parity with quadprog's own output
is unpinned (oracle/matlab_ref.py header)."""
import os

import numpy as np

from oracle import matlab_ref as M

GOLD = os.path.join(os.path.dirname(__file__), "golden", "matlab_lpv_mpc.npz")


def test_yalmip2quadprog_known_answer():
    # x in R^3: one equality 1 + x0 - x2 == 0, one inequality 4 - x0 - x1 >= 0, x1 fixed by lb == ub
    F = np.array([[1.0, 1.0, 0.0, -1.0], [4.0, -1.0, -1.0, 0.0]])
    c = np.array([1.0, 2.0, 3.0])
    Q = np.diag([1.0, 0.0, 2.0])
    lb = np.array([-np.inf, 0.5, 0.0])
    ub = np.array([np.inf, 0.5, 1.0])
    m = M.yalmip2quadprog(F, 1, c, Q, lb, ub)
    # the fixed bound became the FIRST equality row (x1 == 0.5) and the bounds widened by 1 (:27-36)
    np.testing.assert_array_equal(m["Aeq"], [[0.0, -1.0, 0.0], [-1.0, 0.0, 1.0]])
    np.testing.assert_array_equal(m["beq"], [-0.5, 1.0])
    np.testing.assert_array_equal(m["A"], [[1.0, 1.0, -0.0]])
    np.testing.assert_array_equal(m["b"], [4.0])
    np.testing.assert_array_equal(m["lb"], [-np.inf, -0.5, 0.0])
    np.testing.assert_array_equal(m["ub"], [np.inf, 1.5, 1.0])
    np.testing.assert_array_equal(m["H"], 2.0 * Q)      # :61 Q <- 2Q
    # no equalities at all
    m = M.yalmip2quadprog(np.array([[4.0, -1.0, -1.0, 0.0]]), 0, c, Q, -np.ones(3), np.ones(3))
    assert m["Aeq"].shape == (0, 3) and m["A"].shape == (1, 3)


def test_lpv_mpc_models_regenerate_and_are_certified():
    d = np.load(GOLD, allow_pickle=False)
    Hp, dt = int(d["Hp"]), float(d["dt"])
    for j in range(int(d["ncases"])):
        p = {k.split("_", 1)[1]: d[k] for k in d.files if k.startswith(f"p{j}_")}
        F, Kf, c, Q, lb, ub = M.lpv_mpc_interface(Hp, dt, p, float(d[f"max_vel_{j}"]))
        mod = M.yalmip2quadprog(F, Kf, c, Q, lb, ub)
        for k in ("H", "f", "A", "b", "Aeq", "beq", "lb", "ub"):
            np.testing.assert_array_equal(mod[k], d[f"m{j}_{k}"], err_msg=f"case {j} {k}")
        # sizes of the model (121 variables, 75 equalities for Hp = 15)
        assert mod["H"].shape == (121, 121) and mod["Aeq"].shape == (75, 121)
        assert d[f"kkt{j}"].max() < 1e-9
        # the stored optimum is primal feasible in the quadprog form
        z = d[f"z{j}"]
        assert np.abs(mod["Aeq"] @ z - mod["beq"]).max() < 1e-9
        assert (mod["A"] @ z - mod["b"]).max() < 1e-9
        assert (z - mod["lb"]).min() > -1e-9 and (mod["ub"] - z).min() > -1e-9


def test_oval_curvature_lookup():
    seg = M.oval_segments(1)
    # MapMod.m "oval" lane 1: straight 2, arc 9 of radius 9/pi, straight 4, arc, straight 2
    np.testing.assert_allclose(seg[0], [0.0, 2.0, 11.0, 15.0, 24.0])
    assert M.curvature(1.0, seg) == 0.0 and M.curvature(2.0, seg) == np.pi / 9   # both ends inclusive, last wins
    assert M.curvature(26.0 + 3.0, seg) == np.pi / 9                             # wraps by the track length 26
    assert M.curvature(24.5, seg) == 0.0


def test_planner_steps_from_nl_vars_regenerate():
    """Step 1 re-derived from the stored NL_vars.mat arrays (:127-167, limits swapped at :237-238),
    steps 2..4 from the stored optimum of the step before (:171-199, :259-260)."""
    d = np.load(GOLD, allow_pickle=False)
    Hp, steps = int(d["Hp"]), int(d["plan_steps"])
    nl = {k[3:]: d[k] for k in d.files if k.startswith("nl_")}
    p = M.plan_first_step(nl, Hp)
    # the swap: the controller's left parameter is the script's right_limit (-0.5)
    np.testing.assert_array_equal(p["left"], -0.5)
    np.testing.assert_array_equal(p["right"], 0.5)
    np.testing.assert_array_equal(p["x1"], [0.97, 0, 0, 0, 0])
    s_hist = [0.0]
    for j in range(steps):
        for k in p:
            np.testing.assert_array_equal(p[k], d[f"p{j}_{k}"], err_msg=f"step {j + 1} {k}")
        if j + 1 < steps:
            p = M.plan_next_step(d[f"z{j}"], s_hist, j + 2, p["curv"], Hp)
            np.testing.assert_array_equal(p["x1"], d[f"z{j}"][:5])        # x0 = XX_dt(:,1)
    assert len(s_hist) == steps - 1 + Hp and all(np.diff(s_hist) > 0)
