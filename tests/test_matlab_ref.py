"""The MATLAB per-agent QP path restated (oracle/matlab_ref.py): YALMIP's quadprog model
transformation (yalmip2quadprog.m) on hand-built known answers, and the 5-state LPV-MPC models
of LPV_MPC_fnc_dt_Vnew.m regenerated bit for bit against the committed, KKT-certified
fixtures (tests/golden/matlab_lpv_mpc.npz, oracle/gen_matlab_fixtures.py).  MATLAB is absent:
parity with MATLAB's own output is unpinned (oracle/matlab_ref.py header)."""
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
