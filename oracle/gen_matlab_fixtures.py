"""TEST INFRASTRUCTURE: golden vectors for the MATLAB per-agent QP path (oracle/matlab_ref.py):
the quadprog models YALMIP would hand to callquadprog.m:63-69 for the 5-state LPV-MPC of
LPV_MPC_fnc_dt_Vnew.m (Hp = 15, dt = 0.1 as PLAN_NL_LPV_MPC_dt_WORKS_Oval.m uses it), each with
its optimum certified by the dense IPM oracle/qp_ipm.py.  MATLAB is absent, so the parameter
sets are hand-built (matlab_ref.sample_parameters).  Writes tests/golden/matlab_lpv_mpc.npz.

    python oracle/gen_matlab_fixtures.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import matlab_ref as M  # noqa: E402
from oracle import qp_ipm  # noqa: E402

CASES = [dict(seed=0, max_vel=3.5, vx=1.5), dict(seed=1, max_vel=3.5, vx=2.2),
         dict(seed=2, max_vel=3.8, vx=3.0), dict(seed=3, max_vel=3.5, vx=1.0)]
HP, DT = 15, 0.1


def main():
    out = {"Hp": HP, "dt": DT, "ncases": len(CASES)}
    for j, cs in enumerate(CASES):
        p = M.sample_parameters(HP, cs["seed"], vx=cs["vx"])
        F, Kf, c, Q, lb, ub = M.lpv_mpc_interface(HP, DT, p, cs["max_vel"])
        mod = M.yalmip2quadprog(F, Kf, c, Q, lb, ub)
        r = qp_ipm.solve_qp(*M.osqp_form(mod))
        assert r.status == "solved" and r.kkt["stat_rel"] < 1e-9 and r.kkt["prim"] < 1e-9, r.kkt
        print(f"case {j}: n {len(c)}, eq {mod['Aeq'].shape[0]}, ineq {mod['A'].shape[0]}, iters {r.iters}, kkt {r.kkt}")
        for k, v in p.items():
            out[f"p{j}_{k}"] = np.asarray(v, float)
        out[f"max_vel_{j}"] = cs["max_vel"]
        for k in ("H", "f", "A", "b", "Aeq", "beq", "lb", "ub"):
            out[f"m{j}_{k}"] = mod[k]
        out[f"z{j}"] = r.x
        out[f"kkt{j}"] = np.array([r.kkt["stat_rel"], r.kkt["prim"], r.kkt["comp"]])
    path = os.path.join(ROOT, "tests", "golden", "matlab_lpv_mpc.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
