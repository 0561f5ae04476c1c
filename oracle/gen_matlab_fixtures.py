"""TEST INFRASTRUCTURE: golden vectors for the MATLAB per-agent QP path (oracle/matlab_ref.py):
the quadprog models YALMIP would hand to callquadprog.m:63-69 for the 5-state LPV-MPC of
LPV_MPC_fnc_dt_Vnew.m (Hp = 15, dt = 0.1 as PLAN_NL_LPV_MPC_dt_WORKS_Oval.m uses it), each with
its optimum certified by the dense IPM oracle/qp_ipm.py.  Writes tests/golden/matlab_lpv_mpc.npz.

Cases 0..3: the planner script's first control steps.  Step k = 1 is scheduled from the
reference's own NL_vars.mat (PLAN_NL_LPV_MPC_dt_WORKS_Oval.m:19, :127-167; loaded with
scipy.io.loadmat, which reads data only — the MCOS map object in the file is skipped), steps
2..4 from the certified optimum of the step before (:171-199, :259-260).  The six NL_vars arrays
used are stored in the npz too, so tests re-derive the parameters without /root/reference.
Cases 4..7: hand-built parameter sets (matlab_ref.sample_parameters) at other speeds and
max_vel.  MATLAB is absent, so quadprog's own outputs are not available (parity unpinned by
them; matlab_ref.py header).

    python oracle/gen_matlab_fixtures.py          (needs /root/reference; build container only)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import matlab_ref as M  # noqa: E402
from oracle import qp_ipm  # noqa: E402

NL_VARS = "/root/reference/Matlab-tests/mrs_LPV_MPC/NL_vars.mat"
NL_KEYS = ("ss_NL", "ey_NL", "etheta_NL", "Vy_NL", "Vx_NL", "delta")
PLAN_STEPS = 4
CASES = [dict(seed=0, max_vel=3.5, vx=1.5), dict(seed=1, max_vel=3.5, vx=2.2),
         dict(seed=2, max_vel=3.8, vx=3.0), dict(seed=3, max_vel=3.5, vx=1.0)]
HP, DT = 15, 0.1


def solve_case(out, j, p, max_vel):
    F, Kf, c, Q, lb, ub = M.lpv_mpc_interface(HP, DT, p, max_vel)
    mod = M.yalmip2quadprog(F, Kf, c, Q, lb, ub)
    r = qp_ipm.solve_qp(*M.osqp_form(mod))
    assert r.status == "solved" and r.kkt["stat_rel"] < 1e-9 and r.kkt["prim"] < 1e-9, r.kkt
    print(f"case {j}: n {len(c)}, eq {mod['Aeq'].shape[0]}, ineq {mod['A'].shape[0]}, iters {r.iters}, kkt {r.kkt}")
    for k, v in p.items():
        out[f"p{j}_{k}"] = np.asarray(v, float)
    out[f"max_vel_{j}"] = max_vel
    for k in ("H", "f", "A", "b", "Aeq", "beq", "lb", "ub"):
        out[f"m{j}_{k}"] = mod[k]
    out[f"z{j}"] = r.x
    out[f"kkt{j}"] = np.array([r.kkt["stat_rel"], r.kkt["prim"], r.kkt["comp"]])
    return r.x


def main():
    import scipy.io

    nl = scipy.io.loadmat(NL_VARS, variable_names=list(NL_KEYS) + ["Tss"])
    assert float(nl["Tss"].ravel()[0]) == DT
    out = {"Hp": HP, "dt": DT, "ncases": PLAN_STEPS + len(CASES), "plan_steps": PLAN_STEPS}
    for k in NL_KEYS:
        out[f"nl_{k}"] = np.asarray(nl[k], float).ravel()
    p = M.plan_first_step(nl, HP)
    s_hist = [0.0]                                           # :165 s(1) = 0
    for j in range(PLAN_STEPS):
        z = solve_case(out, j, p, 3.5)                       # :58 LPV_MPC_fnc_dt_Vnew(Hp, Tss): max_vel 3.5
        if j + 1 < PLAN_STEPS:
            p = M.plan_next_step(z, s_hist, j + 2, p["curv"], HP)
    for j, cs in enumerate(CASES):
        solve_case(out, PLAN_STEPS + j, M.sample_parameters(HP, cs["seed"], vx=cs["vx"]), cs["max_vel"])
    path = os.path.join(ROOT, "tests", "golden", "matlab_lpv_mpc.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
