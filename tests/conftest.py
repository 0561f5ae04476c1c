import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "colaborativempc-_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device and the built libcmpc.so")


def polish_amax(P):
    """The polish kernel's active-set capacity for this problem shape (cmpc_plan_info.polish_max_active,
    host only), handed to the C restatement so both sides polish the same agents."""
    from cmpc.solver import plan

    return plan(P, 1, rescue=True, polish=True)["polish_max_active"]


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def golden_matrix(d, nm, j):
    shp = tuple(int(v) for v in d[f"{nm}_{j}_shape"])
    return sp.coo_matrix((d[f"{nm}_{j}_data"], (d[f"{nm}_{j}_row"], d[f"{nm}_{j}_col"])), shape=shp).toarray()


LPV_CASES = ["lpv_n10_a2", "lpv_n30_a3", "lpv_n10_lowspeed", "lpv_n10_a1", "lpv_n20_a4", "lpv_n125_a3"]


def lpv_qps(name):
    """Yield (index, dict) for every captured reference QP of a golden file."""
    d = golden(name)
    for j in range(len(d["step"])):
        yield j, dict(N=int(d["N"]), step=int(d["step"][j]), agent=int(d["agent"][j]), x0=d["x0"][j],
                      x_last=d[f"x_last_{j}"], u_last=d[f"u_last_{j}"], u_old=d["u_old"][j],
                      x_agents=d["x_agents"][j], pose=d["pose"][j], z=d["z"][j], y=d["y"][j],
                      planes=d["planes"][j], P=golden_matrix(d, "P", j), A=golden_matrix(d, "A", j),
                      q=d["q"][j], l=d["l"][j], u=d["u"][j], dt=float(d["dt"]), vx_ref=float(d["vx_ref"]),
                      map_name=str(d["map_name"]))


@pytest.fixture(scope="session")
def gpu_ctx():
    import cmpc

    return cmpc.default_context(0)


KKT_TOL = 1e-6


def reference_kkt(P, q, A, l, u, z):
    """Reference-form (OSQP-form, LPV_Planner.py:222-233) KKT residual of a primal point with its
    best sign-feasible multipliers (oracle.qp_ipm.kkt_of_primal): max of the relative
    stationarity, the primal violation and the complementarity."""
    from oracle import qp_ipm

    cert, _ = qp_ipm.kkt_of_primal(P, q, A, l, u, z)
    return max(cert["stat_rel"], cert["prim"], cert["comp"]), cert


def assert_matches_optimum(z, c, ztol=1e-6):
    """z solves the captured reference QP c: within ztol of the certified optimum z*; or — where the
    optimum sits on a weakly active bound (multiplier ~ 0, the degenerate case in which
    interior-point iterates approach the bound only like sqrt(mu)) — z carries its own certificate:
    reference-form KKT residual <= 1e-6 (reference_kkt) and objective equal to z*'s to 1e-10."""
    err = float(np.abs(z - c["z"]).max())
    if err < ztol:
        return err
    P, q, A, l, u = c["P"], c["q"], c["A"], c["l"], c["u"]
    kkt, cert = reference_kkt(P, q, A, l, u, z)
    f, fs = 0.5 * z @ P @ z + q @ z, 0.5 * c["z"] @ P @ c["z"] + q @ c["z"]
    assert kkt <= KKT_TOL and f - fs <= 1e-10 * abs(fs), (err, cert, f - fs)
    return err
