"""ORACLE (test infrastructure only) — generator of tests/golden/*.npz.

Runs ONLY in the build container, where /root/reference exists.  It imports the
reference's own ``plan_lib`` (read-only, PYTHONDONTWRITEBYTECODE=1) with an
``osqp`` module stub injected into ``sys.modules``: the stub's
``OSQP.setup(**kw)`` captures exactly the (P, q, A, l, u) that
``osqp_solve_qp`` (distributedPlanner/LPV_Planner.py:222-239) hands to OSQP, and
its ``solve()`` returns the optimum certified by oracle/qp_ipm.py (OSQP itself
is absent).  The reference's PlannerLPV.solve then unpacks that solution with
its own code, and this script chains the control steps with the loop semantics
of planner/scripts/LPV_HP_N_main.py:96-117 (x0 <- xPred[1], x_old <- xPred[1:],
u_old <- uPred (not shifted), Jacobi exchange of X,Y).

Nothing from /root/reference is written into the fixtures except the numbers
its code computed.  Usage:  python oracle/gen_fixtures.py
"""
import os
import sys
import types

import numpy as np
import scipy.sparse as sp

REF_LIB = "/root/reference/planner/lib"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from oracle import qp_ipm  # noqa: E402

_last = {}


class _Obj:
    pass


class _StubOSQP:
    """Captures OSQP.setup kwargs; solve() returns the certified IPM optimum."""

    def setup(self, **kw):
        self.kw = kw

    def warm_start(self, **kw):
        pass

    def solve(self):
        kw = self.kw
        P, A = kw["P"].toarray(), kw["A"].toarray()
        r = qp_ipm.solve_qp(P, kw["q"], A, kw["l"], kw["u"])
        _last.update(kw=kw, res=r)
        out = _Obj()
        out.x = r.x.copy()
        out.y = r.y.copy()
        out.info = _Obj()
        out.info.status_val = r.status_val
        out.info.status = r.status
        return out


def _import_reference():
    mod = types.ModuleType("osqp")
    mod.OSQP = _StubOSQP
    sys.modules["osqp"] = mod
    sys.path.insert(0, REF_LIB)
    from plan_lib.distributedPlanner import PlannerLPV
    from plan_lib.mapManager import Map
    from plan_lib.utilities import initialise_agents, curvature, get_ey, compute_weights
    from plan_lib.planes import hyperplane_separator
    from plan_lib.config import x0_database, experiment_utilities
    from plan_lib.distributedPlanner.LPV_Planner import _EstimateABC
    return dict(PlannerLPV=PlannerLPV, Map=Map, initialise_agents=initialise_agents,
                curvature=curvature, get_ey=get_ey, compute_weights=compute_weights,
                hyperplane_separator=hyperplane_separator, x0_database=x0_database,
                experiment_utilities=experiment_utilities, _EstimateABC=_EstimateABC)


def _coo(M):
    c = sp.coo_matrix(M)
    return c.data, c.row.astype(np.int32), c.col.astype(np.int32), np.array(M.shape, np.int32)


def gains():
    # planner/scripts/config_files/config_LPV.py:6-11
    return dict(Q=np.diag([10.0, 0.0, 0.0, 25.0, 10.0, 0.0, 0.0, 0, 0]), Qs=10000000 * np.eye(3),
                R=0 * np.diag([1, 1]), dR=50 * np.diag([1, 1]), wq=5.0)


def run_loop(R, name, N, x0s, steps, dt=0.025, vx_ref=3.0, map_name="Highway"):
    g = gains()
    n = len(x0s)
    eu = R["experiment_utilities"](None, dict(path_csv="/nonexistent/", path_pck="/nonexistent/",
                                              vx_ref=vx_ref))
    maps = [R["Map"](map_name)] * n
    agents, x_old, u_old = R["initialise_agents"](x0s, N, dt, maps)
    ns = [[j for j in range(n) if j != i] for i in range(n)]
    planners = [R["PlannerLPV"](g["Q"], g["Qs"], g["R"], g["dR"], N, dt, maps[i], i, g["wq"],
                                eu.model_param, eu.sys_lim) for i in range(n)]
    x0 = [np.array(x_old[i][0, :], float) for i in range(n)]
    rec = {k: [] for k in ("step", "agent", "x0", "x_last", "u_last", "x_agents", "pose", "u_old",
                           "z", "y", "stat", "prim", "comp", "iters", "planes", "xPred", "uPred",
                           "sPred", "P", "q", "A", "l", "u")}
    for step in range(steps):
        x_pred, u_pred = [None] * n, [None] * n
        for i, pl in enumerate(planners):
            u_prev = [pl.OldSteering[0], pl.OldAccelera[0]]
            x_ag = agents[:, ns[i], :].copy()
            pose = agents[:, i, :].copy()
            feas, sol, planes = pl.solve(x0[i], x_old[i], u_old[i], x_ag, ns[i], pose)
            assert feas == 1
            kw, res = _last["kw"], _last["res"]
            rec["step"].append(step); rec["agent"].append(i)
            rec["x0"].append(np.array(x0[i], float))
            rec["x_last"].append(np.array(x_old[i], float))
            rec["u_last"].append(np.array(u_old[i], float))
            rec["x_agents"].append(x_ag); rec["pose"].append(pose)
            rec["u_old"].append(np.array(u_prev, float))
            rec["z"].append(res.x); rec["y"].append(res.y)
            rec["stat"].append(res.kkt["stat_rel"]); rec["prim"].append(res.kkt["prim"])
            rec["comp"].append(res.kkt["comp"]); rec["iters"].append(res.iters)
            rec["planes"].append(np.array(planes)); rec["xPred"].append(pl.xPred.copy())
            rec["uPred"].append(pl.uPred.copy()); rec["sPred"].append(pl.sPred.copy())
            rec["P"].append(_coo(kw["P"].toarray())); rec["q"].append(np.array(kw["q"]))
            rec["A"].append(_coo(kw["A"].toarray())); rec["l"].append(np.array(kw["l"]))
            rec["u"].append(np.array(kw["u"]))
            x_pred[i], u_pred[i] = pl.xPred.copy(), pl.uPred.copy()
            x0[i] = x_pred[i][1, :].copy()
        u_old = u_pred
        x_old = [x_pred[i][1:, :] for i in range(n)]
        agents = np.swapaxes(np.asarray(x_pred)[:, :, -2:], 0, 1)
    out = dict(N=np.int32(N), n_agents=np.int32(n), steps=np.int32(steps), dt=np.float64(dt),
               vx_ref=np.float64(vx_ref), map_name=np.array(map_name))
    nq = len(rec["step"])
    for k in ("step", "agent", "iters"):
        out[k] = np.array(rec[k], np.int32)
    for k in ("stat", "prim", "comp"):
        out[k] = np.array(rec[k], float)
    for k in ("x0", "u_old", "z", "y", "q", "l", "u", "planes", "xPred", "uPred", "sPred", "pose",
              "x_agents"):
        out[k] = np.stack(rec[k])
    for j in range(nq):  # ragged (N+1 rows at step 0, N afterwards)
        out[f"x_last_{j}"] = rec["x_last"][j]
        out[f"u_last_{j}"] = rec["u_last"][j]
        for nm in ("P", "A"):
            d, r, c, s = rec[nm][j]
            out[f"{nm}_{j}_data"], out[f"{nm}_{j}_row"], out[f"{nm}_{j}_col"], out[f"{nm}_{j}_shape"] = d, r, c, s
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{path}: {nq} QPs, max stat_rel {out['stat'].max():.1e} prim {out['prim'].max():.1e} "
          f"comp {out['comp'].max():.1e}, {os.path.getsize(path) / 1e3:.0f} kB")


def map_goldens(R):
    out = {}
    rng = np.random.default_rng(7)
    for nm in ("Highway", "oval", "Oval2", "SL"):
        mp = R["Map"](nm)
        out[f"{nm}_PointAndTangent"] = mp.PointAndTangent
        out[f"{nm}_halfWidth"] = np.asarray(mp.halfWidth, float)
        out[f"{nm}_TrackLength"] = np.asarray(mp.TrackLength, float)
        L = float(mp.TrackLength[0])
        s = np.concatenate([rng.uniform(0, L * 0.999, 64), mp.PointAndTangent[1:-1, 3, 0] + 1e-9])
        out[f"{nm}_s"] = s
        out[f"{nm}_curv"] = np.array([R["curvature"](v, mp) for v in s])
        out[f"{nm}_ey"] = R["get_ey"](s, mp)
        ey = rng.uniform(-0.5, 0.5, s.shape[0])
        out[f"{nm}_ey_in"] = ey
        if not mp.open:
            # the reference's wrap_s indexes TrackLength[None] on closed tracks and
            # raises (track_initialization.py:307-308): no global-position golden there
            continue
        gp = []
        for v, e in zip(s, ey):
            x, y, th = mp.getGlobalPosition(v, e)
            gp.append([float(np.squeeze(x)), float(np.squeeze(y)), float(np.squeeze(th))])
        out[f"{nm}_global"] = np.array(gp)
    path = os.path.join(OUT, "maps.npz")
    np.savez_compressed(path, **out)
    print(path, f"{os.path.getsize(path) / 1e3:.0f} kB")


def schedule_goldens(R):
    """_EstimateABC (LPV_Planner.py:477-591), compute_hyperplane (compute_plane.py:41-68),
    compute_weights (misc.py:10-18) on seeded random inputs (incl. the vx<0.2 branch)."""
    rng = np.random.default_rng(11)
    g = gains()
    eu = R["experiment_utilities"](None, dict(path_csv="/n/", path_pck="/n/", vx_ref=3.0))
    mp = R["Map"]("Highway")
    out = {}
    for case, N in enumerate((10, 30)):
        pl = R["PlannerLPV"](g["Q"], g["Qs"], g["R"], g["dR"], N, 0.025, mp, 0, g["wq"],
                             eu.model_param, eu.sys_lim)
        st = np.zeros((N + 1, 9))
        st[:, 0] = rng.uniform(0.05, 3.0, N + 1)
        st[:3, 0] = [0.1, 0.19, 0.2]
        st[:, 1] = rng.uniform(-0.3, 0.3, N + 1)
        st[:, 2] = rng.uniform(-1, 1, N + 1)
        st[:, 3] = rng.uniform(-0.6, 0.6, N + 1)
        st[:, 4] = rng.uniform(-0.4, 0.4, N + 1)
        st[:, 5] = rng.uniform(-3, 3, N + 1)
        st[:, 6] = rng.uniform(0, 46.0, N + 1)
        st[:, 7:] = rng.uniform(0, 20, (N + 1, 2))
        u = rng.uniform(-0.3, 0.3, (N, 2))
        A, B, C, ey = R["_EstimateABC"](pl, st, u)
        out[f"c{case}_states"], out[f"c{case}_u"] = st, u
        out[f"c{case}_A"], out[f"c{case}_B"], out[f"c{case}_ey"] = np.array(A), np.array(B), ey
        nb = 2
        pose = rng.uniform(0, 10, (N + 1, 2))
        ag = rng.uniform(0, 10, (N + 1, nb, 2))
        hs = R["hyperplane_separator"](nb, N)
        out[f"c{case}_pose"], out[f"c{case}_agents"] = pose, ag
        out[f"c{case}_planes"] = hs.compute_hyperplane(ag, pose, 0, [1, 2], keep_sign=True)
        w, d = R["compute_weights"](pose, ag, 0.25)
        out[f"c{case}_w"], out[f"c{case}_dist"] = w, d
    path = os.path.join(OUT, "schedule.npz")
    np.savez_compressed(path, **out)
    print(path, f"{os.path.getsize(path) / 1e3:.0f} kB")


def main():
    if not os.path.isdir(REF_LIB):
        raise SystemExit("reference not present: fixtures are generated in the build container only")
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    os.makedirs(OUT, exist_ok=True)
    R = _import_reference()
    x0db = R["x0_database"]
    only = set(sys.argv[1:])          # optional subset of fixture names
    want = lambda nm: not only or nm in only
    if want("maps"):
        map_goldens(R)
    if want("schedule"):
        schedule_goldens(R)
    if want("lpv_n10_a2"):
        run_loop(R, "lpv_n10_a2", 10, x0db[0:2], steps=4)
    if want("lpv_n30_a3"):
        run_loop(R, "lpv_n30_a3", 30, x0db[0:3], steps=4)
    slow = [list(x0db[0]), list(x0db[1])]
    slow[0][0] = 0.1                                   # vx < 0.2 -> LPV_Planner.py:505-517
    slow[1][0] = 0.15
    if want("lpv_n10_lowspeed"):
        run_loop(R, "lpv_n10_lowspeed", 10, slow, steps=3)
    if want("lpv_n10_a1"):
        run_loop(R, "lpv_n10_a1", 10, x0db[0:1], steps=2)  # no neighbours: nb = 0
    if want("lpv_n20_a4"):
        run_loop(R, "lpv_n20_a4", 20, x0db[0:4], steps=2)
    if want("lpv_n125_a3"):
        # the reference's shipped configuration: N = 125, 3 agents, Highway
        # (planner/scripts/config_files/config_LPV.py:13-24, LPV_HP_N_main.py)
        run_loop(R, "lpv_n125_a3", 125, x0db[0:3], steps=2)


if __name__ == "__main__":
    main()
