"""Where the time of one literal ``osqp_solve_qp`` call goes (test infrastructure; GPU box).

bench.py's `osqp_dropin` line times the whole call on the 12 reference-captured N = 30 agent QPs of
tests/golden/lpv_n30_a3.npz.  This splits it into the host-side structure recognition
(cmpc.structure.recognize), the structured solve (cmpc.solver.solve_mpc with the rescue + polish
policy: host -> HBM copies, the launches, HBM -> host) and the OSQP-style result (objective, primal
residual), per QP, mean over `reps` passes.

  python tools/dropin_breakdown.py [reps]
"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def qps_of_golden():
    d = np.load(os.path.join(ROOT, "tests", "golden", "lpv_n30_a3.npz"), allow_pickle=False)

    def mat(nm, j):
        shp = tuple(int(v) for v in d[f"{nm}_{j}_shape"])
        return sp.csr_matrix((d[f"{nm}_{j}_data"], (d[f"{nm}_{j}_row"], d[f"{nm}_{j}_col"])), shape=shp)

    qps = []
    for j in range(len(d["step"])):
        Aall, l, u = mat("A", j), d["l"][j], d["u"][j]
        eq = np.isfinite(l) & (l == u)
        qps.append((mat("P", j), d["q"][j], Aall[np.flatnonzero(~eq)], u[~eq], Aall[np.flatnonzero(eq)], u[eq]))
    return qps, d["z"]


def main(reps):
    import cmpc
    from cmpc import qp as Q
    from cmpc import structure as St
    from cmpc.solver import solve_mpc

    ctx = cmpc.default_context() if hasattr(cmpc, "default_context") else None
    qps, zc = qps_of_golden()
    t_rec, t_sol, t_res, t_all, iters = [], [], [], [], []
    for rep in range(reps + 1):
        for j, (P, q, G, h, A, b) in enumerate(qps):
            t0 = time.perf_counter()
            p = St.recognize(P, q, G, h, A, b)
            t1 = time.perf_counter()
            z, kkt, it, st = solve_mpc(St.stack([p]), ctx, rescue=True, polish=True)
            t2 = time.perf_counter()
            x = z[0]
            Q._osqp_result(x, int(st[0]), "solved", int(it[0]), float(0.5 * x @ (P @ x) + q @ x), float(kkt[0]),
                           Q._pri_res(x, G, h, A, b), "structured")
            t3 = time.perf_counter()
            cmpc.osqp_solve_qp(P, q, G, h, A, b, ctx=ctx)
            t4 = time.perf_counter()
            if rep:   # the first pass warms up
                t_rec.append(t1 - t0)
                t_sol.append(t2 - t1)
                t_res.append(t3 - t2)
                t_all.append(t4 - t3)
                iters.append(int(it[0]))
            assert np.abs(x - zc[j]).max() < 1e-6
    ms = lambda v: round(float(np.mean(v)) * 1e3, 4)  # noqa: E731
    print(json.dumps({"qps": len(qps), "reps": reps, "recognize_ms": ms(t_rec), "solve_ms": ms(t_sol),
                      "result_ms": ms(t_res), "osqp_solve_qp_ms": ms(t_all),
                      "solve_ms_max": round(float(np.max(t_sol)) * 1e3, 4),
                      "iters": sorted(set(iters))}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
