"""Diagnostic: solve every captured reference QP case through PlannerLPVBatch on the GPU and print
status / iterations / KKT / max|z - z*| per agent (test infrastructure; reads tests/golden)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd"), os.path.join(ROOT, "tests")]

import cmpc  # noqa: E402
from conftest import LPV_CASES, lpv_qps  # noqa: E402
from oracle import lpv_ref as L  # noqa: E402


def main(names, riccati=False):
    ctx = cmpc.Context(0)
    g = L.paper_gains()
    tr = L.Track.build("Highway")
    for name in names:
        groups = {}
        for j, c in lpv_qps(name):
            groups.setdefault(c["x_last"].shape[0], []).append(c)
        for rows, cs in groups.items():
            N = cs[0]["N"]
            bp = cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], N, cs[0]["dt"], tr, g["wq"],
                                      L.SCALED_CAR_MODEL, L.scaled_car_limits(cs[0]["vx_ref"]), ctx=ctx,
                                      riccati=riccati)
            xa = np.stack([c["x_agents"] for c in cs])
            args = (np.stack([c["x0"] for c in cs]), np.stack([c["x_last"] for c in cs]),
                    np.stack([c["u_last"] for c in cs]), np.stack([c["u_old"] for c in cs]),
                    xa if xa.shape[2] else None, np.stack([c["pose"] for c in cs]))
            res = bp.solve(*args)
            t0 = time.perf_counter()
            for _ in range(3):
                bp.solve(*args)
            ms = (time.perf_counter() - t0) / 3 * 1e3
            print(f"{name} rows {rows} riccati={riccati}: {len(cs)} agents in {ms:.3f} ms per call "
                  f"(host arrays in/out)", flush=True)
            for a, c in enumerate(cs):
                err = float(np.abs(res["z"][a] - c["z"]).max())
                print(f"{name} rows {rows} agent {a}: status {res['status'][a]} iters {res['iters'][a]} "
                      f"kkt {res['kkt'][a]:.2e} err {err:.2e}", flush=True)


if __name__ == "__main__":
    ric = "--riccati" in sys.argv
    names = [a for a in sys.argv[1:] if not a.startswith("--")] or LPV_CASES
    main(names, False)
    if ric:
        main(names, True)
