"""Diagnostic: the GPU LPV builder (cmpc_lpv_build_dev) against the reference's own scheduling
goldens (tests/golden/schedule.npz) and the oracle builder (oracle/lpv_ref.py) — max abs / ulp
differences per output."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd"), os.path.join(ROOT, "tests")]

import cmpc  # noqa: E402
from conftest import golden, lpv_qps  # noqa: E402
from oracle import lpv_ref as L  # noqa: E402


def ulps(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    d = np.abs(a - b)
    sc = np.spacing(np.maximum(np.abs(a), np.abs(b)))
    with np.errstate(invalid="ignore", divide="ignore"):
        u = np.where(d == 0, 0.0, d / np.where(sc > 0, sc, 1))
    return float(d.max(initial=0)), float(u.max(initial=0))


def planner(N, ctx):
    g = L.paper_gains()
    return cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], N, 0.025, L.Track.build("Highway"), g["wq"],
                                L.SCALED_CAR_MODEL, L.scaled_car_limits(3.0), ctx=ctx)


def main():
    ctx = cmpc.Context(0)
    d = golden("schedule")
    for case, N in enumerate((10, 30)):
        st, u = d[f"c{case}_states"], d[f"c{case}_u"]
        out = planner(N, ctx).build(st[None], u[None], d[f"c{case}_agents"][None], d[f"c{case}_pose"][None])
        print(f"schedule c{case} N={N}: err {out['err'].tolist()}")
        for k, ref in (("A", d[f"c{case}_A"]), ("B", d[f"c{case}_B"]), ("planes", d[f"c{case}_planes"])):
            print(f"  {k:7s} max|d| {ulps(out[k][0], ref)[0]:.2e}  max ulp {ulps(out[k][0], ref)[1]:.1f}")
        hw = out["h"][0][:, 2]
        print(f"  hw rows equal to ey[:N]: {np.array_equal(hw, d[f'c{case}_ey'][:N])}")
    g = L.paper_gains()
    tr = L.Track.build("Highway")
    for name in ("lpv_n10_a2", "lpv_n30_a3", "lpv_n10_lowspeed", "lpv_n20_a4"):
        worst = {}
        for j, c in lpv_qps(name):
            lim = L.scaled_car_limits(c["vx_ref"])
            qp = L.assemble(c["x0"], c["x_last"], c["u_last"], c["x_agents"], c["pose"], c["u_old"], c["N"], c["dt"],
                            tr, L.SCALED_CAR_MODEL, lim, g)
            s = L.structured(qp, c["x0"], c["u_old"], c["N"], lim, g)
            xa = c["x_agents"] if c["x_agents"].shape[1] else None
            o = planner(c["N"], ctx).build(c["x_last"][None], c["u_last"][None], None if xa is None else xa[None],
                                           c["pose"][None])
            for k in ("A", "B", "qlin", "C", "h"):
                a, u_ = ulps(o[k][0], s[k][0])
                w = worst.get(k, (0.0, 0.0))
                worst[k] = (max(w[0], a), max(w[1], u_))
        print(name, {k: f"{v[0]:.1e} ({v[1]:.0f} ulp)" for k, v in worst.items()})


if __name__ == "__main__":
    main()
