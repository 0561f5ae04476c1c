"""Diagnostic: per-section shader-clock breakdown of the Riccati kernel (mpc_riccati.hip) on the
reference's N = 125 captured QPs (tests/golden/lpv_n125_a3.npz), or a synthetic long horizon.
Usage: python tools/ric_stamps.py [lpv_case] | python tools/ric_stamps.py --di n N"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import cmpc  # noqa: E402
from cmpc import _lib as L  # noqa: E402

SLOTS = 16
NAMES = {14: "setup + output", 0: "residuals (2 adjoints)", 1: "stage weights, max th", 2: "factor (fp64)",
         3: "factor (double-double)", 4: "rhs (rho, C'rt, adjoint)", 5: "solve (2 sweeps)",
         6: "refinement (dd residual + solve)", 7: "rows, slacks, step", 8: "update"}


def report(st, iters, label, ms):
    a = st.astype(np.float64)
    print(f"{label}: {ms:.3f} ms per call; iterations {iters.tolist()}; dd iterations {a[:, 12].astype(int).tolist()}; "
          f"refinement steps {a[:, 13].astype(int).tolist()}")
    tot = a[:, [k for k in NAMES]].sum(1)
    for k, nm in NAMES.items():
        print(f"  {nm:34s} " + " ".join(f"{v / 1e6:8.3f}M" for v in a[:, k]) + "   clk per agent")
    it = np.maximum(a[:, SLOTS - 1], 1)
    print(f"  {'total':34s} " + " ".join(f"{v / 1e6:8.3f}M" for v in tot) +
          "   | per iteration " + " ".join(f"{v / 1e3:.0f}k" for v in tot / it))


def lpv(name):
    from conftest import lpv_qps
    from oracle import lpv_ref as R

    ctx = cmpc.Context(0)
    g = R.paper_gains()
    tr = R.Track.build("Highway")
    groups = {}
    for j, c in lpv_qps(name):
        groups.setdefault(c["x_last"].shape[0], []).append(c)
    for rows, cs in groups.items():
        N = cs[0]["N"]
        bp = cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], N, cs[0]["dt"], tr, g["wq"], R.SCALED_CAR_MODEL,
                                  R.scaled_car_limits(cs[0]["vx_ref"]), ctx=ctx, riccati=True)
        xa = np.stack([c["x_agents"] for c in cs])
        args = (np.stack([c["x0"] for c in cs]), np.stack([c["x_last"] for c in cs]),
                np.stack([c["u_last"] for c in cs]), np.stack([c["u_old"] for c in cs]),
                xa if xa.shape[2] else None, np.stack([c["pose"] for c in cs]))
        st = torch.zeros((len(cs), SLOTS), dtype=torch.int64, device="cuda")
        t0 = time.perf_counter()
        res = bp.solve(*args)
        ms = (time.perf_counter() - t0) * 1e3
        bp.opts = L.opts(flags=L.CMPC_FLAG_RICCATI, stamps=st.data_ptr())
        res = bp.solve(*args)
        torch.cuda.synchronize()
        report(st.cpu().numpy(), res["iters"], f"{name} rows {rows} ({len(cs)} agents, status {res['status'].tolist()})",
               ms)


if __name__ == "__main__":
    lpv(sys.argv[1] if len(sys.argv) > 1 else "lpv_n125_a3")
