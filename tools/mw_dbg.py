"""Lab (GPU): the Riccati kernel's latency mode (four wavefronts per agent) against the one-wave kernel on
the reference's N = 125 captured QPs, iteration by iteration (max_iter = 1, 2, ...): the first cap at
which z / kkt / status differ.

  python tools/mw_dbg.py [max_cap]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd"), os.path.join(ROOT, "tests")]


def main():
    import cmpc
    from cmpc import _lib as L
    from conftest import lpv_qps
    from oracle import lpv_ref as R

    cap = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ctx = cmpc.Context(0)
    g = R.paper_gains()
    tr = R.Track.build("Highway")
    cs = [c for _, c in lpv_qps("lpv_n125_a3")]
    for rows in sorted({c["x_last"].shape[0] for c in cs}):
        grp = [c for c in cs if c["x_last"].shape[0] == rows]
        bp = cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], grp[0]["N"], grp[0]["dt"], tr, g["wq"],
                                  R.SCALED_CAR_MODEL, R.scaled_car_limits(grp[0]["vx_ref"]), ctx=ctx)
        args = (np.stack([c["x0"] for c in grp]), np.stack([c["x_last"] for c in grp]),
                np.stack([c["u_last"] for c in grp]), np.stack([c["u_old"] for c in grp]),
                np.stack([c["x_agents"] for c in grp]), np.stack([c["pose"] for c in grp]))
        base = bp.opts.flags
        for m in list(range(1, cap + 1)) + [60]:
            bp.opts = L.opts(None, m, base)
            a = bp.solve(*args)
            bp.opts = L.opts(None, m, base | L.CMPC_FLAG_ONE_WAVE)
            o = bp.solve(*args)
            print(f"rows {rows} max_iter {m:2d}: |dz| {np.abs(a['z'] - o['z']).max():.3e} kkt mw {a['kkt']} one {o['kkt']} "
                  f"status {a['status'].tolist()} / {o['status'].tolist()} iters {a['iters'].tolist()} / "
                  f"{o['iters'].tolist()}", flush=True)


if __name__ == "__main__":
    main()
