"""Lab (GPU): re-solve the agents tools/f32_capture.py saved (fp32-path solves that ended with KKT > 1e-6)
on the GPU: the fp32 path, and the fp64 Riccati kernel at tol 1e-9 / 1e-6.

  python tools/f32_replay.py CAPTURE.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    import cmpc

    d = np.load(sys.argv[1])
    P = {k[7:]: d[k] for k in d.files if k.startswith("shared_")}
    for k in ("nx", "nu", "N", "ns", "mc"):
        P[k] = int(P[k])
    for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
        P[k] = np.ascontiguousarray(d[k])
    print("capture: kkt", d["kkt"], "status", d["status"], "iters", d["iters"], flush=True)
    ctx = cmpc.Context(0)
    for name, kw in (("fp32 path", dict(fp32=True, tol=1e-6)), ("fp64 tol 1e-9", dict(riccati=True)),
                     ("fp64 tol 1e-6", dict(riccati=True, tol=1e-6)), ("fp64 tol 1e-12", dict(riccati=True, tol=1e-12))):
        z, kkt, it, st = cmpc.solve_mpc(P, ctx, **kw)
        print(f"{name}: status {st.tolist()} iters {it.tolist()} kkt {kkt.tolist()} |z - z_capture| "
              f"{np.abs(z - d['z']).max():.2e}", flush=True)


if __name__ == "__main__":
    main()
