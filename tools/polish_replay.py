"""Diagnostic (GPU): re-solve the agents tools/polish_diag.py saved at GPU status 2 through the host-array
path with rescue + polish, and print the polish kernel's per-agent diagnostics (MpcPtrs::stamps:
passes, |A|, polished merit, the method's best merit, H factored).

  python tools/polish_replay.py DIAG.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    import torch

    import cmpc
    from cmpc import _lib as L

    d = np.load(sys.argv[1])
    sel = np.flatnonzero(d["st_gpu"] == 2)
    P = {k: d[k] for k in ("Q", "R", "dR", "Qs", "u_ub", "u_lb", "row_slack", "row_sign")}
    for k in ("nx", "nu", "N", "ns", "mc"):
        P[k] = int(d[k])
    for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
        P[k] = d[k][sel]
    for rep in range(3):
        st_buf = torch.zeros((len(sel), 16), dtype=torch.int64, device="cuda")
        z, kkt, it, st = cmpc.solve_mpc(P, L.default_context(), rescue=True, polish=True, stamps=st_buf.data_ptr())
        s = st_buf.cpu().numpy()
        print("rep", rep, "status", st.tolist(), flush=True)
    f = lambda i, j: float(s[i, j:j + 1].view(np.float64)[0])  # noqa: E731
    for i in range(len(sel)):
        print(i, "iters", int(it[i]), "passes", int(s[i, 0]), "nA", int(s[i, 1]), "pol merit %.3e" % f(i, 2),
              "best_m %.3e" % f(i, 3), "h_ok", int(s[i, 4]) & 1, "newton steps", int(s[i, 4]) >> 1, "res d/s/p %.2e %.2e %.2e" % (f(i, 5), f(i, 6), f(i, 7)),
              "clk init/H/chol H/G_A/Y/S/sweeps %s" % s[i, 8:15].tolist())


if __name__ == "__main__":
    main()
