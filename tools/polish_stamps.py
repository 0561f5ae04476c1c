"""Diagnostic (GPU): per-section clocks of the polish kernel (mpc_polish.hip) on one round of bench.py's
lpv_rounds population.  The round's structured problems (the GPU builder's arrays read back) are re-solved
through the host-array path with rescue + polish and a stamps buffer; the polish kernel writes its section
clocks (slots 8..14: init, H build, H factor, G_A rows, Y, S build + factor + Newton linear algebra,
residual sweeps) for the agents it polished (slots 0 / 1 / 4 >> 1: passes / |A| / Newton steps; the v3 kernel's own clocks
stay in the others' slots).

  python tools/polish_stamps.py [round] [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    import torch

    import bench
    import cmpc
    from cmpc.rounds import LPVRounds

    rnd = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ctx = cmpc.Context(0)
    bp, args, kw = bench.lpv_population(ctx)
    R = LPVRounds(bp, *args, **kw)
    for _ in range(rnd):
        R.step(halt=False)
    R.gather()
    R.solve()
    torch.cuda.synchronize()
    _, _, P = bench.lpv_check_round(bp, R, np.arange(R.B))
    names = ["init", "H build", "H factor", "G_A rows", "Y", "S + Newton l.a.", "residual sweeps"]
    for rep in range(reps):
        st = torch.zeros((R.B, 16), dtype=torch.int64, device="cuda")
        z, kkt, it, status = cmpc.solve_mpc(P, ctx, rescue=True, polish=True, stamps=st.data_ptr())
        s = st.cpu().numpy()
        pol = (s[:, 0] >= 1) & (s[:, 0] <= 2) & (s[:, 1] < 1000)
        print(f"rep {rep}: {int(pol.sum())} polished agents of {R.B}; status {dict(zip(*np.unique(status, return_counts=True)))}")
        if pol.any():
            sec = s[pol][:, 8:15].astype(np.float64)
            print("   |A| mean %.1f max %d, passes mean %.2f, Newton steps mean %.2f max %d" % (
                s[pol, 1].mean(), s[pol, 1].max(), s[pol, 0].mean(), (s[pol, 4] >> 1).mean(), (s[pol, 4] >> 1).max()))
            for j, nm in enumerate(names):
                print(f"   {nm:16s} mean {sec[:, j].mean() / 1e3:8.1f} k clk   max {sec[:, j].max() / 1e3:8.1f} k")
            if os.environ.get("CMPC_LIB_PATH"):  # lab builds (-DCMPC_POL_LAB): a lab figure in slot 7
                print(f"   slot 7 (lab)     mean {s[pol, 7].mean() / 1e3:8.1f} k clk   max {s[pol, 7].max() / 1e3:8.1f} k")
            tot = sec.sum(1)
            print(f"   total            mean {tot.mean() / 1e3:8.1f} k clk   max {tot.max() / 1e3:8.1f} k")


if __name__ == "__main__":
    main()
