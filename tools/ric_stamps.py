"""Diagnostic: per-section shader-clock breakdown of the Riccati kernel (mpc_riccati.hip) on the
reference's N = 125 captured QPs (tests/golden/lpv_n125_a3.npz), or a synthetic long horizon.
Usage: python tools/ric_stamps.py [--one-wave] [lpv_case] | python tools/ric_stamps.py --cfg5 [agents]
(--cfg5: the first round of the BASELINE cfg5 population, N = 50, nx 6, nu 3; means over agents.
The N = 125 agent runs the kernel's latency mode, four wavefronts per agent, unless --one-wave: there
slot 0 is the overlapped phase — residual adjoints on wave 0 beside the factorisation on wave 1 —, and
slots 2 / 3 hold only a factorisation redone after a missed precision guess)"""
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
# lab build with -DCMPC_RIC_SUBSTAMP (CMPC_LIB_PATH): phases of the fp64 factor sweep, inside slot 2
SUB = {9: "  factor: T = P[A|B]", 10: "  factor: G = [A|B]'T", 11: "  factor: Hvv, chol, K"}
if os.environ.get("CMPC_SUB_MODE") == "2":  # lab build -DCMPC_RIC_SUBSTAMP=2: sweep bodies (without the stage advance)
    SUB = {9: "  solve: backward bodies", 10: "  solve: forward bodies", 11: "  residual adjoint bodies"}


def report(st, iters, label, ms):
    a = st.astype(np.float64)
    print(f"{label}: {ms:.3f} ms per call; iterations {iters.tolist()}; dd iterations {a[:, 12].astype(int).tolist()}; "
          f"refinement steps {a[:, 13].astype(int).tolist()}")
    tot = a[:, [k for k in NAMES]].sum(1)
    for k, nm in NAMES.items():
        print(f"  {nm:34s} " + " ".join(f"{v / 1e6:8.3f}M" for v in a[:, k]) + "   clk per agent")
        if k == 2 and a[:, 9:12].any() and (ONE_WAVE or not label.startswith("lpv")):
            for k2, nm2 in SUB.items():
                print(f"  {nm2:34s} " + " ".join(f"{v / 1e6:8.3f}M" for v in a[:, k2]) + "   clk per agent")
    if not ONE_WAVE and label.startswith("lpv") and a[:, 9:12].any():  # latency mode: each role's own clocks
        for k2, nm2 in ((9, "  role: residual adjoints (wave 0)"), (10, "  role: factorisation (wave 1)"),
                        (11, "  role: piped backward pass (wave 2)")):
            print(f"  {nm2:34s} " + " ".join(f"{v / 1e6:8.3f}M" for v in a[:, k2]) + "   clk per agent")
    it = np.maximum(a[:, SLOTS - 1], 1)
    print(f"  {'total':34s} " + " ".join(f"{v / 1e6:8.3f}M" for v in tot) +
          "   | per iteration " + " ".join(f"{v / 1e3:.0f}k" for v in tot / it))


ONE_WAVE = "--one-wave" in sys.argv
if ONE_WAVE:
    sys.argv.remove("--one-wave")


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
        flags = L.CMPC_FLAG_RICCATI | (L.CMPC_FLAG_ONE_WAVE if ONE_WAVE else 0)
        if ONE_WAVE:
            bp.opts = L.opts(flags=flags)
            bp.solve(*args)
            t0 = time.perf_counter()
            res = bp.solve(*args)
            ms = (time.perf_counter() - t0) * 1e3
        bp.opts = L.opts(flags=flags, stamps=st.data_ptr())
        res = bp.solve(*args)
        torch.cuda.synchronize()
        mode = "one wave per agent" if ONE_WAVE else "latency mode, four waves per agent (slot 0: residuals | factor)"
        report(st.cpu().numpy(), res["iters"], f"{name} rows {rows} ({len(cs)} agents, status {res['status'].tolist()}; "
               f"{mode})", ms)


def cfg5(agents):
    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    R = DIRounds(S.make_di(agents, 50, 2, 3))
    R.build()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    R.solve()
    ev[1].record()
    st = torch.zeros((agents, SLOTS), dtype=torch.int64, device="cuda")
    plain = R.opts
    R.opts = L.opts(flags=0, stamps=st.data_ptr())
    ev[2].record()
    R.solve()
    ev[3].record()
    torch.cuda.synchronize()
    R.opts = plain
    a = st.cpu().numpy().astype(np.float64)
    it = a[:, SLOTS - 1]
    print(f"cfg5 {agents} agents: kernel {ev[0].elapsed_time(ev[1]):.2f} ms (stamped {ev[2].elapsed_time(ev[3]):.2f} ms); "
          f"iterations mean {it.mean():.2f} max {int(it.max())}; dd iterations {int(a[:, 12].sum())}")
    tot = a[:, list(NAMES)].sum(1)
    for k, nm in NAMES.items():
        print(f"  {nm:34s} {a[:, k].sum() / it.sum() / 1e3:9.1f}k clk/iter  {a[:, k].sum() / tot.sum() * 100:5.1f} %")
        if k == 2 and a[:, 9:12].any():
            for k2, nm2 in SUB.items():
                print(f"  {nm2:34s} {a[:, k2].sum() / it.sum() / 1e3:9.1f}k clk/iter")
    print(f"  {'total':34s} {tot.sum() / it.sum() / 1e3:9.1f}k clk/iter; slowest agent {tot.max() / 1e6:.2f}M clk")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--cfg5":
        cfg5(int(sys.argv[2]) if len(sys.argv) > 2 else 8192)
    else:
        lpv(sys.argv[1] if len(sys.argv) > 1 else "lpv_n125_a3")
