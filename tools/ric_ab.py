"""Diagnostic A/B of the Riccati kernel (mpc_riccati.hip) across two builds of the library.

  CMPC_LIB_PATH=<old .so> python tools/ric_ab.py dump gpurun_out/a.npz
  python tools/ric_ab.py dump gpurun_out/b.npz
  python tools/ric_ab.py cmp gpurun_out/a.npz gpurun_out/b.npz

dump: the reference's N = 125 captured QPs (tests/golden/lpv_n125_a3.npz, both steps), two
rounds of the BASELINE cfg5 population (8192 agents, N = 50, nx 6, nu 3) and one of the DI
nx 4 family forced onto the Riccati kernel; z, iterations, status and kernel times.
cmp: bit equality of z / iterations / status per case, and the time ratio."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd"), os.path.join(ROOT, "tests")]


def dump(out):
    import torch

    import cmpc
    from cmpc import _lib as L
    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds
    from conftest import lpv_qps
    from oracle import lpv_ref as R

    rec = {}
    ctx = cmpc.Context(0)
    g = R.paper_gains()
    tr = R.Track.build("Highway")
    groups = {}
    for j, c in lpv_qps("lpv_n125_a3"):
        groups.setdefault(c["x_last"].shape[0], []).append(c)
    for gi, (rows, cs) in enumerate(groups.items()):
        bp = cmpc.PlannerLPVBatch(g["Q"], g["Qs"], g["R"], g["dR"], cs[0]["N"], cs[0]["dt"], tr, g["wq"],
                                  R.SCALED_CAR_MODEL, R.scaled_car_limits(cs[0]["vx_ref"]), ctx=ctx, riccati=True)
        xa = np.stack([c["x_agents"] for c in cs])
        args = (np.stack([c["x0"] for c in cs]), np.stack([c["x_last"] for c in cs]),
                np.stack([c["u_last"] for c in cs]), np.stack([c["u_old"] for c in cs]),
                xa if xa.shape[2] else None, np.stack([c["pose"] for c in cs]))
        bp.solve(*args)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            res = bp.solve(*args)
            ts.append((time.perf_counter() - t0) * 1e3)
        key = f"n125_step{gi}"
        rec[key + "_z"] = res["z"]
        rec[key + "_it"] = np.asarray(res["iters"])
        rec[key + "_st"] = np.asarray(res["status"])
        rec[key + "_ms"] = np.array(min(ts))
    for name, (n, N, nb, dim, rounds) in {"cfg5": (8192, 50, 2, 3, 2), "di4": (1024, 30, 2, 2, 1)}.items():
        Rr = DIRounds(S.make_di(n, N, nb, dim))
        Rr.opts = L.opts(flags=L.CMPC_FLAG_RICCATI)
        for rnd in range(rounds):
            Rr.build()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            Rr.solve()
            ev[1].record()
            torch.cuda.synchronize()
            key = f"{name}_r{rnd}"
            rec[key + "_z"] = Rr.z.cpu().numpy()
            rec[key + "_it"] = Rr.iters.cpu().numpy()
            rec[key + "_st"] = Rr.status.cpu().numpy()
            rec[key + "_ms"] = np.array(ev[0].elapsed_time(ev[1]))
            Rr.advance()
            Rr.exchange()
    np.savez(out, **rec)
    for k in sorted(rec):
        if k.endswith("_ms"):
            print(f"{k[:-3]:14s} {float(rec[k]):9.3f} ms  iters max {int(rec[k[:-3] + '_it'].max())}"
                  f"  status {np.unique(rec[k[:-3] + '_st'], return_counts=True)}")


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in sorted(A.files):
        if not k.endswith("_z"):
            continue
        c = k[:-2]
        same = (np.array_equal(A[k].view(np.uint64), B[k].view(np.uint64)) and np.array_equal(A[c + "_it"], B[c + "_it"])
                and np.array_equal(A[c + "_st"], B[c + "_st"]))
        ok &= same
        d = float(np.nanmax(np.abs(A[k] - B[k]))) if A[k].size else 0.0
        print(f"{c:14s} bit-equal {same}  max|dz| {d:.2e}  ms {float(A[c + '_ms']):9.3f} -> {float(B[c + '_ms']):9.3f}"
              f"  ({float(A[c + '_ms']) / max(float(B[c + '_ms']), 1e-9):.2f}x)")
    print("ALL BIT-EQUAL" if ok else "DIFFERENT")


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
