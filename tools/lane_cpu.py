"""Host check of the lane-per-agent solver body: builds tools/lane_cpu.cpp (the code of
mpc_lane_kernel, run per agent on the CPU) and compares it with the C restatement on cfg5
problems (oracle/cmpc_oracle.c: Riccati newton 1 for the fp64 body).

  python tools/lane_cpu.py [--agents 256] [--rounds 1] [--mixed]
"""
import argparse
import ctypes as ct
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd"), os.path.join(ROOT, "tools")]
SO = "/tmp/lane_cpu/lane_cpu.so"


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-host-only", "-x", "hip",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "colaborativempc-_amd", "csrc"),
                    os.path.join(ROOT, "tools", "lane_cpu.cpp"), "-o", SO], check=True)
    return ct.CDLL(SO)


def solve(lib, p, tol=1e-9, max_iter=60, mixed=False):
    from oracle import cmpc_oracle as CO

    keep, args = [], []

    def arr(a, t=np.float64, c=ct.c_double):
        a = np.ascontiguousarray(a, dtype=t)
        keep.append(a)
        return a.ctypes.data_as(ct.POINTER(c))

    for k in ("Q", "R", "dR", "Qs", "u_ub", "u_lb"):
        args.append(arr(p[k]))
    for k in ("row_slack", "row_sign"):
        args.append(arr(p[k], np.int32, ct.c_int))
    for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h"):
        args.append(arr(p[k]))
    nb = p["A"].shape[0]
    z = np.zeros((nb, CO.nz_of(p)))
    kkt = np.zeros(nb)
    it = np.zeros(nb, np.int32)
    st = np.zeros(nb, np.int32)
    rc = lib.lane_cpu_solve(ct.c_int(p["nx"]), ct.c_int(p["nu"]), ct.c_int(p["N"]), ct.c_int(p["ns"]), ct.c_int(p["mc"]),
                            ct.c_int(nb), *args, ct.c_double(tol), ct.c_int(max_iter), ct.c_int(int(mixed)),
                            z.ctypes.data_as(ct.POINTER(ct.c_double)), kkt.ctypes.data_as(ct.POINTER(ct.c_double)),
                            it.ctypes.data_as(ct.POINTER(ct.c_int)), st.ctypes.data_as(ct.POINTER(ct.c_int)))
    assert rc == 0
    return z, kkt, it, st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--mixed", action="store_true")
    ap.add_argument("--tol", type=float, default=None)
    a = ap.parse_args()
    import f32_lab
    from oracle import cmpc_oracle as CO

    lib = build()
    tol = a.tol or (1e-6 if a.mixed else 1e-9)
    for P, zr, sr in f32_lab.population(a.agents, a.rounds):
        z, kkt, it, st = solve(lib, P, tol, mixed=a.mixed)
        zc, kc, ic, sc = CO.solve_batch(P, tol, nthreads=8, newton=1)
        d = np.abs(z - zc).max(1)
        e = (np.abs(z - zr) / np.maximum(1.0, np.abs(zr))).max(1)
        print(f"lane body ({'mixed' if a.mixed else 'fp64'}): status {dict(zip(*np.unique(st, return_counts=True)))} "
              f"iters {it.mean():.2f} | oracle newton 1: status {dict(zip(*np.unique(sc, return_counts=True)))} "
              f"iters {ic.mean():.2f} | status agree {np.mean(st == sc):.3f}, iters agree {np.mean(it == ic):.3f}, "
              f"max |dz| {d.max():.2e} | vs dd Riccati rel err max {e.max():.2e}")
        bad = np.flatnonzero((st != sc) | (it != ic))[:5]
        for b in bad:
            print(f"   agent {b}: lane st {st[b]} it {it[b]} kkt {kkt[b]:.2e} | oracle st {sc[b]} it {ic[b]} kkt {kc[b]:.2e}")


if __name__ == "__main__":
    main()
