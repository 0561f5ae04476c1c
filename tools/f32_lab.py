"""CPU laboratory for the cfg5 fp32 path (test infrastructure; never on the product path).

Solves BASELINE cfg5 populations (3-D double integrator nx=6 nu=3, N=50, nb=2) with variants of
the C restatement oracle/cmpc_oracle.c compiled into /tmp/f32_lab:
  * "f32": the whole restatement in single precision (-Ddouble=float: every array, every
    operation), i.e. what a pure fp32 kernel computes;
  * "f64": the reference build,
and compares statuses, iterations and z against the fp64 Riccati solve (double-double near the
solution, newton 3) at tol 1e-9.

  python tools/f32_lab.py [--agents 1024] [--rounds 1] VARIANT...
  VARIANT = name:newton:tol[:-DFLAG...]   e.g. f32:1:1e-5:-DMU_FACTOR=10
"""
import argparse
import ctypes as ct
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]
OUT = "/tmp/f32_lab"

from oracle import cmpc_oracle as CO  # noqa: E402
from oracle import synth  # noqa: E402


def build(flags, f32):
    os.makedirs(OUT, exist_ok=True)
    tag = ("f32_" if f32 else "f64_") + "_".join(f.strip("-D").replace("=", "") for f in flags)
    so = os.path.join(OUT, f"lib_{tag}.so")
    src = os.path.join(ROOT, "oracle", "cmpc_oracle.c")
    if f32:   # system headers first (their long double must stay), then every double of the oracle -> float
        src = os.path.join(OUT, "f32_wrap.c")
        with open(src, "w") as f:
            f.write("#include <math.h>\n#include <stdio.h>\n#include <stdlib.h>\n#include <string.h>\n#include <omp.h>\n"
                    f"#define double float\n#include \"{os.path.join(ROOT, 'oracle', 'cmpc_oracle.c')}\"\n")
    cmd = ["gcc", "-O2", "-fPIC", "-fopenmp", "-std=c99", "-shared", "-o", so, src, "-lm"] + list(flags)
    subprocess.run(cmd, check=True)
    return ct.CDLL(so)


def solve(lib, p, f32, tol, newton, refine=0, max_iter=80):
    dt, cp = (np.float32, ct.c_float) if f32 else (np.float64, ct.c_double)
    keep, args = [], []

    def arr(a, t=dt, c=cp):
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
    z = np.zeros((nb, CO.nz_of(p)), dt)
    kkt = np.zeros(nb, dt)
    it = np.zeros(nb, np.int32)
    st = np.zeros(nb, np.int32)
    lib.cmpc_oracle_solve_ex.restype = ct.c_int
    rc = lib.cmpc_oracle_solve_ex(ct.c_int(p["nx"]), ct.c_int(p["nu"]), ct.c_int(p["N"]), ct.c_int(p["ns"]),
                                  ct.c_int(p["mc"]), ct.c_int(nb), *args, cp(tol), ct.c_int(max_iter), ct.c_int(8),
                                  ct.c_int(newton), ct.c_int(refine), None, z.ctypes.data_as(ct.POINTER(cp)),
                                  kkt.ctypes.data_as(ct.POINTER(cp)), it.ctypes.data_as(ct.POINTER(ct.c_int)),
                                  st.ctypes.data_as(ct.POINTER(ct.c_int)))
    assert rc == 0
    return z.astype(np.float64), kkt.astype(np.float64), it, st


def population(n, rounds):
    from cmpc import scenarios as S

    sc = S.make_di(n, 50, 2, 3)
    x0, up, traj = sc.x0.copy(), sc.u_prev.copy(), sc.traj.copy()
    ne, N = sc.shared["nx"] + sc.shared["ns"], sc.N
    out = []
    for r in range(rounds):
        P = synth.structured(sc.shared, sc.params, sc.A, sc.B, x0, up, sc.lane, sc.nbr, traj, np.arange(n))
        z, kkt, it, st = CO.solve_batch(P, nthreads=8, newton=3)   # fp64 Riccati with double-double (cfg5's fp64 method)
        out.append((P, z, st))
        x0 = z[:, ne:ne + sc.shared["nx"]].copy()
        up = z[:, ne * (N + 1):ne * (N + 1) + sc.shared["nu"]].copy()
        traj = np.stack([z[:, [k * ne for k in range(N + 1)]], z[:, [k * ne + 1 for k in range(N + 1)]]], -1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import pickle  # (a cache of this script's own populations, under /tmp)

    cache = os.path.join(OUT, f"pop_{a.agents}_{a.rounds}.pkl")
    if os.path.exists(cache):
        with open(cache, "rb") as f:
            pops = pickle.load(f)
    else:
        pops = population(a.agents, a.rounds)
        os.makedirs(OUT, exist_ok=True)
        with open(cache, "wb") as f:
            pickle.dump(pops, f)
    for v in a.variants:
        name, newton, tol, *flags = v.split(":")
        refine = 0
        fl = []
        for f in flags:
            if f.startswith("refine="):
                refine = int(f.split("=")[1])
            else:
                fl.append(f)
        f32 = name == "f32"
        lib = build(fl, f32)
        sts, its, errs, kks = [], [], [], []
        for P, zr, str_ in pops:
            z, kkt, it, st = solve(lib, P, f32, float(tol), int(newton), refine)
            kks.append(kkt)
            err = np.abs(z - zr) / np.maximum(1.0, np.abs(zr))
            sts.append(st)
            its.append(it)
            errs.append(err.max(axis=1))
        st, it, err, kk = np.concatenate(sts), np.concatenate(its), np.concatenate(errs), np.concatenate(kks)
        u, c = np.unique(st, return_counts=True)
        ok = st == 1
        e1 = err[ok].max() if ok.any() else np.nan
        cnt = ""
        try:
            f32i = ct.c_long.in_dll(lib, "cmpc_f32_iters").value
            f64i = ct.c_long.in_dll(lib, "cmpc_f64_iters").value
            f64a = ct.c_long.in_dll(lib, "cmpc_f64_agents").value
            cnt = f" | fp32 iters {f32i} fp64 iters {f64i} switched agents {f64a}"
            cnt += f" restarts {ct.c_long.in_dll(lib, 'cmpc_f32_restarts').value}"
        except ValueError:
            pass
        try:
            cnt += f" | dd iters {ct.c_long.in_dll(lib, 'cmpc_dd_iters').value}"
        except ValueError:
            pass
        print(f"{v}: status {dict(zip(u.tolist(), c.tolist()))} solved {np.mean(st == 1):.4f} iters mean {it.mean():.1f} "
              f"max {it.max()} | rel err max {err.max():.2e} p99 {np.quantile(err, 0.99):.2e} "
              f"median {np.median(err):.2e} | solved-only max {e1:.2e}{cnt} | max kkt {kk.max():.2e} "
              f"status-2 kkt {np.sort(kk[st == 2])[::-1][:8].tolist()} (agents {np.nonzero(st == 2)[0].tolist()[:8]})",
              flush=True)


if __name__ == "__main__":
    main()
