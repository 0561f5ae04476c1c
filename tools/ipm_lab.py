"""CPU laboratory for interior-point variants (test infrastructure; never on the product path).

Builds a problem set — consecutive cfg3 rounds of the synthetic double-integrator population
(oracle builder + the C restatement + the round advance of cmpc_di_advance_dev, i.e. what
DIRounds does on the GPU) and every captured reference QP (tests/golden) — and solves it with
a variant of oracle/cmpc_oracle.c compiled with extra -D flags, reporting IPM iteration
statistics (the kernel time follows the slowest agent of a round) and accuracy against the
certified optima.

  python tools/ipm_lab.py gen [rounds]            # cache the round problems in /tmp/ipm_lab
  python tools/ipm_lab.py run "-DFLAG=..." ...     # one line of statistics per flag set
"""
import ctypes as ct
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd"), os.path.join(ROOT, "tests")]
CACHE = "/tmp/ipm_lab"

from oracle import cmpc_oracle as CO  # noqa: E402
from oracle import synth  # noqa: E402


def gen(rounds):
    from cmpc import scenarios as S

    os.makedirs(CACHE, exist_ok=True)
    sc = S.make_di(1024, 30, 2, 2)
    x0, up, traj = sc.x0.copy(), sc.u_prev.copy(), sc.traj.copy()
    ne, N = sc.shared["nx"] + sc.shared["ns"], sc.N
    for r in range(rounds):
        P = synth.structured(sc.shared, sc.params, sc.A, sc.B, x0, up, sc.lane, sc.nbr, traj, np.arange(1024))
        z, kkt, it, st = CO.solve_batch(P, nthreads=8)
        np.savez(os.path.join(CACHE, f"round{r}.npz"), **{k: np.asarray(v) for k, v in P.items()})
        x0 = z[:, ne:ne + sc.shared["nx"]].copy()
        up = z[:, ne * (N + 1):ne * (N + 1) + sc.shared["nu"]].copy()
        traj = np.stack([z[:, [k * ne for k in range(N + 1)]], z[:, [k * ne + 1 for k in range(N + 1)]]], -1)
        print(f"round {r}: iters mean {it.mean():.2f} max {it.max()} status {np.unique(st, return_counts=True)}",
              flush=True)


def load_rounds():
    out = []
    r = 0
    while os.path.exists(os.path.join(CACHE, f"round{r}.npz")):
        d = np.load(os.path.join(CACHE, f"round{r}.npz"))
        p = {k: d[k] for k in d.files}
        for k in ("nx", "nu", "N", "ns", "mc"):
            p[k] = int(p[k])
        out.append(p)
        r += 1
    return out


def load_lpv():
    from conftest import LPV_CASES, lpv_qps
    from oracle import lpv_ref as L

    tr = L.Track.build("Highway")
    g = L.paper_gains()
    cases = []
    for nm in LPV_CASES:
        probs, zs = [], []
        for j, c in lpv_qps(nm):
            lim = L.scaled_car_limits(c["vx_ref"])
            qp = L.assemble(c["x0"], c["x_last"], c["u_last"], c["x_agents"], c["pose"], c["u_old"], c["N"],
                            c["dt"], tr, L.SCALED_CAR_MODEL, lim, g)
            probs.append(L.structured(qp, c["x0"], c["u_old"], c["N"], lim, g))
            zs.append(c["z"])
        cases.append((nm, L.stack(probs), np.array(zs)))
    return cases


def variant(flags):
    tag = "".join(ch if ch.isalnum() else "_" for ch in flags) or "base"
    so = f"/tmp/ipm_lab_{tag}.so"
    src = os.path.join(ROOT, "oracle", "cmpc_oracle.c")
    subprocess.run(f"gcc -O2 -fPIC -shared -fopenmp {flags} -o {so} {src} -lm", shell=True, check=True)
    lib = ct.CDLL(so)
    lib.cmpc_oracle_solve.restype = ct.c_int
    lib.cmpc_oracle_solve_ex.restype = ct.c_int
    return lib


def run(flag_sets):
    rounds = load_rounds()
    lpv = load_lpv()
    base = None
    for flags in flag_sets:
        CO._LIB = variant(flags)
        mx, mean, bad, zs = [], [], 0, []
        for p in rounds:
            z, kkt, it, st = CO.solve_batch(p, nthreads=8)
            mx.append(int(it.max()))
            mean.append(float(it.mean()))
            bad += int((~np.isin(st, (1, 2))).sum())
            zs.append(z)
        dz = None if base is None else max(float(np.abs(a - b).max()) for a, b in zip(zs, base))
        if base is None:
            base = zs
        lerr, lit, lbad = 0.0, [], 0
        for nm, P, zref in lpv:
            z, kkt, it, st = CO.solve_batch(P, nthreads=8)
            lerr = max(lerr, float(np.abs(z - zref).max()))
            lit += it.tolist()
            lbad += int((st != 1).sum())
        gz = ct.c_long.in_dll(CO._LIB, "cmpc_gz_solves").value if "GONDZIO" in flags else 0
        print(f"[{flags or 'base'}] corrector solves {gz} DI rounds: sum(max it) {sum(mx)} max {max(mx)} mean {np.mean(mean):.2f} "
              f"unsolved {bad} |dz vs base| {dz} | LPV: max err {lerr:.1e} iters sum {sum(lit)} max {max(lit)} "
              f"not-solved {lbad}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "gen":
        gen(int(sys.argv[2]) if len(sys.argv) > 2 else 40)
    else:
        run(sys.argv[2:] or [""])
