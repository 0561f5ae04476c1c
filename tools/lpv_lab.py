"""CPU laboratory for the reference-model LPV rounds (test infrastructure; never on the product path).

The population of bench.py's `lpv_rounds` line (341 copies of the reference's 3-agent Highway
scenario at lpv_n30_a3 step 0, initial v_x jittered by U[0.98, 1.02]; neighbours = the other two
agents of the copy) is driven through consecutive consensus rounds on the CPU: the numpy builder
(oracle/lpv_ref.py: planes, weights, _EstimateABC, rows, costs) and the C restatement of the
solver (oracle/cmpc_oracle.c, CMPC_FLAG_RESCUE policy), advanced with the reference's loop
semantics (LPV_HP_N_main.py:96-117).  Each round's structured problems are cached; `run`
re-solves the cached rounds with variants of cmpc_oracle.c compiled with extra -D flags and
reports what the kernel time follows (the slowest agent of a round) and the failures.

  python tools/lpv_lab.py gen [rounds]          # cache rounds in /tmp/lpv_lab
  python tools/lpv_lab.py run "-DFLAG=..." ...   # one line of statistics per flag set
"""
import ctypes as ct
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd"), os.path.join(ROOT, "tests")]
CACHE = "/tmp/lpv_lab"

from oracle import cmpc_oracle as CO  # noqa: E402
from oracle import lpv_ref as L  # noqa: E402


def population(replicas=341, seed=5):
    """bench.py lpv_rounds population (host arrays)."""
    d = np.load(os.path.join(ROOT, "tests", "golden", "lpv_n30_a3.npz"), allow_pickle=False)
    N, dt = int(d["N"]), float(d["dt"])
    sel = sorted([j for j in range(len(d["step"])) if d["step"][j] == 0], key=lambda j: d["agent"][j])
    x0 = np.tile(d["x0"][sel], (replicas, 1))
    x0[:, 0] *= np.repeat(1.0 + 0.02 * np.random.default_rng(seed).uniform(-1, 1, replicas), 3)
    x_last = np.tile(np.stack([d[f"x_last_{j}"] for j in sel]), (replicas, 1, 1))
    u_last = np.tile(np.stack([d[f"u_last_{j}"] for j in sel]), (replicas, 1, 1))
    u_old = np.tile(d["u_old"][sel], (replicas, 1))
    traj = np.tile(d["pose"][sel], (replicas, 1, 1))
    g3 = np.arange(3 * replicas) // 3 * 3
    nbr = np.sort(np.stack([g3 + (np.arange(3 * replicas) + 1) % 3, g3 + (np.arange(3 * replicas) + 2) % 3], 1), 1)
    return dict(N=N, dt=dt, vx_ref=float(d["vx_ref"]), x0=x0, x_last=x_last, u_last=u_last, u_old=u_old,
                traj=traj, nbr=nbr)


def build_round(pop, x0, x_last, u_last, u_old, traj, track, gains, lim):
    """Structured problems of every agent (the GPU builder's arithmetic, numpy form)."""
    N, dt, nbr = pop["N"], pop["dt"], pop["nbr"]
    probs = []
    for b in range(x0.shape[0]):
        xa = np.swapaxes(traj[nbr[b]], 0, 1)                 # (N+1, nb, 2)
        pose = traj[b]
        planes = L.compute_hyperplane(xa, pose, N, keep_sign=True)
        weights, _ = L.compute_weights(pose, xa, lim["min_dist"])
        A, B, ey = L.estimate_abc(x_last[b], u_last[b], N, dt, L.SCALED_CAR_MODEL, track)
        qp = L.LPVQP(None, None, None, None, None, planes, A, B, ey, weights)
        probs.append(L.structured(qp, x0[b], u_old[b], N, lim, gains))
    return L.stack(probs)


def gen(rounds):
    os.makedirs(CACHE, exist_ok=True)
    pop = population()
    track = L.Track.build("Highway")
    gains = L.paper_gains()
    lim = L.scaled_car_limits(pop["vx_ref"])
    N = pop["N"]
    x0, x_last, u_last, u_old, traj = (pop[k].copy() for k in ("x0", "x_last", "u_last", "u_old", "traj"))
    base = 12 * (N + 1)
    for r in range(rounds):
        P = build_round(pop, x0, x_last, u_last, u_old, traj, track, gains, lim)
        z, kkt, it, st = CO.solve_batch_rescue(P, nthreads=8)
        np.savez(os.path.join(CACHE, f"round{r}.npz"), **{k: np.asarray(v) for k, v in P.items()})
        xp = z[:, :base].reshape(-1, N + 1, 12)[:, :, :9]
        up = z[:, base: base + 2 * N].reshape(-1, N, 2)
        x0, x_last, u_last, u_old = xp[:, 1].copy(), xp[:, 1:].copy(), up.copy(), up[:, 0].copy()
        traj = xp[:, :, 7:9].copy()
        print(f"round {r}: iters mean {it.mean():.2f} max {it.max()} status "
              f"{dict(zip(*[a.tolist() for a in np.unique(st, return_counts=True)]))} max kkt {kkt.max():.1e}",
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


def variant(flags):
    tag = "".join(ch if ch.isalnum() else "_" for ch in flags) or "base"
    so = f"/tmp/lpv_lab_{tag}.so"
    src = os.path.join(ROOT, "oracle", "cmpc_oracle.c")
    subprocess.run(f"gcc -O2 -fPIC -shared -fopenmp {flags} -o {so} {src} -lm", shell=True, check=True)
    lib = ct.CDLL(so)
    lib.cmpc_oracle_solve.restype = ct.c_int
    lib.cmpc_oracle_solve_ex.restype = ct.c_int
    return lib


def run(flag_sets, rescue=True, newton=0):
    rounds = load_rounds()
    base = None
    for flags in flag_sets:
        CO._LIB = variant(flags)
        mx, mean, zs, cnt = [], [], [], {}
        for p in rounds:
            if rescue and newton == 0:
                z, kkt, it, st = CO.solve_batch_rescue(p, nthreads=8)
            else:
                z, kkt, it, st = CO.solve_batch(p, nthreads=8, newton=newton)
            z0, _, _, st0 = (z, kkt, it, st) if not rescue else CO.solve_batch(p, nthreads=8, newton=newton)
            mx.append(int(it.max()))
            mean.append(float(it.mean()))
            for k, v in zip(*np.unique(st0, return_counts=True)):
                cnt[f"pre{int(k)}"] = cnt.get(f"pre{int(k)}", 0) + int(v)
            for k, v in zip(*np.unique(st, return_counts=True)):
                cnt[int(k)] = cnt.get(int(k), 0) + int(v)
            zs.append(z)
        dz = None if base is None else max(float(np.abs(a - b).max()) for a, b in zip(zs, base))
        if base is None:
            base = zs
        print(f"[{flags or 'base'}] rounds {len(rounds)}: sum(max it) {sum(mx)} max {max(mx)} "
              f"mean {np.mean(mean):.2f} status {cnt} |dz vs first| {dz}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "gen":
        gen(int(sys.argv[2]) if len(sys.argv) > 2 else 20)
    else:
        run(sys.argv[2:] or [""])
