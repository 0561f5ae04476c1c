"""Fixture for the polish tests (test infrastructure): agent-QPs of the reference's agent model whose
condensed factorisation breaks down at the rounding floor.

bench.py's lpv_rounds population (341 jittered copies of the reference's 3-agent N = 30 Highway run,
tools/lpv_lab.py) is driven through closed-loop rounds on the CPU — the numpy builder
(oracle/lpv_ref.py) and the C restatement with the rescue policy — until round ROUND; the agents of
that round that end at status 2 without polish and at status 1 with it (a factorisation breakdown at
the rounding floor, CMPC_FLAG_POLISH) are saved, with a few that converge normally, as structured
problems in tests/golden/polish_lpv.npz.

  python oracle/gen_polish_fixture.py            # (about a minute, 8 threads)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "colaborativempc-_amd")]

ROUND, KEEP_FLOOR, KEEP_PLAIN = 4, 6, 2


def main():
    import lpv_lab
    from oracle import cmpc_oracle as CO
    from oracle import lpv_ref as L

    pop = lpv_lab.population()
    track = L.Track.build("Highway")
    gains = L.paper_gains()
    lim = L.scaled_car_limits(pop["vx_ref"])
    N = pop["N"]
    x0, x_last, u_last, u_old, traj = (pop[k].copy() for k in ("x0", "x_last", "u_last", "u_old", "traj"))
    base = 12 * (N + 1)
    for r in range(ROUND + 1):
        P = lpv_lab.build_round(pop, x0, x_last, u_last, u_old, traj, track, gains, lim)
        z, kkt, it, st = CO.solve_batch_rescue(P, nthreads=8)
        if r == ROUND:
            break
        xp = z[:, :base].reshape(-1, N + 1, 12)[:, :, :9]
        up = z[:, base: base + 2 * N].reshape(-1, N, 2)
        x0, x_last, u_last, u_old = xp[:, 1].copy(), xp[:, 1:].copy(), up.copy(), up[:, 0].copy()
        traj = xp[:, :, 7:9].copy()
    from cmpc.solver import plan  # the polish kernel's active-set capacity for this shape (host only)

    amax = plan(P, 1, rescue=True, polish=True)["polish_max_active"]
    zp, kp, ip, sp = CO.solve_batch_rescue(P, nthreads=8, polish=True, polish_amax=amax)
    floor = np.flatnonzero((st == 2) & (sp == 1))[:KEEP_FLOOR]
    plain = np.flatnonzero((st == 1) & (sp == 1))[:KEEP_PLAIN]
    sel = np.concatenate([floor, plain])
    out = {k: (v[sel] if isinstance(v, np.ndarray) and v.ndim and v.shape[0] == len(st) else v)
           for k, v in P.items()}
    out["status_plain"], out["status_polish"] = st[sel], sp[sel]
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "polish_lpv.npz"), **{k: np.asarray(v) for k, v in out.items()})
    print("saved agents", sel.tolist(), "status", st[sel].tolist(), "->", sp[sel].tolist())


if __name__ == "__main__":
    main()
