"""ORACLE fixture generator (runs only in the build container, where /root/reference exists):
golden OCD coupling-dual rounds computed by the reference's OWN functions.

The dual update of the reference's NL-DMPC loop (planner/scripts/NL_EU_N_main.py:127-138) is

    cost[i, j, k-1] = eval_constraintEU(agents[k, i, :], agents[k, j, :], dth)   (i < j, k = 1..N)
    lambdas += get_alpha() * cost

with eval_constraintEU and get_alpha imported from plan_lib.config.NL (config/NL/config.py:5-8,
19-23; a data-free module, importable here), and the convergence test of :143-149 is numpy's
allclose(x_old[i], x_pred[i], atol=0.01).  This script imports those functions from
/root/reference/planner/lib (read only, PYTHONDONTWRITEBYTECODE) and applies them to seeded
trajectories: several consecutive rounds of 3 and 5 agents at N = 20 (the NL config's horizon,
config_files/config_NL.py) with the reference's dth = 0.25, positions drifting like a platoon so
that some pairs come closer than dth.  The loop around the two calls is the script's own
(NL_EU_N_main.py:130-138), restated literally.  Inputs and outputs go to tests/golden/ocd_rounds.npz;
nothing from the reference is copied.

  PYTHONDONTWRITEBYTECODE=1 python oracle/gen_ocd_fixtures.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_LIB = "/root/reference/planner/lib"


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF_LIB)
    from plan_lib.config.NL.config import eval_constraintEU, get_alpha  # the reference's own functions

    out = {}
    rng = np.random.default_rng(20240611)
    for case, (n, N, rounds) in enumerate(((3, 20, 4), (5, 20, 3))):
        dth = 0.25
        # platoon on a lane pair, spacing ~0.3 with jitter: some pairs inside dth
        base = np.stack([0.3 * np.arange(n) + rng.uniform(-0.1, 0.1, n), 0.5 * (np.arange(n) % 2)], 1)
        lam = np.zeros((n, n, N))
        out[f"c{case}_n"], out[f"c{case}_N"], out[f"c{case}_dth"] = np.array(n), np.array(N), np.array(dth)
        out[f"c{case}_rounds"] = np.array(rounds)
        x_old = None
        for r in range(rounds):
            v = np.stack([1.0 + rng.uniform(-0.05, 0.05, n), rng.uniform(-0.05, 0.05, n)], 1)
            agents = base[None] + 0.025 * np.arange(N + 1)[:, None, None] * v[None] + \
                rng.normal(0, 0.01, (N + 1, n, 2))                        # (N+1, n, 2) as in :125
            out[f"c{case}_r{r}_agents"] = agents
            out[f"c{case}_r{r}_lam_in"] = lam.copy()
            cost = np.zeros((n, n, N))
            for k in range(1, N + 1):                                      # :130-135
                for i in range(0, n):
                    for j in range(0, n):
                        if (i != j) and i < j:
                            cost[i, j, k - 1] = eval_constraintEU(agents[k, i, :], agents[k, j, :], dth)
            alpha = get_alpha()                                            # :137
            lam = lam + alpha * cost                                       # :138 (lambdas += ...)
            out[f"c{case}_r{r}_lam_out"] = lam.copy()
            # states for the convergence test (:143-149): predictions (n, N+1, 9), some agents moved
            x_pred = rng.normal(0, 1, (n, N + 1, 9))
            if x_old is not None:
                x_pred[::2] = x_old[::2] + rng.uniform(-0.009, 0.009, x_old[::2].shape)
                out[f"c{case}_r{r}_close"] = np.array([np.allclose(x_old[i], x_pred[i], atol=0.01) for i in range(n)])
                out[f"c{case}_r{r}_x_old"] = x_old
                out[f"c{case}_r{r}_x_pred"] = x_pred
            x_old = x_pred
    path = os.path.join(ROOT, "tests", "golden", "ocd_rounds.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


if __name__ == "__main__":
    main()
