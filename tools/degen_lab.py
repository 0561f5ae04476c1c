"""CPU laboratory: how far the polish's degenerate-row test reaches at a loose tolerance
(test infrastructure; never on the product path).

ADVICE (round 5) pointed out that the test "a converged solve with some row at min(t, lambda) >
kPolishDegenerate = 1e-9 is polished" does not scale with tol: at tol 1e-6 an ordinary converged row
could trip it, and many status-1 agents would run the polish.  This re-solves the cached reference-
model LPV rounds of tools/lpv_lab.py (`python tools/lpv_lab.py gen` first) with the C restatement
(oracle/cmpc_oracle.c built with -DLAB_DEGEN_COUNT, the product's rescue + polish policy) at several
tolerances and counts the converged solves that the test flags, and those whose polished point
replaced the endpoint.

  python tools/degen_lab.py [tol ...]
  DEGEN_FLAGS='-DPOLISH_DEGENERATE=(1e-9*sqrt(tol/1e-9))' python tools/degen_lab.py   # a tol-scaled test
"""
import ctypes as ct
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]

import lpv_lab  # noqa: E402
from oracle import cmpc_oracle as CO  # noqa: E402

POLISH_AMAX = 88  # the polish kernel's capacity for the reference agent at N = 30 (cmpc.solver.plan)


def main(tols):
    rounds = lpv_lab.load_rounds()
    if not rounds:
        sys.exit("no cached rounds: python tools/lpv_lab.py gen")
    CO._LIB = lpv_lab.variant("-DLAB_DEGEN_COUNT " + os.environ.get("DEGEN_FLAGS", ""))
    flagged = ct.c_long.in_dll(CO._LIB, "cmpc_degen_flagged")
    taken = ct.c_long.in_dll(CO._LIB, "cmpc_degen_taken")
    agents = sum(int(p["A"].shape[0]) for p in rounds)
    for tol in tols:
        flagged.value = taken.value = 0
        cnt, mx, err, t0 = {}, [], 0.0, time.perf_counter()
        for p in rounds:
            z, kkt, it, st = CO.solve_batch_rescue(p, tol=tol, nthreads=8, polish=True, polish_amax=POLISH_AMAX)
            mx.append(int(it.max()))
            err = max(err, float(kkt.max()))
            for k, v in zip(*np.unique(st, return_counts=True)):
                cnt[int(k)] = cnt.get(int(k), 0) + int(v)
        dt = time.perf_counter() - t0
        print(f"tol {tol:.0e}: {len(rounds)} rounds, {agents} agent-QPs; degenerate-flagged {flagged.value} "
              f"({100.0 * flagged.value / agents:.2f} %), polished point taken {taken.value}; status {cnt}; "
              f"max kkt {err:.1e}; sum(max it) {sum(mx)}; {dt:.1f} s on 8 threads", flush=True)


if __name__ == "__main__":
    main([float(a) for a in sys.argv[1:]] or [1e-9, 1e-8, 1e-7, 1e-6, 1e-5])
