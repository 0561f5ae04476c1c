"""Run bench.py's `lpv_rounds` line alone (the reference's agent model in device-resident rounds),
for profiling it under rocprofv3 and for A/B runs of solver options.

  python tools/run_lpv_rounds.py [--rounds R] [--no-rescue] [--finish] [--riccati] [--check]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--no-rescue", action="store_true")
    ap.add_argument("--check", action="store_true", help="also run the oracle checks of the bench line")
    ap.add_argument("--finish", action="store_true", help="CMPC_FLAG_FINISH")
    ap.add_argument("--riccati", action="store_true", help="CMPC_FLAG_RICCATI: every agent on the stage-wise kernel")
    a = ap.parse_args()
    import bench
    import cmpc

    ctx = cmpc.Context(0)
    out = bench.lpv_rounds(ctx, rounds=a.rounds, rescue=not a.no_rescue, check=a.check, finish=a.finish,
                           riccati=a.riccati)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
