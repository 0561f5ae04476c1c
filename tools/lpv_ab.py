"""Lab A/B of the reference-model rounds (bench.lpv_population, LPVRounds with the rescue policy):
run `rounds` rounds with the library named by CMPC_LIB_PATH and save z / status / iterations per
round, to compare two builds bit for bit (tools/lpv_ab.py cmp A.npz B.npz).
Usage: python tools/lpv_ab.py OUT.npz [rounds] | python tools/lpv_ab.py cmp A.npz B.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]


def run(out, rounds):
    import time

    import torch

    import bench
    from cmpc.rounds import LPVRounds

    bp, args, kw = bench.lpv_population(None)
    R = LPVRounds(bp, *args, **kw)
    zs, st, it = [], [], []
    t0 = time.perf_counter()
    for _ in range(rounds):
        R.step(halt=False)
        torch.cuda.synchronize()
        zs.append(R.z.cpu().numpy().copy())
        st.append(R.status.cpu().numpy().copy())
        it.append(R.iters.cpu().numpy().copy())
    el = time.perf_counter() - t0
    import hashlib

    hs = np.array([hashlib.sha256(z.tobytes()).hexdigest() for z in zs])
    np.savez(out, z=np.stack(zs[:2]), zsha=hs, status=np.stack(st), iters=np.stack(it))
    s = np.stack(st)
    print(f"lib {os.environ.get('CMPC_LIB_PATH', 'in-tree')}: {rounds} rounds {el / rounds * 1e3:.2f} ms/round (with host "
          f"copies); status {dict(zip(*np.unique(s, return_counts=True)))}")


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    for r in range(A["zsha"].shape[0]):
        dz = f", max |dz| {np.abs(A['z'][r] - B['z'][r]).max():.2e}" if r < A["z"].shape[0] else ""
        print(f"round {r}: bit-equal {A['zsha'][r] == B['zsha'][r]}{dz}, status diff "
              f"{int((A['status'][r] != B['status'][r]).sum())}, iterations diff {int((A['iters'][r] != B['iters'][r]).sum())}")


if __name__ == "__main__":
    if sys.argv[1] == "cmp":
        cmp(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
