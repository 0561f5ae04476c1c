"""Lab A/B of the cfg3 solver (the bench's fused round, DIRounds): run `rounds` consecutive rounds
with the library named by CMPC_LIB_PATH (default: the in-tree build), print per-round kernel time,
iterations and statuses, check a 128-agent sample of round 0 and of the last round against the C
restatement, and save z / iterations per round to OUT.npz for a comparison between builds
(tools/v3_ab.py cmp A.npz B.npz).

Usage: python tools/v3_ab.py OUT.npz [rounds] [agents]
       python tools/v3_ab.py cmp A.npz B.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
sys.path.insert(0, ROOT)


def run(out, rounds, agents):
    import torch

    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds
    from oracle import cmpc_oracle as CO

    sc = S.make_di(agents, 30, 2, 2)
    R = DIRounds(sc)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(rounds)]
    it = torch.empty((rounds, R.B), dtype=torch.int32, device=R.dev)
    kk = torch.empty((rounds, R.B), dtype=torch.float64, device=R.dev)
    st = torch.empty((rounds, R.B), dtype=torch.int32, device=R.dev)
    zs, errs = [], []
    smp = np.arange(0, agents, max(1, agents // 128))[:128]
    for r in range(rounds):
        R.bind_outputs(kk[r], it[r], st[r])
        check = r in (0, rounds - 1)
        if check:
            R.build()
            P = R.snapshot()
        R.step(timer=ev[r])
        if r < 3 or check:
            torch.cuda.synchronize()
            z = R.z.cpu().numpy().copy()
            if r < 3:
                zs.append(z)
            if check:
                Ps = {k: (v[smp] if isinstance(v, np.ndarray) and v.ndim and v.shape[0] == agents else v)
                      for k, v in P.items()}
                zc, _, _, _ = CO.solve_batch(Ps, nthreads=min(16, os.cpu_count() or 1))
                errs.append(float(np.abs(z[smp] - zc).max()))
    torch.cuda.synchronize()
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    itn, stn, kkn = it.cpu().numpy(), st.cpu().numpy(), kk.cpu().numpy()
    np.savez(out, z=np.stack(zs), iters=itn, status=stn, kkt=kkn, ms=ms)
    w = min(3, rounds - 1)
    print(f"lib {os.environ.get('CMPC_LIB_PATH', 'in-tree')}: kernel ms mean {ms[w:].mean():.4f} (rounds {w}..) "
          f"iters mean {itn.mean():.3f} mean-max {itn.max(1).mean():.2f} ms/maxit {ms[w:].sum() / itn[w:].max(1).sum():.5f} "
          f"status {dict(zip(*np.unique(stn, return_counts=True)))} max kkt {kkn.max():.2e} "
          f"|z - z_cpu| (128 agents, first/last round) {errs}", flush=True)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    w = 3
    print(f"kernel ms {A['ms'][w:].mean():.4f} -> {B['ms'][w:].mean():.4f} "
          f"({A['ms'][w:].mean() / B['ms'][w:].mean():.3f}x); per max-iteration "
          f"{A['ms'][w:].sum() / A['iters'][w:].max(1).sum() * 1e3:.2f} -> "
          f"{B['ms'][w:].sum() / B['iters'][w:].max(1).sum() * 1e3:.2f} us")
    print(f"iters equal {np.mean(A['iters'] == B['iters']):.4f}; round 0..2 max |z_a - z_b| "
          f"{[float(np.abs(x - y).max()) for x, y in zip(A['z'], B['z'])]}")


if __name__ == "__main__":
    if sys.argv[1] == "cmp":
        cmp(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40, int(sys.argv[3]) if len(sys.argv) > 3 else 1024)
