"""Diagnostic: is the cfg5 Riccati launch bound by its per-agent work or by how the 8192 agents pack
onto the 1024 SIMDs?  On the BASELINE cfg5 problem (8192 agents, N = 50, nx 6, nu 3) after two
closed-loop rounds: per-agent shader clocks (stamps), the launch time under the identity order, the
order by this solve's own IPM iterations and by its own clocks (longest first), and the packing
lower bound max(slowest agent, sum of clocks / 1024 SIMDs).
Usage: python tools/cfg5_sched.py [agents] [flags: fp32]"""
import ctypes as ct
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "colaborativempc-_amd")]
import torch  # noqa: E402

from cmpc import _lib as L  # noqa: E402
from cmpc import scenarios as S  # noqa: E402
from cmpc.rounds import DIRounds  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
fp32 = "fp32" in sys.argv[2:]
R = DIRounds(S.make_di(n, 50, 2, 3), fused=False, fp32=fp32, lpt=False)
for _ in range(2):
    R.step()
R.build()
torch.cuda.synchronize()
flags = L.CMPC_FLAG_FP32 if fp32 else 0


def solve(order=None, stamps=None, reps=3):
    R.opts = L.opts(R.opts.tol, None, flags, stamps=None if stamps is None else stamps.data_ptr(),
                    order=None if order is None else order.data_ptr())
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e in ev:
        e[0].record()
        R.ctx.check(R.ctx.lib.cmpc_solve_mpc_batch_dev(R.ctx.h, ct.byref(R.mdims), ct.byref(R.w), ct.byref(R.data),
                                                       ct.byref(R.out), ct.byref(R.opts), R._stream()))
        e[1].record()
    torch.cuda.synchronize()
    return min(a.elapsed_time(b) for a, b in ev)


st = torch.zeros((n, 16), dtype=torch.int64, device=R.dev)
solve(stamps=st, reps=1)
a = st.cpu().numpy().astype(np.float64)
cyc = a[:, [0, 1, 2, 3, 4, 5, 6, 7, 8, 14]].sum(1)
it = R.iters.cpu().numpy().copy()
t_id = solve()
o_it = torch.as_tensor(np.argsort(-it, kind="stable"), dtype=torch.int32, device=R.dev)
o_cy = torch.as_tensor(np.argsort(-cyc, kind="stable"), dtype=torch.int32, device=R.dev)
o_rnd = torch.as_tensor(np.random.default_rng(3).permutation(n), dtype=torch.int32, device=R.dev)
t_it, t_cy, t_rnd = solve(o_it), solve(o_cy), solve(o_rnd)
sims = 1024
lb = max(cyc.max(), cyc.sum() / sims)
print(f"cfg5{' fp32' if fp32 else ''} x{n}: iterations mean {it.mean():.2f} max {it.max()}; clocks per agent (stamped) "
      f"mean {cyc.mean() / 1e6:.2f}M p99 {np.percentile(cyc, 99) / 1e6:.2f}M max {cyc.max() / 1e6:.2f}M")
print(f"launch ms: identity {t_id:.2f}, random {t_rnd:.2f}, longest-first by iterations {t_it:.2f}, "
      f"by clocks {t_cy:.2f}")
print(f"packing lower bound {lb / 1e6:.1f}M clk = {lb / 2.4e9 * 1e3:.2f} ms at 2.4 GHz (stamped clocks, ~+10 % over "
      f"unstamped); sum/SIMDs {cyc.sum() / sims / 1e6:.1f}M, slowest agent {cyc.max() / 1e6:.1f}M")
