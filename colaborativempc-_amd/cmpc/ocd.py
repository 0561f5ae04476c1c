"""OCD coupling-dual round on the GPU (the consensus step of the reference's NL-DMPC loop,
planner/scripts/NL_EU_N_main.py:105-162; ROS variant OCD_ROS_main.py:200-239).

* ``dual_update``: lambda += alpha * (D - ||p_i(k) - p_j(k)||) for every neighbour pair with
  i < j and k = 1..N (eval_constraintEU, config/NL/config.py:19-23; alpha = get_alpha() =
  0.25, :5-8) — cmpc_ocd_update_dev, on the neighbour graph instead of the reference's dense
  (n_agents, n_agents, N) array.
* ``converged``: the per-agent np.allclose(x_old, x_pred, atol=0.01) test (:143-149) —
  cmpc_ocd_converged_dev; across ranks the flags are AND-ed with one all-reduce(MIN).
* ``OCDLoopState``: the loop's counters (it_OCD, itc, finished; :105-162) unchanged.
"""
from __future__ import annotations

import ctypes as ct

from . import _lib as L
from .solver import _tptr

ALPHA = 0.25   # get_alpha(), config/NL/config.py:5-8


def _stream(t, stream):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream(t.device)
    return ct.c_void_p(s.cuda_stream)


def dual_update(lam, traj_all, nbr, self_offset=0, alpha=ALPHA, dth=0.25, ctx=None, stream=None):
    """lam (B, nb, N) float64 CUDA, updated in place; traj_all (n_total, N+1, 2); nbr (B, nb) int32."""
    B, nb, N = lam.shape
    ctx = ctx or L.default_context(lam.device.index or 0)
    dims = L.cmpc_ocd_dims(B, N, nb, int(self_offset))
    ctx.check(ctx.lib.cmpc_ocd_update_dev(ctx.h, ct.byref(dims), float(alpha), float(dth), _tptr(nbr),
                                          _tptr(traj_all), _tptr(lam), _stream(lam, stream)))


def converged(x_old, x_pred, atol=0.01, rtol=1e-5, ctx=None, stream=None, group=None):
    """Per-agent np.allclose(x_old[b], x_pred[b], atol, rtol) on the device -> (close (B,) int32, all (bool))."""
    import torch

    B = x_old.shape[0]
    per = x_old[0].numel() if B else 0
    close = torch.empty(B, dtype=torch.int32, device=x_old.device)
    ctx = ctx or L.default_context(x_old.device.index or 0)
    ctx.check(ctx.lib.cmpc_ocd_converged_dev(ctx.h, B, per, float(atol), float(rtol), _tptr(x_old), _tptr(x_pred),
                                             _tptr(close), _stream(x_old, stream)))
    flag = close.min().reshape(1) if B else torch.ones(1, dtype=torch.int32, device=x_old.device)
    if group is not None or _dist_ready():
        import torch.distributed as dist

        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return close, bool(flag.item())


def _dist_ready():
    try:
        import torch.distributed as dist

        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    except Exception:
        return False


class OCDLoopState:
    """The OCD round counters of NL_EU_N_main.py:102-162 (min_it_OCD, it_conv, max_it_OCD)."""

    def __init__(self, min_it_OCD=2, it_conv=1, max_it_OCD=10):
        self.min_it_OCD, self.it_conv, self.max_it_OCD = min_it_OCD, it_conv, max_it_OCD
        self.it_OCD = 0
        self.itc = 0
        self.finished = False
        self.finished_ph = 0

    def running(self):
        """while(not (it_OCD > min_it_OCD and finished))  (:105)"""
        return not (self.it_OCD > self.min_it_OCD and self.finished)

    def after_round(self, all_close):
        """Counter update after a round (:143-162); `all_close` = AND over agents of allclose."""
        if self.it_OCD != 0:
            self.finished_ph = 1 if all_close else 0
            self.itc += 1
        if not self.finished_ph:
            self.itc = 0
        elif self.itc > self.it_conv:
            self.finished = True
        if self.it_OCD > self.max_it_OCD:
            self.finished = True
        self.it_OCD += 1
