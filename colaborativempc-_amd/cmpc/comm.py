"""RCCL communicator of a libcmpc context (cmpc_comm_* / cmpc_allgather_trajectories in
include/cmpc.h): the per-round exchange of predicted trajectories for hosts that shard agents
without torch.distributed — the replacement of the ROS topic exchange
(ROS/src/planner_experiments/src/LPV_ROS_main.py:66-77 publish, :124-150 subscribe) and of
the in-process np.swapaxes of planner/scripts/LPV_HP_N_main.py:117.

    uid = Comm.new_id()                # rank 0; hand the bytes to every rank
    comm = Comm(ctx, nranks, rank, uid) # collective
    comm.allgather(traj_local, traj_all)  # CUDA float64 tensors, stream-ordered
"""
from __future__ import annotations

import ctypes as ct

from . import _lib as L


class Comm:
    def __init__(self, ctx, nranks, rank, uid: bytes):
        if len(uid) != L.CMPC_COMM_ID_BYTES:
            raise ValueError(f"communicator id must be {L.CMPC_COMM_ID_BYTES} bytes")
        self.ctx, self.nranks, self.rank = ctx, int(nranks), int(rank)
        ctx.check(ctx.lib.cmpc_comm_init(ctx.h, self.nranks, self.rank, bytes(uid)))

    @staticmethod
    def new_id() -> bytes:
        buf = ct.create_string_buffer(L.CMPC_COMM_ID_BYTES)
        rc = L.load().cmpc_comm_id(buf)
        if rc != L.CMPC_OK:
            raise L.CmpcError(rc, "cmpc_comm_id failed (RCCL unavailable)")
        return buf.raw

    def allgather(self, traj_local, traj_all, stream=None):
        """traj_all (nranks*B, N+1, 2) <- every rank's traj_local (B, N+1, 2), rank order."""
        import torch

        for t in (traj_local, traj_all):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()):
                raise ValueError("trajectory buffers must be contiguous CUDA float64 tensors")
        if traj_all.numel() != self.nranks * traj_local.numel():
            raise ValueError("traj_all must hold nranks x the local trajectories")
        s = stream if stream is not None else torch.cuda.current_stream(traj_local.device)
        self.ctx.check(self.ctx.lib.cmpc_allgather_trajectories(
            self.ctx.h, ct.cast(traj_local.data_ptr(), L._DP), ct.cast(traj_all.data_ptr(), L._DP),
            traj_local.numel(), ct.c_void_p(s.cuda_stream)))

    def sum_i32(self, buf, stream=None):
        """buf (contiguous CUDA int32 tensor) <- its sum over every rank, in place (cmpc_comm_sum_i32)."""
        import torch

        if not (isinstance(buf, torch.Tensor) and buf.is_cuda and buf.dtype == torch.int32 and buf.is_contiguous()):
            raise ValueError("buf must be a contiguous CUDA int32 tensor")
        s = stream if stream is not None else torch.cuda.current_stream(buf.device)
        self.ctx.check(self.ctx.lib.cmpc_comm_sum_i32(self.ctx.h, ct.cast(buf.data_ptr(), L._IP), buf.numel(),
                                                      ct.c_void_p(s.cuda_stream)))

    def close(self):
        if getattr(self, "ctx", None) is not None:
            self.ctx.lib.cmpc_comm_destroy(self.ctx.h)
            self.ctx = None
