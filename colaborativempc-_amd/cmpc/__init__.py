"""cmpc — MI355X-native batched collaborative-MPC QP solver (host side).

The compute path is libcmpc.so (HIP kernels for gfx950 behind the C ABI in
include/cmpc.h).  This package is the host-side mirror of the reference's
planner interface (MarcFacerias/ColaborativeMPC-, planner/lib/plan_lib) plus the
round driver and synthetic workloads.  There is no CPU solve path here.
"""
from ._lib import (CMPC_MAX_ITER_REACHED, CMPC_SOLVED, CMPC_SOLVED_INACCURATE, CMPC_UNSOLVED, CmpcError,
                   Context, default_context, load)
from .planner import PlannerLPV, PlannerLPVBatch, feasible_of, unpack
from .qp import osqp_solve_qp, osqp_solve_qp_batch, quadprog
from .solver import nz_of, selftest_mfma, solve_mpc, solve_mpc_dev

__all__ = ["Context", "CmpcError", "default_context", "load", "PlannerLPV", "PlannerLPVBatch", "feasible_of",
           "unpack", "quadprog", "osqp_solve_qp", "osqp_solve_qp_batch", "solve_mpc", "solve_mpc_dev", "nz_of", "selftest_mfma", "CMPC_SOLVED",
           "CMPC_SOLVED_INACCURATE", "CMPC_MAX_ITER_REACHED", "CMPC_UNSOLVED"]
