"""ctypes binding of libcmpc.so (include/cmpc.h).

The shared library is built in-tree (``colaborativempc-_amd/lib/libcmpc.so``) by
``__graft_entry__.build()`` / ``make -C colaborativempc-_amd/csrc``.  There is no
CPU fallback: if the library is missing, ``load()`` raises, and if no gfx950
device is present ``Context()`` raises ``CmpcError(CMPC_ERR_DEVICE)``.
"""
from __future__ import annotations

import ctypes as ct
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
# CMPC_LIB_PATH: an alternative build of the same ABI (profiling variants under tools/)
LIB_PATH = os.environ.get("CMPC_LIB_PATH") or os.path.join(ROOT, "lib", "libcmpc.so")
HEADER = os.path.join(os.path.dirname(ROOT), "include", "cmpc.h")

CMPC_OK = 0
CMPC_ERR_ARG = -1
CMPC_ERR_DEVICE = -2
CMPC_ERR_UNSUPPORTED = -3
CMPC_ERR_NOMEM = -4

CMPC_SOLVED = 1
CMPC_SOLVED_INACCURATE = 2
CMPC_MAX_ITER_REACHED = -2
CMPC_PRIMAL_INFEASIBLE = -3
CMPC_UNSOLVED = -10

STATUS_TEXT = {1: "solved", 2: "solved inaccurate", -2: "maximum iterations reached",
               -3: "primal infeasible", -10: "unsolved"}

_DP = ct.POINTER(ct.c_double)
_IP = ct.POINTER(ct.c_int)


CMPC_FLAG_GENERIC = 1
CMPC_FLAG_FP32 = 8
CMPC_FLAG_RICCATI = 16
CMPC_FLAG_RESCUE = 32   # Riccati continuation of agents whose condensed factorisation broke down
CMPC_FLAG_FINISH = 64   # ... also of breakdowns already at the rounding floor (status 2)
CMPC_FLAG_LANE = 128    # lane-per-agent stage-wise kernel, fp64
CMPC_FLAG_POLISH = 256  # with RESCUE: active-set polish of breakdowns at the rounding floor (OSQP polish=True)
CMPC_FLAG_ONE_WAVE = 512   # fused DS round: one wavefront per agent (the default)
CMPC_FLAG_TWO_WAVES = 1024  # ... two wavefronts per agent (opt-in: bit-identical, no faster at 512 agents)


class cmpc_opts(ct.Structure):
    _fields_ = [("tol", ct.c_double), ("max_iter", ct.c_int), ("flags", ct.c_int), ("stamps", ct.c_void_p),
                ("order", ct.c_void_p)]


class cmpc_mpc_dims(ct.Structure):
    _fields_ = [(k, ct.c_int) for k in ("nx", "nu", "N", "ns", "mc", "batch")]


class cmpc_mpc_weights(ct.Structure):
    _fields_ = [("Q", _DP), ("R", _DP), ("dR", _DP), ("Qs", _DP), ("u_ub", _DP), ("u_lb", _DP),
                ("row_slack", _IP), ("row_sign", _IP)]


CMPC_SOLVER_CONDENSED_V3, CMPC_SOLVER_CONDENSED, CMPC_SOLVER_RICCATI, CMPC_SOLVER_LANE = 1, 2, 3, 4


class cmpc_plan_info(ct.Structure):
    _fields_ = [(k, ct.c_int) for k in ("solver", "lds_bytes", "wg_per_cu", "agents_per_wg", "waves_per_agent",
                                        "polish_lds_bytes", "polish_max_active")]


class cmpc_mpc_data(ct.Structure):
    _fields_ = [(k, _DP) for k in ("A", "B", "x0", "u_prev", "qlin", "C", "h")]


class cmpc_mpc_out(ct.Structure):
    _fields_ = [("z", _DP), ("kkt", _DP), ("iters", _IP), ("status", _IP)]


class cmpc_lpv_params(ct.Structure):
    _fields_ = [(k, ct.c_double) for k in ("lf", "lr", "m", "I", "Cf", "Cr", "mu", "vx_ref", "min_dist",
                                           "max_vel", "min_vel", "max_rs", "max_ls", "max_ac", "max_dc",
                                           "dt", "wq")] + \
               [("Q", ct.c_double * 81), ("Qs", ct.c_double * 3), ("R", ct.c_double * 4), ("dR", ct.c_double * 4)]


class cmpc_track(ct.Structure):
    _fields_ = [("nseg", ct.c_int), ("s0", _DP), ("len", _DP), ("curv", _DP), ("half_width", _DP)]


class cmpc_lpv_dims(ct.Structure):
    _fields_ = [(k, ct.c_int) for k in ("batch", "N", "nb", "last_rows")]


class cmpc_lpv_data(ct.Structure):
    _fields_ = [(k, _DP) for k in ("x0", "x_last", "u_last", "u_old", "x_agents", "pose")]


class cmpc_lpv_out(ct.Structure):
    _fields_ = [("z", _DP), ("planes", _DP), ("kkt", _DP), ("iters", _IP), ("status", _IP)]


class cmpc_lpv_build_out(ct.Structure):
    _fields_ = [("A", _DP), ("B", _DP), ("qlin", _DP), ("C", _DP), ("h", _DP), ("planes", _DP), ("err", _IP)]


class cmpc_di_params(ct.Structure):
    _fields_ = [("dim", ct.c_int)] + [(k, ct.c_double) for k in ("v_ref", "q_v", "q_lane", "hw", "min_vel",
                                                                 "max_vel", "min_dist", "wq")]


class cmpc_di_dims(ct.Structure):
    _fields_ = [(k, ct.c_int) for k in ("batch", "N", "nb", "self_offset")]


CMPC_ROUNDS_HOST_EXCHANGE = 1
CMPC_ROUNDS_NO_HALT = 2


class cmpc_lpv_rounds_dims(ct.Structure):
    _fields_ = [(k, ct.c_int) for k in ("n_total", "batch", "self_offset", "N", "nb", "flags")]


class cmpc_lpv_rounds_init(ct.Structure):
    _fields_ = [("x0", _DP), ("x_last", _DP), ("u_last", _DP), ("u_old", _DP), ("nbr", _IP), ("traj", _DP)]


class cmpc_lpv_rounds_out(ct.Structure):
    _fields_ = [("z", _DP), ("kkt", _DP), ("iters", _IP), ("status", _IP), ("x0", _DP), ("planes", _DP)]


class cmpc_qp_dims(ct.Structure):
    _fields_ = [(k, ct.c_int) for k in ("n", "m_ineq", "m_eq", "batch", "col_major")]


class cmpc_qp_data(ct.Structure):
    _fields_ = [(k, _DP) for k in ("H", "f", "A", "b", "Aeq", "beq", "lb", "ub")]


class cmpc_qp_out(ct.Structure):
    _fields_ = [("x", _DP), ("fval", _DP), ("exitflag", _IP), ("iters", _IP), ("lambda_ineqlin", _DP),
                ("lambda_eqlin", _DP), ("lambda_lower", _DP), ("lambda_upper", _DP), ("residual", _DP)]


CMPC_QP_CONVERGED = 1
CMPC_QP_MAXITER = 0
CMPC_QP_INFEASIBLE = -2
CMPC_QP_UNBOUNDED = -3
CMPC_QP_NONCONVEX = -6


class cmpc_ocd_dims(ct.Structure):
    _fields_ = [(k, ct.c_int) for k in ("batch", "N", "nb", "self_offset")]


class CmpcError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"libcmpc error {code}: {msg}")
        self.code = code


_LIB = None

# name -> (restype, argtypes) for every function declared in include/cmpc.h
SIGNATURES = {
    "cmpc_abi_version": (ct.c_int, []),
    "cmpc_create": (ct.c_int, [ct.POINTER(ct.c_void_p), ct.c_int]),
    "cmpc_destroy": (ct.c_int, [ct.c_void_p]),
    "cmpc_last_error": (ct.c_char_p, [ct.c_void_p]),
    "cmpc_solve_mpc_batch": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_mpc_dims), ct.POINTER(cmpc_mpc_weights),
                                        ct.POINTER(cmpc_mpc_data), ct.POINTER(cmpc_mpc_out), ct.POINTER(cmpc_opts)]),
    "cmpc_solve_mpc_batch_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_mpc_dims), ct.POINTER(cmpc_mpc_weights),
                                            ct.POINTER(cmpc_mpc_data), ct.POINTER(cmpc_mpc_out),
                                            ct.POINTER(cmpc_opts), ct.c_void_p]),
    "cmpc_solve_lpv_batch": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_lpv_params), ct.POINTER(cmpc_track),
                                        ct.POINTER(cmpc_lpv_dims), ct.POINTER(cmpc_lpv_data),
                                        ct.POINTER(cmpc_lpv_out), ct.POINTER(cmpc_opts)]),
    "cmpc_solve_lpv_batch_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_lpv_params), ct.POINTER(cmpc_track),
                                            ct.POINTER(cmpc_lpv_dims), ct.POINTER(cmpc_lpv_data),
                                            ct.POINTER(cmpc_lpv_out), ct.POINTER(cmpc_opts), ct.c_void_p]),
    "cmpc_di_build_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_di_params), ct.POINTER(cmpc_di_dims),
                                     _IP, _DP, _DP, _DP, _DP, _DP, ct.c_void_p]),
    "cmpc_di_solve_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_di_params), ct.POINTER(cmpc_di_dims), _IP, _DP,
                                     _DP, ct.POINTER(cmpc_mpc_dims), ct.POINTER(cmpc_mpc_weights),
                                     ct.POINTER(cmpc_mpc_data), ct.POINTER(cmpc_mpc_out), ct.POINTER(cmpc_opts),
                                     ct.c_void_p]),
    "cmpc_lpv_gather_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_di_dims), _IP, _DP, _DP, _DP, ct.c_void_p]),
    "cmpc_lpv_advance_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_di_dims), _DP, _DP, _DP, _DP, _DP, _DP,
                                        _IP, _IP, ct.c_void_p]),
    "cmpc_di_advance_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_di_params), ct.POINTER(cmpc_di_dims),
                                       _DP, _DP, _DP, _DP, ct.c_void_p]),
    "cmpc_solve_qp_batch": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_qp_dims), ct.POINTER(cmpc_qp_data),
                                       ct.POINTER(cmpc_qp_out), ct.POINTER(cmpc_opts)]),
    "cmpc_ocd_update_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_ocd_dims), ct.c_double, ct.c_double, _IP, _DP,
                                       _DP, ct.c_void_p]),
    "cmpc_ocd_converged_dev": (ct.c_int, [ct.c_void_p, ct.c_int, ct.c_int, ct.c_double, ct.c_double, _DP, _DP, _IP,
                                          ct.c_void_p]),
    "cmpc_selftest_mfma": (ct.c_int, [ct.c_void_p, _DP, _DP, _DP]),
    "cmpc_lpv_build_dev": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_lpv_params), ct.POINTER(cmpc_track),
                                      ct.POINTER(cmpc_lpv_dims), ct.POINTER(cmpc_lpv_data),
                                      ct.POINTER(cmpc_lpv_build_out), ct.c_void_p]),
    "cmpc_comm_id": (ct.c_int, [ct.c_char_p]),
    "cmpc_comm_init": (ct.c_int, [ct.c_void_p, ct.c_int, ct.c_int, ct.c_char_p]),
    "cmpc_allgather_trajectories": (ct.c_int, [ct.c_void_p, _DP, _DP, ct.c_ulonglong, ct.c_void_p]),
    "cmpc_comm_sum_i32": (ct.c_int, [ct.c_void_p, _IP, ct.c_ulonglong, ct.c_void_p]),
    "cmpc_plan_mpc": (ct.c_int, [ct.POINTER(cmpc_mpc_dims), ct.POINTER(cmpc_mpc_weights), ct.POINTER(cmpc_opts),
                                 ct.POINTER(cmpc_plan_info)]),
    "cmpc_comm_destroy": (ct.c_int, [ct.c_void_p]),
    "cmpc_lpv_rounds_create": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_lpv_params), ct.POINTER(cmpc_track),
                                          ct.POINTER(cmpc_lpv_rounds_dims), ct.POINTER(cmpc_lpv_rounds_init),
                                          ct.POINTER(cmpc_opts), ct.POINTER(ct.c_void_p)]),
    "cmpc_lpv_rounds_step": (ct.c_int, [ct.c_void_p, ct.c_int, _IP, _IP]),
    "cmpc_lpv_rounds_read": (ct.c_int, [ct.c_void_p, ct.POINTER(cmpc_lpv_rounds_out)]),
    "cmpc_lpv_rounds_get_traj": (ct.c_int, [ct.c_void_p, _DP]),
    "cmpc_lpv_rounds_set_traj": (ct.c_int, [ct.c_void_p, _DP]),
    "cmpc_lpv_rounds_destroy": (ct.c_int, [ct.c_void_p]),
}

CMPC_COMM_ID_BYTES = 128


def load():
    """Load libcmpc.so (raises FileNotFoundError if it was not built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                                    f"or make -C colaborativempc-_amd/csrc")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (SONAME
        # libamdhip64.so.7) and loads it by the unversioned name.  Loading torch first
        # makes libcmpc's NEEDED libamdhip64.so.7 bind to that same runtime; loading
        # libcmpc first would give the process two runtimes and torch would see no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ct.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
    return _LIB


def dptr(a):
    return None if a is None else a.ctypes.data_as(_DP)


def iptr(a):
    return None if a is None else a.ctypes.data_as(_IP)


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def opts(tol=None, max_iter=None, flags=0, stamps=None, order=None):
    """cmpc_opts; stamps / order: device pointers (int) or None."""
    return cmpc_opts(float(tol or 0.0), int(max_iter or 0), int(flags), stamps, order)


class Context:
    """One libcmpc context on one HIP device (cmpc_create / cmpc_destroy)."""

    def __init__(self, device=0):
        self.lib = load()
        h = ct.c_void_p()
        rc = self.lib.cmpc_create(ct.byref(h), int(device))
        if rc != CMPC_OK:
            raise CmpcError(rc, f"cmpc_create(device={device}) failed: no usable gfx950 device")
        self.h = h
        self.device = device

    def check(self, rc):
        if rc != CMPC_OK:
            msg = self.lib.cmpc_last_error(self.h)
            raise CmpcError(rc, msg.decode() if msg else "")

    def close(self):
        if getattr(self, "h", None):
            self.lib.cmpc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_DEFAULT = {}


def default_context(device=0):
    if device not in _DEFAULT:
        _DEFAULT[device] = Context(device)
    return _DEFAULT[device]
