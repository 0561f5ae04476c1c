"""C-ABI boundary checks that need no GPU: the in-tree libcmpc.so loads, exports
every function include/cmpc.h declares, and refuses to run without a gfx950
device (there is no CPU fallback)."""
import ctypes as ct
import re

import numpy as np
import pytest

import cmpc
from cmpc import _lib as L


def declared_functions():
    src = open(L.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(cmpc_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for need in ("cmpc_create", "cmpc_destroy", "cmpc_solve_mpc_batch", "cmpc_solve_mpc_batch_dev",
                 "cmpc_solve_lpv_batch", "cmpc_solve_lpv_batch_dev", "cmpc_di_build_dev", "cmpc_di_solve_dev",
                 "cmpc_di_advance_dev", "cmpc_lpv_gather_dev", "cmpc_lpv_advance_dev", "cmpc_lpv_rounds_create",
                 "cmpc_lpv_rounds_step", "cmpc_lpv_rounds_read", "cmpc_lpv_rounds_destroy"):
        assert need in fns


def test_library_exports_every_declared_symbol():
    lib = L.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in L.SIGNATURES, f"{name} has no ctypes signature"


def test_abi_version():
    assert L.load().cmpc_abi_version() == 6


def test_plan_occupancy_of_the_bench_configs():
    """cmpc_plan_mpc (host only): the solver each BASELINE shape runs and how many of its workgroups
    share a CU.  Guards the occupancy the bench numbers rest on: the cfg3 condensed kernel and the
    cfg5 Riccati kernel (fp64 and the fp32 mode) must keep four one-wave workgroups per CU — one per
    SIMD (round 3's cfg5 image grew to 41.3 KB, over the 40 KB for four, and ran three)."""
    from cmpc import scenarios as S
    from cmpc.solver import plan

    p3 = plan(S.di_shared(2, 30, 2), 1024)
    assert p3["solver"] == "condensed_v3" and p3["wg_per_cu"] == 4 and p3["lds_bytes"] <= 40 * 1024, p3
    for fp32 in (False, True):
        p5 = plan(S.di_shared(3, 50, 2), 8192, fp32=fp32)
        assert p5["solver"] == "riccati" and p5["wg_per_cu"] == 4 and p5["lds_bytes"] <= 40 * 1024, p5
    pl = plan(S.di_shared(3, 50, 2), 8192, fp32=True, lane=True)
    assert pl["solver"] == "lane" and pl["agents_per_wg"] == 32
    assert plan(S.di_shared(2, 30, 2), 1024, generic=True)["solver"] == "condensed"
    with pytest.raises(cmpc.CmpcError):   # no fp32 path for nb = 3 at these dimensions
        plan(S.di_shared(2, 20, 3), 16, fp32=True)
    # CMPC_FLAG_POLISH (with CMPC_FLAG_RESCUE) is a known option bit: the condensed plan is unchanged
    pp = plan(S.di_shared(2, 30, 2), 1024, rescue=True, polish=True)
    assert pp["solver"] == "condensed_v3" and pp["wg_per_cu"] == 4, pp
    # the two wave-count flags are exclusive; a structured batch runs one wave per agent
    with pytest.raises(cmpc.CmpcError):
        plan(S.di_shared(2, 30, 2), 512, flags=L.CMPC_FLAG_ONE_WAVE | L.CMPC_FLAG_TWO_WAVES)
    assert plan(S.di_shared(2, 30, 2), 512, flags=L.CMPC_FLAG_TWO_WAVES)["waves_per_agent"] == 1
    # the Riccati kernel's latency mode: the PlannerLPV agent at the reference's N = 125 (an LDS image over
    # half a CU) gets four wavefronts; CMPC_FLAG_ONE_WAVE keeps one; the synthetic shapes keep one
    lpv = dict(nx=9, nu=2, N=125, ns=3, mc=6, Q=np.diag([10.0, 0, 0, 25, 10, 0, 0, 0, 0]), R=np.zeros((2, 2)),
               dR=50 * np.eye(2), Qs=1e7 * np.ones(3), u_ub=np.array([0.3, 5.0]), u_lb=np.array([-0.3, -10.0]),
               row_slack=np.array([-1, 0, 1, 1, 2, 2]), row_sign=np.array([1, 1, 1, 1, -1, -1]))
    p125 = plan(lpv, 3)
    assert p125["solver"] == "riccati" and p125["waves_per_agent"] == 4 and p125["lds_bytes"] <= 160 * 1024, p125
    p125one = plan(lpv, 3, flags=L.CMPC_FLAG_ONE_WAVE)
    assert p125one["waves_per_agent"] == 1 and p125one["lds_bytes"] < p125["lds_bytes"], p125one
    assert plan(dict(lpv, N=30), 3, riccati=True)["waves_per_agent"] == 1
    assert all(plan(S.di_shared(3, 50, 2), 8192, fp32=f)["waves_per_agent"] == 1 for f in (False, True))


def test_no_cpu_fallback_without_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("device present")
    h = ct.c_void_p()
    rc = L.load().cmpc_create(ct.byref(h), 0)
    assert rc == L.CMPC_ERR_DEVICE
    with pytest.raises(cmpc.CmpcError):
        cmpc.Context(0)
