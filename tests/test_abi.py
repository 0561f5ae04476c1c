"""C-ABI boundary checks that need no GPU: the in-tree libcmpc.so loads, exports
every function include/cmpc.h declares, and refuses to run without a gfx950
device (there is no CPU fallback)."""
import ctypes as ct
import re

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
    assert L.load().cmpc_abi_version() == 3


def test_no_cpu_fallback_without_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("device present")
    h = ct.c_void_p()
    rc = L.load().cmpc_create(ct.byref(h), 0)
    assert rc == L.CMPC_ERR_DEVICE
    with pytest.raises(cmpc.CmpcError):
        cmpc.Context(0)
