"""The MEX gateway (quadprog drop-in) compiled against the mock mex.h:
argument validation and the no-device error path run on CPU; the solve path is in
tests/test_qp_gpu.py (marked gpu)."""
import numpy as np
import pytest
import torch

import mex_harness as MH

pytestmark = pytest.mark.skipif(not __import__("os").path.exists(MH.MOCK), reason="libcmpc_mex_mock.so not built")


@pytest.mark.parametrize("args,msg", [
    ((np.eye(3),), "usage"),
    ((np.ones((3, 2)), np.zeros(3)), "n x n"),
    ((np.eye(3), np.zeros(2)), "f has 2 elements"),
    ((np.eye(3), np.zeros(3), np.ones((2, 4)), np.zeros(2)), "A must have n columns"),
    ((np.eye(3), np.zeros(3), np.ones((2, 3)), None), "A given without b"),
    ((np.eye(3), np.zeros(3), None, None, np.ones((1, 3)), None), "Aeq given without beq"),
    ((np.eye(3), np.zeros(3), None, None, None, None, np.zeros(2)), "lb has 2 elements"),
])
def test_argument_errors(args, msg):
    out, err = MH.call(args)
    assert out is None and err[0] == "cmpc:quadprog:args" and msg in err[1], err


def test_no_device_raises_device_error():
    if torch.cuda.is_available():
        pytest.skip("device present")
    out, err = MH.call((np.eye(2), np.zeros(2)))
    assert out is None and err[0] == "cmpc:device", err
