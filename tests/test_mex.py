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


# ---- cmpc_lpv: the LPV gateway (PlannerLPV batch and the round handle) ----
lpv_built = pytest.mark.skipif(not __import__("os").path.exists(MH.LPV_MOCK), reason="libcmpc_lpv_mex_mock.so not built")


def lpv_params(N=10):
    """cmpc_lpv's P struct for the reference's gains, SCALED CAR model and limits, Highway track."""
    from oracle import lpv_ref as L

    g, tr = L.paper_gains(), L.Track.build("Highway")
    tab = tr.PointAndTangent[:, :, 0]
    f = {k: np.array([v]) for k, v in L.SCALED_CAR_MODEL.items()}
    f.update({k: np.array([float(v)]) for k, v in L.scaled_car_limits().items() if k != "sm"})
    f.update(dt=np.array([0.025]), wq=np.array([g["wq"]]), Q=g["Q"], Qs=g["Qs"], R=g["R"], dR=g["dR"],
             N=np.array([float(N)]))
    f["track"] = MH.mx_struct(dict(s0=tab[:, 3], len=tab[:, 4], curv=tab[:, 5], half_width=tr.halfWidth[: tab.shape[0]]))
    return f


@lpv_built
@pytest.mark.parametrize("cmd,extra,msg", [
    ("nope", [], "unknown command"),
    ("solve", [], "usage"),
    ("rounds_step", [np.array([3.0]), np.array([1.0])], "bad rounds handle"),
    ("rounds_read", [np.array([0.0])], "bad rounds handle"),
])
def test_lpv_gateway_argument_errors(cmd, extra, msg):
    out, err = MH.call_lpv([MH.mx_str(cmd)] + [MH.mx(a) for a in extra], 1)
    assert out is None and err[0] == "cmpc:lpv:args" and msg in err[1], err


@lpv_built
def test_lpv_gateway_rejects_bad_structs():
    P = MH.mx_struct(lpv_params())
    out, err = MH.call_lpv([MH.mx_str("solve"), P, MH.mx_struct({"x0": np.zeros((9, 2))})], 1)
    assert out is None and err[0] == "cmpc:lpv:args" and "x_last is required" in err[1], err
    D = MH.mx_struct({"x0": np.zeros((9, 2)), "x_last": np.zeros((9, 7, 2))})
    out, err = MH.call_lpv([MH.mx_str("solve"), P, D], 1)
    assert out is None and "x_last must be 9 x (N or N+1) x B" in err[1], err
    out, err = MH.call_lpv([MH.mx_str("solve"), MH.mx_struct({"lf": np.array([0.1])}), D], 1)
    assert out is None and "is required" in err[1], err
