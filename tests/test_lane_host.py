"""The lane-per-agent solver body (colaborativempc-_amd/csrc/lane_body.h, the code every lane of
mpc_lane_kernel runs) compiled for the HOST (tools/lane_cpu.cpp, hipcc --offload-host-only) and
checked against the C restatement on CPU: the fp64 body runs the restatement's Riccati method
(oracle newton 1), the mixed body (fp32 factorisation, BASELINE cfg5's fp32 path) reaches the fp64
optimum within the fp32 bar.  The stage images the device fills by LDS-DMA are emulated per agent;
the GPU runs are in tests/test_gpu.py."""
import ctypes as ct
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


@pytest.fixture(scope="module")
def lane_lib(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("lane") / "lane_cpu.so")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-host-only", "-x", "hip",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "colaborativempc-_amd", "csrc"),
                    os.path.join(ROOT, "tools", "lane_cpu.cpp"), "-o", so], check=True)
    return ct.CDLL(so)


@pytest.fixture(scope="module")
def cfg5_batch():
    from cmpc import scenarios as S
    from oracle import synth

    n = 24
    sc = S.make_di(n, 50, 2, 3)
    return synth.structured(sc.shared, sc.params, sc.A, sc.B, sc.x0, sc.u_prev, sc.lane, sc.nbr, sc.traj,
                            np.arange(n))


def _solve(lib, p, tol, mixed):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import lane_cpu

    return lane_cpu.solve(lib, p, tol, mixed=mixed)


def test_lane_body_fp64_matches_riccati_restatement(lane_lib, cfg5_batch):
    from oracle import cmpc_oracle as CO

    z, kkt, it, st = _solve(lane_lib, cfg5_batch, 1e-9, False)
    zc, kc, ic, sc = CO.solve_batch(cfg5_batch, nthreads=4, newton=1)
    both = (st == 1) & (sc == 1)
    assert np.mean(st == sc) >= 0.9 and both.mean() >= 0.8
    assert np.abs(z[both] - zc[both]).max() < 1e-6


def test_lane_body_mixed_meets_fp32_bar(lane_lib, cfg5_batch):
    from oracle import cmpc_oracle as CO

    z, kkt, it, st = _solve(lane_lib, cfg5_batch, 1e-6, True)
    zc, _, _, sc = CO.solve_batch(cfg5_batch, nthreads=4, newton=3)
    err = np.abs(z - zc) / np.maximum(1.0, np.abs(zc))
    assert np.isin(st, (1, 2)).all() and np.mean(st == 1) >= 0.9
    assert err.max() < 1e-3
