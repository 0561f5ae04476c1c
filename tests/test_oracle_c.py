"""The plain-C condensed IPM (oracle/cmpc_oracle.c — CPU baseline and at-scale
checker) against the reference-form certified optima."""
import os
import sys

import numpy as np
import pytest

from conftest import LPV_CASES, assert_matches_optimum, lpv_qps
from oracle import cmpc_oracle as CO
from oracle import lpv_ref as L
from oracle import qp_ipm, synth


@pytest.mark.parametrize("name", LPV_CASES)
def test_c_oracle_matches_golden(name):
    tr = L.Track.build("Highway")
    g = L.paper_gains()
    probs, refs = [], []
    for j, c in lpv_qps(name):
        lim = L.scaled_car_limits(c["vx_ref"])
        qp = L.assemble(c["x0"], c["x_last"], c["u_last"], c["x_agents"], c["pose"], c["u_old"], c["N"],
                        c["dt"], tr, L.SCALED_CAR_MODEL, lim, g)
        probs.append(L.structured(qp, c["x0"], c["u_old"], c["N"], lim, g))
        refs.append(c["z"])
    z, kkt, it, st = CO.solve_batch(L.stack(probs))
    assert np.isin(st, (1, 2)).all() and (st == 1).mean() >= 0.8
    for a, (j, c) in enumerate(lpv_qps(name)):
        assert_matches_optimum(z[a], c, 1e-6)


def test_structured_expansion_equals_reference_form():
    """synth.reference_form applied to the LPV structured statement reproduces the
    captured reference QP exactly: the structured layout IS the reference QP."""
    tr = L.Track.build("Highway")
    g = L.paper_gains()
    for j, c in lpv_qps("lpv_n10_a2"):
        lim = L.scaled_car_limits(c["vx_ref"])
        qp = L.assemble(c["x0"], c["x_last"], c["u_last"], c["x_agents"], c["pose"], c["u_old"], c["N"],
                        c["dt"], tr, L.SCALED_CAR_MODEL, lim, g)
        s = L.structured(qp, c["x0"], c["u_old"], c["N"], lim, g)
        P, q, A, l, u = synth.reference_form(s, 0)
        assert np.array_equal(P, c["P"]) and np.array_equal(q, c["q"])
        # same rows; the reference keeps its 0=0 slack rows, which are identical here
        assert np.array_equal(A, c["A"]) and np.array_equal(u, c["u"]) and np.array_equal(l, c["l"])


@pytest.mark.parametrize("n,N,nb,dim", [(2, 10, 1, 2), (8, 20, 2, 2), (6, 30, 2, 2), (4, 10, 2, 3)])
def test_c_oracle_synthetic_vs_reference_form(n, N, nb, dim):
    from cmpc import scenarios as S

    sc = S.make_di(n, N, nb, dim)
    P = synth.structured(sc.shared, sc.params, sc.A, sc.B, sc.x0, sc.u_prev, sc.lane, sc.nbr, sc.traj,
                         np.arange(n))
    z, kkt, it, st = CO.solve_batch(P)
    assert (st == 1).all()
    for a in range(min(n, 2)):
        r = qp_ipm.solve_qp(*synth.reference_form(P, a))
        assert np.abs(z[a] - r.x).max() < 1e-6
