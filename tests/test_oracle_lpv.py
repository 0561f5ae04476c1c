"""The oracle's numpy restatement of PlannerLPV against QPs captured from the
reference's own code (tests/golden/*.npz, oracle/gen_fixtures.py)."""
import numpy as np
import pytest

from conftest import LPV_CASES, golden, lpv_qps
from oracle import lpv_ref as L
from oracle import qp_ipm


@pytest.mark.parametrize("name", LPV_CASES)
def test_assembly_matches_reference_bit_exact(name):
    tr = L.Track.build("Highway")
    g = L.paper_gains()
    for j, c in lpv_qps(name):
        lim = L.scaled_car_limits(c["vx_ref"])
        xa = c["x_agents"]
        qp = L.assemble(c["x0"], c["x_last"], c["u_last"], xa, c["pose"], c["u_old"], c["N"], c["dt"], tr,
                        L.SCALED_CAR_MODEL, lim, g)
        assert np.array_equal(qp.P, c["P"]), (name, j)
        assert np.array_equal(qp.q, c["q"]), (name, j)
        assert np.array_equal(qp.A, c["A"]), (name, j)
        assert np.array_equal(qp.u, c["u"]), (name, j)
        assert np.array_equal(qp.l, c["l"]), (name, j)
        if xa.shape[1]:
            assert np.array_equal(qp.planes, c["planes"]), (name, j)


@pytest.mark.parametrize("name", LPV_CASES)
def test_golden_solutions_are_kkt_certified(name):
    d = golden(name)
    assert d["stat"].max() < 1e-11
    assert d["prim"].max() < 1e-12
    assert d["comp"].max() < 5e-9


def test_ipm_resolves_golden():
    for j, c in lpv_qps("lpv_n10_a2"):
        r = qp_ipm.solve_qp(c["P"], c["q"], c["A"], c["l"], c["u"])
        assert r.status == "solved"
        assert np.abs(r.x - c["z"]).max() < 1e-7


def test_unpack_matches_reference_unpack():
    d = golden("lpv_n30_a3")
    for j in range(len(d["step"])):
        x, u, s = L.unpack(d["z"][j], int(d["N"]))
        assert np.array_equal(x, d["xPred"][j])
        assert np.array_equal(u, d["uPred"][j])
        assert np.array_equal(s, d["sPred"][j])


def test_maps_and_lookups():
    d = golden("maps")
    for nm in ("Highway", "oval", "Oval2", "SL"):
        tr = L.Track.build(nm)
        np.testing.assert_allclose(tr.PointAndTangent, d[f"{nm}_PointAndTangent"], rtol=0, atol=1e-12)
        assert np.array_equal(tr.TrackLength, d[f"{nm}_TrackLength"]) or \
            np.allclose(tr.TrackLength, d[f"{nm}_TrackLength"], atol=1e-12)
        s = d[f"{nm}_s"]
        assert np.array_equal(np.array([L.curvature(v, tr) for v in s]), d[f"{nm}_curv"])
        assert np.array_equal(L.get_ey(s, tr), d[f"{nm}_ey"])
        if f"{nm}_global" in d:
            gp = np.array([L.Track.getGlobalPosition(tr, v, e) for v, e in zip(s, d[f"{nm}_ey_in"])], float)
            np.testing.assert_allclose(gp, d[f"{nm}_global"], rtol=0, atol=1e-12)


def test_scheduling_planes_weights():
    d = golden("schedule")
    tr = L.Track.build("Highway")
    for case, N in enumerate((10, 30)):
        A, B, ey = L.estimate_abc(d[f"c{case}_states"], d[f"c{case}_u"], N, 0.025, L.SCALED_CAR_MODEL, tr)
        assert np.array_equal(A, d[f"c{case}_A"])
        assert np.array_equal(B, d[f"c{case}_B"])
        assert np.array_equal(ey, d[f"c{case}_ey"])
        pl = L.compute_hyperplane(d[f"c{case}_agents"], d[f"c{case}_pose"], N)
        assert np.array_equal(pl, d[f"c{case}_planes"])
        w, dist = L.compute_weights(d[f"c{case}_pose"], d[f"c{case}_agents"], 0.25)
        assert np.array_equal(w, d[f"c{case}_w"])
        assert np.array_equal(dist, d[f"c{case}_dist"])


def test_low_speed_branch_exercised():
    d = golden("schedule")
    st = d["c0_states"]
    assert (st[:10, 0] < 0.2).any()
    A = d["c0_A"]
    i = int(np.argmax(st[:10, 0] < 0.2))
    assert A[i, 0, 1] == 0.0 and A[i, 1, 1] == 1.0  # A12 = A22 = 0 -> identity row parts
