"""Host logic of the PlannerLPV mirror (no GPU): solution unpacking with the reference's
index expressions (LPV_Planner.py:164-178) and the coverage weights / distances it sets on
every call (:132-139, utilities/misc.py:10-18), checked against the captured reference data."""
import numpy as np

from conftest import golden

from cmpc import planner as P


def test_unpack_index_expressions():
    d = golden("lpv_n30_a3")
    N = int(d["N"])
    nexp, ns, nu = 12, 9, 2
    for j in range(len(d["step"])):
        z = d["z"][j]
        x, u, du, s, raw = P.unpack(z, N)
        assert np.array_equal(x, d["xPred"][j]) and np.array_equal(u, d["uPred"][j])
        assert np.array_equal(s, d["sPred"][j])
        # duPred: the reference's expression at :175, verbatim (an every-other-entry view of
        # [u | du], not the rates); the rates themselves come from du_of
        k = np.arange(nu * N)
        assert np.array_equal(du, z[nexp * (N + 1) + k + k].reshape(N, nu))
        assert np.array_equal(du[: N // 2].ravel(), u[:, 0])
        assert np.array_equal(P.du_of(z, N), z[nexp * (N + 1) + nu * N + k].reshape(N, nu))
        assert np.array_equal(raw, z[: nexp * (N + 1)].reshape(N + 1, nexp))
        assert raw.shape[1] - ns == 3


def test_weights_and_dist_match_reference_capture():
    d = golden("schedule")
    for case in (0, 1):
        w, dist = P.weights_of(d[f"c{case}_pose"], d[f"c{case}_agents"], 0.25)
        assert np.array_equal(w, d[f"c{case}_w"])
        assert np.array_equal(dist, d[f"c{case}_dist"])


def test_feasible_rule():
    # LPV_Planner.py:243-249: status_val in {1, 2, -2} is feasible
    assert [P.feasible_of(s) for s in (1, 2, -2, -3, -10)] == [1, 1, 1, 0, 0]
