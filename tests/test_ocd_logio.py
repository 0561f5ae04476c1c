"""OCD round semantics (oracle restatement of NL_EU_N_main.py:105-162) and the log /
wire formats (base_class.py:64-166, misc.py:264-275, utilities_ros.py:7-45) — CPU."""
import os
import re

import numpy as np

from cmpc import logio
from cmpc.ocd import OCDLoopState
from oracle import ocd_ref


def test_ocd_update_only_fills_upper_pairs():
    rng = np.random.default_rng(0)
    n, N = 3, 5
    agents = rng.standard_normal((N + 1, n, 2))
    lam = ocd_ref.ocd_update(np.zeros((n, n, N)), agents, N, 0.25)
    assert np.all(lam[np.tril_indices(n)[0], np.tril_indices(n)[1]] == 0)
    d = np.linalg.norm(agents[1:, 0] - agents[1:, 1], axis=1)
    assert np.allclose(lam[0, 1], 0.25 * (0.25 - d), rtol=0, atol=1e-15)


def test_loop_counters_follow_reference():
    # rounds 0..3: it_OCD 0 skips the test, round 1 not close (itc reset), rounds 2, 3 close ->
    # itc = 2 > it_conv finishes, and it_OCD = 4 > min_it_OCD ends the loop
    st = OCDLoopState(min_it_OCD=2, it_conv=1, max_it_OCD=10)
    seq = [False, False, True, True, True, True]
    rounds = 0
    while st.running():
        st.after_round(seq[min(rounds, len(seq) - 1)])
        rounds += 1
    assert rounds == 4 and st.finished
    st = OCDLoopState(min_it_OCD=2, it_conv=1, max_it_OCD=3)
    rounds = 0
    while st.running():
        st.after_round(False)
        rounds += 1
    assert rounds == 5  # it_OCD > max_it_OCD after the 5th round, and it_OCD > min_it_OCD


def test_csv_format_matches_reference_writer(tmp_path):
    rng = np.random.default_rng(1)
    states = rng.standard_normal((4, 9))
    p = logio.save_to_csv(str(tmp_path), 2, states, rng.standard_normal((4, 2)), rng.random(4),
                          [0.1, 0.2, 0.3, 0.4, 0.1, 0.2, 0.3, 0.4], ocd_it=[2, 2, 2, 2])
    line = open(os.path.join(p, "states.dat")).readline().strip()
    assert re.fullmatch(r"(-?\d\.\d{5}e[+-]\d{2} ){8}-?\d\.\d{5}e[+-]\d{2}", line)
    assert np.allclose(np.loadtxt(os.path.join(p, "states.dat")), states, rtol=1e-5)
    assert np.allclose(np.loadtxt(os.path.join(p, "time.dat")), [0.3, 0.7, 0.3, 0.7])
    assert np.loadtxt(os.path.join(p, "time_OCD.dat")).shape == (4, 2)
    logio.save_settings(str(tmp_path), {"N": 30, "dt": 0.025})
    assert open(os.path.join(str(tmp_path), "settings.csv")).read().splitlines() == ["N,30", "dt,0.025"]


def test_ros_payload_round_trip():
    x = np.arange(31 * 9, dtype=np.float64).reshape(31, 9) / 7.0
    back = logio.deserialise_np(logio.serialise_np([x]))[0]
    assert back.dtype == np.float32 and back.shape == x.shape
    assert np.array_equal(back, x.astype(np.float32))


REF_LOGS = os.path.join(os.path.dirname(__file__), "golden", "ref_logs")


def _bytes(p):
    with open(p, "rb") as f:
        return f.read()


def test_lpv_log_rewrite_is_byte_identical_to_reference_files(tmp_path):
    """Rows the reference's writer produced (an LPV run: OCD_it == [] so time / time_OCD are the
    raw solve times and OCD_it.dat is empty) re-written by cmpc.logio: the same bytes."""
    src = os.path.join(REF_LOGS, "lpv", "csv", "0")
    st, u = np.loadtxt(os.path.join(src, "states.dat")), np.loadtxt(os.path.join(src, "u.dat"))
    la, t = np.loadtxt(os.path.join(src, "plan_dist.dat")), np.loadtxt(os.path.join(src, "time.dat"))
    out = logio.save_to_csv(str(tmp_path) + "/", 0, st, u, la, t, ocd_it=[])
    for nm in ("states", "u", "plan_dist", "time", "OCD_it"):
        assert _bytes(os.path.join(out, f"{nm}.dat")) == _bytes(os.path.join(src, f"{nm}.dat")), nm


def test_ocd_log_rewrite_matches_reference_files(tmp_path):
    """An OCD run (NL_3agents_def_t2, agent 2): states / u / plan_dist / time_OCD / OCD_it
    byte-identical; time.dat (per-step sums of the round times) equal to the printed digits
    (re-summed from the 6-digit time_OCD rows the reference printed)."""
    src = os.path.join(REF_LOGS, "ocd", "csv", "2")
    rd = lambda nm: np.loadtxt(os.path.join(src, f"{nm}.dat"))   # noqa: E731
    it = rd("OCD_it").astype(int)
    tocd = np.atleast_2d(rd("time_OCD"))
    time_op = np.concatenate([tocd[i, :it[i]] for i in range(len(it))])
    out = logio.save_to_csv(str(tmp_path) + "/", 2, rd("states"), rd("u"), rd("plan_dist"), time_op, ocd_it=list(it))
    for nm in ("states", "u", "plan_dist", "time_OCD", "OCD_it"):
        assert _bytes(os.path.join(out, f"{nm}.dat")) == _bytes(os.path.join(src, f"{nm}.dat")), nm
    np.testing.assert_allclose(np.loadtxt(os.path.join(out, "time.dat")), rd("time"), rtol=2e-5)


def test_settings_rewrite_is_byte_identical_to_reference_file(tmp_path):
    import csv

    src = os.path.join(REF_LOGS, "lpv", "settings.csv")
    with open(src, newline="") as f:
        rows = [tuple(r) for r in csv.reader(f)]
    logio.save_settings(str(tmp_path), dict(rows))
    assert _bytes(os.path.join(tmp_path, "settings.csv")) == _bytes(src)


def _ocd_cases():
    from conftest import golden

    d = golden("ocd_rounds")
    c = 0
    while f"c{c}_n" in d.files:
        yield c, d
        c += 1


def test_ocd_oracle_bit_exact_against_reference_functions():
    """oracle.ocd_ref restates the dual update and the convergence test of NL_EU_N_main.py:127-149;
    tests/golden/ocd_rounds.npz holds rounds computed by the reference's own get_alpha and
    eval_constraintEU (oracle/gen_ocd_fixtures.py): bit-exact."""
    from oracle import ocd_ref

    for c, d in _ocd_cases():
        n, N, dth = int(d[f"c{c}_n"]), int(d[f"c{c}_N"]), float(d[f"c{c}_dth"])
        for r in range(int(d[f"c{c}_rounds"])):
            got = ocd_ref.ocd_update(d[f"c{c}_r{r}_lam_in"], d[f"c{c}_r{r}_agents"], N, dth)
            assert np.array_equal(got, d[f"c{c}_r{r}_lam_out"]), (c, r)
            if f"c{c}_r{r}_close" in d.files:
                assert np.array_equal(ocd_ref.allclose_agents(d[f"c{c}_r{r}_x_old"], d[f"c{c}_r{r}_x_pred"]),
                                      d[f"c{c}_r{r}_close"])
