"""CPU checks of how bench.py picks the committed counter evidence it reports (`roofline.traffic`,
`roofline.counters`): the summary whose `sources_sha` matches the current kernel sources wins over a
newer-named or newer-taken one that does not (the file-name order had reported a stale
round-5 SQ summary), then the one taken last, then the file name; and the committed summaries describe
the kernel sources in the tree (`stale` false)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _write(tmp_path, name, rec):
    p = tmp_path / name
    p.write_text(json.dumps(rec))
    return str(p)


def test_select_profile_prefers_matching_sources_then_time_then_name(tmp_path):
    a = _write(tmp_path, "sq_cfg5_r05sq.json", {"sources_sha": "old", "taken_unix": 300.0})
    b = _write(tmp_path, "sq_cfg5_r05am.json", {"sources_sha": "now", "taken_unix": 100.0})
    c = _write(tmp_path, "sq_cfg5_r06a.json", {"sources_sha": "now", "taken_unix": 200.0})
    d = _write(tmp_path, "sq_cfg5_r06b.json", {"sources_sha": "now"})             # no time: oldest
    bad = tmp_path / "sq_cfg5_r07.json"
    bad.write_text("{not json")
    path, rec = bench.select_profile([a, b, c, d, str(bad)], "now")
    assert path == c and rec["taken_unix"] == 200.0
    # no record of the current sources: the one taken last
    path, _ = bench.select_profile([a, b, c], "other")
    assert path == a
    # equal keys: the file name decides
    e = _write(tmp_path, "sq_cfg5_r06c.json", {"sources_sha": "now", "taken_unix": 200.0})
    path, _ = bench.select_profile([c, e], "now")
    assert path == e
    assert bench.select_profile([], "now") == (None, None)


@pytest.mark.parametrize("kind", [None, "cfg5", "cfg5fp32"])
def test_committed_traffic_summary_describes_current_sources(kind):
    traffic, src = bench.pmc_traffic(kind)
    assert traffic and traffic > 0
    assert src["stale"] is False, src


@pytest.mark.parametrize("kind", ["cfg3", "cfg5", "cfg5fp32"])
def test_committed_sq_summary_describes_current_sources(kind):
    rec = bench.sq_profile(kind)
    assert rec is not None and rec["stale"] is False, rec
    shares = rec["active_inst_any"] + rec["wait_any"] + rec["wait_inst_any"]
    assert 0.8 < shares < 1.2   # the SQ_WAVE_CYCLES split adds up (SQ counters)
