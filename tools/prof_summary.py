"""Summarise rocprofv3 output of bench.py runs into profiles/.

  python tools/prof_summary.py trace  <run_kernel_trace.csv> <warmup> <steps> <out.json>
      per-dispatch durations of the solver kernel; the average over the bench's timed
      launches (dispatches warmup .. warmup+steps-1) is the number bench.py's
      roofline.kernel_ms_per_launch must agree with.
  python tools/prof_summary.py pmc <counter_collection.csv (FETCH pass)> <(WRITE pass)> <out.json> [commit]
  SOLVER=<kernel name substring> selects the solver kernel (default mpc_ipm; cfg5: mpc_riccati,
  the fp32 path: mpc_lane_kernel).
      HBM bytes per launch of the solver kernel from FETCH_SIZE / WRITE_SIZE (kB), with the
      gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE counts half the
      bytes of wide coalesced reads: x2).
"""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def solver_sources_sha():
    """sha256 over the HIP sources and headers libcmpc is built from (bench.py recomputes it to
    tell whether a committed PMC figure still describes the current kernels)."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "colaborativempc-_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "colaborativempc-_amd", "csrc", "*.h")) +
                   [os.path.join(ROOT, "include", "cmpc.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]

SOLVER = os.environ.get("SOLVER", "mpc_ipm")   # default: mpc_ipm_kernel<...>, mpc_ipm3_kernel<...>


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def trace(path, warmup, steps, out):
    rows = [r for r in _rows(path) if SOLVER in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]
    timed = dur[warmup:warmup + steps]
    res = {"kernel": rows[0]["Kernel_Name"] if rows else None, "dispatches": len(dur),
           "all_avg_ms": sum(dur) / max(1, len(dur)),
           "timed_avg_ms": sum(timed) / max(1, len(timed)), "timed_dispatches": len(timed),
           "timed_ms": timed}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "timed_ms"}))


def _pmc(path, counter):
    vals = {}
    for r in _rows(path):
        if SOLVER not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
            continue
        d = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def pmc(fetch_csv, write_csv, out, commit=None):
    fk = _pmc(fetch_csv, "FETCH_SIZE")
    wk = _pmc(write_csv, "WRITE_SIZE")
    # skip the first dispatch of each run (cold caches / first touch)
    f = fk[1:] or fk
    w = wk[1:] or wk
    fetch_b = 2.0 * 1024.0 * sum(f) / max(1, len(f))   # kB -> B, x2 gfx950 read correction
    write_b = 1024.0 * sum(w) / max(1, len(w))
    res = {"solve_kernel": {"fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
                            "hbm_bytes_per_launch": fetch_b + write_b,
                            "fetch_kB_raw": fk, "write_kB_raw": wk,
                            "note": "FETCH_SIZE x2 (gfx950 half-count of wide reads); first dispatch skipped",
                            "kernel_filter": SOLVER},
           "commit": commit, "sources_sha": solver_sources_sha()}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        trace(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else None)
