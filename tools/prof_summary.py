"""Summarise rocprofv3 output of bench.py runs into profiles/.

  python tools/prof_summary.py trace  <run_kernel_trace.csv> <warmup> <steps> <out.json>
      per-dispatch durations of the solver kernel; the average over the bench's timed
      launches (dispatches warmup .. warmup+steps-1) is the number bench.py's
      roofline.kernel_ms_per_launch must agree with.
  python tools/prof_summary.py pmc <counter_collection.csv (FETCH pass)> <(WRITE pass)> <out.json> [commit]
  python tools/prof_summary.py sq <out.json> <commit> <pass1.csv> [pass2.csv ...]   (tools/pmc_sq.sh passes)
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
import time

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
           "commit": commit, "sources_sha": solver_sources_sha(), "taken_unix": time.time()}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


def _pmc_all(path):
    """{counter: [per-dispatch values of the solver kernel]} of one --pmc pass."""
    vals = {}
    for r in _rows(path):
        if SOLVER not in r.get("Kernel_Name", ""):
            continue
        d = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        c = vals.setdefault(r["Counter_Name"], {})
        c[d] = c.get(d, 0.0) + float(r["Counter_Value"])
    return {k: [v[d] for d in sorted(v)] for k, v in vals.items()}


def sq(out, commit, *csvs):
    """Instruction-mix / wave-state summary of the solver kernel from SQ (and GRBM) counter passes
    (tools/pmc_sq.sh: one pass per counter group).  Per-launch means over the dispatches after the
    first; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES
    and SQ_BUSY_CYCLES cycles (MI355X_MICROARCH.md, PMC units).  Fractions of the kernel's wave time:
    active (an instruction issued), waiting (s_waitcnt: LDS / memory latency), issue-stalled
    (dependency / pipe hazards), VALU active, MFMA busy."""
    per = {}
    for path in csvs:
        for k, v in _pmc_all(path).items():
            per[k] = v
    mean = {k: (sum(v[1:]) / len(v[1:]) if len(v) > 1 else v[0]) for k, v in per.items() if v}
    g = mean.get
    wc = g("SQ_WAVE_CYCLES")
    res = {"counters_per_launch": mean, "kernel_filter": SOLVER, "commit": commit, "sources_sha": solver_sources_sha(),
           "taken_unix": time.time()}
    if wc:
        res["fractions_of_wave_time"] = {
            "active_inst_any": g("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "active_valu": g("SQ_ACTIVE_INST_VALU", 0.0) / wc,
            "active_lds": g("SQ_ACTIVE_INST_LDS", 0.0) / wc,
            "active_salu": g("SQ_ACTIVE_INST_SCA", 0.0) / wc,
            "wait_any": g("SQ_WAIT_ANY", 0.0) / wc,
            "wait_inst_any": g("SQ_WAIT_INST_ANY", 0.0) / wc,
            "mfma_busy": g("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (4.0 * wc),
        }
        waves = g("SQ_WAVES") or 1.0
        res["per_wave"] = {"cycles": 4.0 * wc / waves, "valu_insts": g("SQ_INSTS_VALU", 0.0) / waves,
                           "fma_f64_insts": g("SQ_INSTS_VALU_FMA_F64", 0.0) / waves,
                           "mfma_insts": g("SQ_INSTS_MFMA", 0.0) / waves, "lds_insts": g("SQ_INSTS_LDS", 0.0) / waves,
                           "salu_insts": g("SQ_INSTS_SALU", 0.0) / waves}
        if g("SQ_LDS_IDX_ACTIVE"):
            res["lds_bank_conflict_frac"] = g("SQ_LDS_BANK_CONFLICT", 0.0) / g("SQ_LDS_IDX_ACTIVE")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}))


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        trace(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    elif sys.argv[1] == "sq":   # prof_summary.py sq OUT.json COMMIT pass1.csv pass2.csv ...
        sq(sys.argv[2], sys.argv[3], *sys.argv[4:])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else None)
