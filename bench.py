"""Benchmark: agent-QP solves/s for the whole node (BASELINE.json metric) on the
per-control-step distributed QP loop, device-resident, one process per GPU.

A step = one consensus round over every agent of every rank:
  build (stage rows / costs from the exchanged trajectories, cmpc_di_build_dev)
  -> batched condensed IPM, one wavefront per agent (cmpc_solve_mpc_batch_dev)
  -> round advance (cmpc_di_advance_dev) -> RCCL all-gather of predicted positions.
Workload (BASELINE.json configs[2], the config the metric is quoted on):
1024 agents per GPU, N=30, 2-D double integrator (nx=4, nu=2), nb=2 neighbours,
fp64 — weak scaling (1024 agents per rank; the 4096-agent cfg4 at 4 GPUs).

Usage: python bench.py [--gpus N --steps K --warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "colaborativempc-_amd"))
sys.path.insert(0, ROOT)

METRIC = "agent-QP solves/sec (whole node) at N=30, nx=4 nu=2; max KKT residual vs ref"
FP64_PEAK_TFLOPS = 78.6   # MI355X dense FP64 (vector == matrix): AMD's datasheet figure; the MI355X guide has no FP64 line
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector, spec
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=["cfg3", "cfg5"], default="cfg3",
                    help="cfg3 (the metric's config, default) or cfg5: 8192 agents/GPU, N=50, 3-D double "
                         "integrator (nx=6, nu=3) on the fp64 stage-wise Riccati kernel")
    ap.add_argument("--fp32", action="store_true",
                    help="cfg5 only: BASELINE cfg5's fp32 path (the Riccati kernel's fp32 mode: an fp32 Riccati "
                         "factorisation, fp64 iterates / residuals, tol 1e-6), checked against the fp64 solve")
    ap.add_argument("--agents", type=int, default=None, help="agents per GPU (default: the config's)")
    ap.add_argument("--agents-total", type=int, default=None,
                    help="strong scaling: this many agents in all, split evenly over the ranks (BASELINE cfg4: "
                         "--agents-total 4096 on 8 GPUs); default: weak scaling, --agents per GPU")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--nb", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ref", action="store_true", help="skip the reference-configuration (N=125) line")
    ap.add_argument("--no-cfg5", action="store_true",
                    help="skip the cfg5 sub-object of the default line (BASELINE configs[4]: fp64 and fp32 paths)")
    args = ap.parse_args()
    cfg5 = args.config == "cfg5"
    if args.fp32 and not cfg5:
        raise SystemExit("--fp32 is the cfg5 path (use --config cfg5 --fp32)")
    if args.agents_total is not None and args.agents is not None:
        raise SystemExit("--agents (per GPU, weak scaling) and --agents-total (strong scaling) exclude each other")
    strong = args.agents_total is not None
    args.agents = args.agents or (8192 if cfg5 else 1024)
    args.horizon = args.horizon or (50 if cfg5 else 30)
    dim = 3 if cfg5 else 2

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # CMPC_DIST_BACKEND: "nccl" (RCCL over xGMI, one GPU per rank: the default) or "gloo" (ranks that
    # share a device, exchange staged through the host: tests/test_dist_gpu.py rehearses the
    # multi-rank bench path this way on a one-GPU box); CMPC_DEVICE overrides LOCAL_RANK's device
    backend = os.environ.get("CMPC_DIST_BACKEND", "nccl")
    local = int(os.environ.get("CMPC_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import cmpc
    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    if strong:
        if args.agents_total % world:
            raise SystemExit(f"--agents-total {args.agents_total} is not divisible by {world} ranks")
        args.agents = args.agents_total // world
    n_total = args.agents * world
    scen = S.make_di(n_total, args.horizon, args.nb, dim)
    ctx = cmpc.Context(local)
    R = DIRounds(scen, rank=rank, world=world, device=local, ctx=ctx, fp32=args.fp32)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    # per-round solver outputs land in their own rows (no accounting kernels in the timed loop);
    # the tallies are taken after it
    B = R.B
    hist_kkt = torch.empty((args.steps, B), dtype=torch.float64, device=dev)
    hist_it = torch.empty((args.steps, B), dtype=torch.int32, device=dev)
    hist_st = torch.empty((args.steps, B), dtype=torch.int32, device=dev)
    for _ in range(max(1, args.warmup)):   # warm-up also loads every kernel the timed loop uses
        R.step(timer=ev[0])
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        R.bind_outputs(hist_kkt[k], hist_it[k], hist_st[k])
        R.step(timer=ev[k])
    barrier()
    elapsed = time.perf_counter() - t0
    iters_sum = hist_it.to(torch.float64).sum()
    kkt_max = hist_kkt.max()
    # unsolved: neither solved nor solved-inaccurate (OSQP status_val 1 / 2)
    bad = ((hist_st != cmpc.CMPC_SOLVED) & (hist_st != cmpc.CMPC_SOLVED_INACCURATE)).sum()
    inacc = (hist_st == cmpc.CMPC_SOLVED_INACCURATE).sum()
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    red_dev = dev if backend == "nccl" else torch.device("cpu")   # gloo reduces host tensors
    stats = torch.tensor([elapsed, kern_ms, kkt_max.item()], dtype=torch.float64, device=red_dev)
    tot = torch.tensor([iters_sum.item(), float(bad.item()), float(inacc.item())], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed, kern_ms, kkt_all = stats.tolist()
    it_all, bad_all, inacc_all = tot.tolist()
    mean_iters = it_all / (n_total * args.steps)

    value = n_total * args.steps / elapsed
    sh = scen.shared
    nx, nu, N, mc = sh["nx"], sh["nu"], sh["N"], sh["mc"]
    m_rows = N * mc + 2 * nu * N
    flops = S.riccati_flops(nx, nu, N, mean_iters) if cfg5 else S.alg_flops(nx, nu, N, m_rows, mean_iters)
    achieved_tf = flops * args.agents / (kern_ms * 1e-3) / 1e12
    alg_bytes = S.di_alg_bytes(nx, nu, N, args.nb)
    pmc_kind = ("cfg5fp32" if args.fp32 else "cfg5") if cfg5 else None
    traffic, traffic_src = pmc_traffic(pmc_kind)
    peak = FP32_PEAK_TFLOPS if args.fp32 else FP64_PEAK_TFLOPS
    fp32_check = fp32_vs_fp64(R) if (args.fp32 and rank == 0) else None

    cpu = None
    max_err = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu, max_err = cpu_baseline(R, args.cpu_seconds, rounds=1 if cfg5 else 4, newton=3 if cfg5 else 0,
                                    label=args.config)
    ref_line = osqp_line = cfg5_sub = None
    if rank == 0 and world == 1 and not args.no_cfg5 and not cfg5 and not strong:
        cfg5_sub = cfg5_line(ctx)
    if rank == 0 and world == 1 and not args.no_ref and not cfg5:
        ref_line = reference_config(ctx)
        ref_line["lpv_rounds"] = lpv_rounds(ctx)
        ref_line["lpv_rounds_finish"] = lpv_rounds(ctx, finish=True, check=False)
        osqp_line = osqp_dropin(ctx)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "agent-QP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32 factorisation / f64 residuals" if args.fp32 else "f64",
            "data": "synthetic (seeded double-integrator agent population, SURVEY.md §8d)",
            "config": {
                "workload": (f"cfg5: {args.agents} agents/GPU, N={N}, 3-D double integrator nx={nx} nu={nu}, "
                             f"nb={args.nb}, " +
                             ("fp32 path: stage-wise Riccati IPM (one wavefront per agent) with the Riccati "
                              "factorisation and Newton recursions in fp32, fp64 iterates and residuals, per-agent "
                              "fp64 finish, tol 1e-6"
                              if args.fp32 else
                              "fp64 stage-wise Riccati IPM (BASELINE asks fp32; fp64 >= it)") +
                             "; step = build+solve+advance+all-gather") if cfg5 else
                            (f"cfg4: {n_total} agents in all ({args.agents} per GPU over {world}), N={N}, 2-D double "
                             f"integrator nx={nx} nu={nu}, nb={args.nb}, fp64 condensed IPM, strong scaling; step = "
                             f"build+solve+advance+all-gather" if strong and n_total == 4096 else
                             f"cfg3: {args.agents} agents/GPU, N={N}, 2-D double integrator nx={nx} nu={nu}, "
                             f"nb={args.nb}, fp64 condensed IPM; step = build+solve+advance+all-gather"),
                "agents_total": n_total, "horizon": N, "nx": nx, "nu": nu, "neighbours": args.nb,
                "parallelism": f"agents sharded over {world} GPU(s), "
                               f"{'RCCL' if backend == 'nccl' else backend} all-gather per round",
            },
            "fp32_vs_fp64": fp32_check,
            "max_kkt": kkt_all,
            "unsolved": int(bad_all),
            "solved_inaccurate": int(inacc_all),
            "mean_ipm_iters": mean_iters,
            "max_abs_err_vs_cpu": max_err,
            "roofline": {
                "kernel": ("mpc_riccati_kernel<Cfg<2,6,3,6,GR,F32>>" if args.fp32 else
                           "mpc_riccati_kernel<Cfg<2,6,3,6,GR>>") if cfg5 else "mpc_ipm3_kernel<4,4,2,2>",
                # neither MFMA- nor HBM-bound: one wavefront per agent runs dependent chains (sq_profile:
                # the wave's instruction-issue, wait and MFMA-busy shares of its cycles, from SQ counters)
                "bound": "latency",
                "counters": sq_profile(pmc_kind or "cfg3"),
                "achieved": achieved_tf,
                "peak": peak,
                "peak_note": "fp32 vector (the factorisation's precision)" if args.fp32 else
                             "fp64 vector = matrix, AMD datasheet figure (not in the MI355X guide)",
                "unit": "TFLOP/s",
                "frac": achieved_tf / peak,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel_ms_per_launch": kern_ms,
                "alg_flops_per_qp": flops,
                "alg_bytes_per_qp": alg_bytes,
                "hbm_alg_GBs": alg_bytes * args.agents / (kern_ms * 1e-3) / 1e9,
                "hbm_frac": alg_bytes * args.agents / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            },
            "cpu_baseline": cpu,
            "cfg5": cfg5_sub,
            "reference_config": ref_line,
            "osqp_dropin": osqp_line,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def cfg5_line(ctx, steps=10, warmup=2):
    """BASELINE configs[4] inside the default line, so the driver observes it: 8192 agents, N = 50,
    3-D double integrator (nx 6, nu 3), nb 2 — the fp64 stage-wise Riccati path and the fp32 path
    (the Riccati kernel's fp32 mode: fp32 factorisation and Newton recursions, fp64 iterates,
    tol 1e-6), each timed over `steps` device-resident rounds after `warmup` (10 / 2: the standalone
    `--config cfg5` line's counts, so the two agree; 5 timed rounds read ~7 % lower: 237.7k against
    255.8k agent-QP/s in profiles/r05ad_*) (the same step as the
    main line: build + solve + advance + exchange), with the fp32 path's tolerance check against the
    fp64 solve of the same problems (fp32_vs_fp64: every agent's max |z32 - z64| / max(1, |z64|),
    bar 1e-3) and its roofline (stage-wise Riccati flops at the measured iterations)."""
    import torch

    from cmpc import scenarios as S
    from cmpc.rounds import DIRounds

    scen = S.make_di(8192, 50, 2, 3)
    out = {"workload": "cfg5: 8192 agents/GPU, N=50, 3-D double integrator nx=6 nu=3, nb=2; step = "
                       "build+solve+advance+exchange", "steps": steps, "warmup": warmup}
    for fp32 in (False, True):
        R = DIRounds(scen, ctx=ctx, fp32=fp32)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        its = torch.empty((steps, R.B), dtype=torch.int32, device=R.dev)
        kk = torch.empty((steps, R.B), dtype=torch.float64, device=R.dev)
        st = torch.empty((steps, R.B), dtype=torch.int32, device=R.dev)
        for _ in range(warmup):
            R.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            R.bind_outputs(kk[k], its[k], st[k])
            R.step(timer=ev[k])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern = sum(a.elapsed_time(b) for a, b in ev) / steps
        mean_it = float(its.to(torch.float64).mean())
        flops = S.riccati_flops(6, 3, 50, mean_it)
        ach = flops * R.B / (kern * 1e-3) / 1e12
        peak = FP32_PEAK_TFLOPS if fp32 else FP64_PEAK_TFLOPS
        kind = "cfg5fp32" if fp32 else "cfg5"
        traffic, src = pmc_traffic(kind)
        stn, kkn = st.cpu().numpy(), kk.cpu().numpy()
        k2 = np.sort(kkn[stn == 2])[::-1]  # the rounding-floor solves' KKT residuals (scaled), largest first
        line = {"value": R.B * steps / el, "unit": "agent-QP/s", "ms_per_step": el / steps * 1e3,
                "mean_ipm_iters": mean_it, "max_kkt": float(kk.max()),
                "max_kkt_status1": float(kkn[stn == 1].max()) if (stn == 1).any() else None,
                "status2_kkt": {"count": int(len(k2)), "max": float(k2[0]) if len(k2) else None,
                                "values": [float(v) for v in k2[:40]],
                                "over_1e-6": int((k2 > 1e-6).sum())},
                "status_counts": {int(a): int(b) for a, b in zip(*np.unique(stn, return_counts=True))},
                "roofline": {"kernel": f"mpc_riccati_kernel<Cfg<2,6,3,6,GR{',F32' if fp32 else ''}>>",
                             "bound": "latency", "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
                             "traffic": traffic, "traffic_source": src, "kernel_ms_per_launch": kern,
                             "alg_flops_per_qp": flops, "counters": sq_profile(kind)}}
        if fp32:
            line["fp32_vs_fp64"] = fp32_vs_fp64(R)
            line["dtype"] = "f32 factorisation / f64 residuals"
        else:
            line["dtype"] = "f64"
        out["fp32" if fp32 else "fp64"] = line
        del R
    out["fp32_over_fp64"] = out["fp32"]["value"] / out["fp64"]["value"]
    return out


def sq_profile(kind):
    """The solver kernel's wave-time shares from the newest committed SQ counter summary
    (profiles/sq_{kind}_r*.json, tools/pmc_sq.sh + tools/prof_summary.py sq): instruction issue
    (active_inst_any, of which VALU), s_waitcnt waits (wait_any), dependency / pipe stalls
    (wait_inst_any) and MFMA busy — the evidence for the `bound` label.  "stale": whether the kernel
    sources changed since the counters were taken."""
    import glob

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from prof_summary import solver_sources_sha

    path, rec = select_profile(glob.glob(os.path.join(ROOT, "profiles", f"sq_{kind}_r*.json")), solver_sources_sha())
    if rec is None:
        return None
    sha = rec.get("sources_sha")
    out = dict(rec.get("fractions_of_wave_time", {}))
    out.update({"valu_insts_per_wave": rec.get("per_wave", {}).get("valu_insts"),
                "source": os.path.relpath(path, ROOT), "commit": rec.get("commit"),
                "stale": None if sha is None else sha != solver_sources_sha()})
    return out


def select_profile(files, sha_now):
    """The committed counter summary that describes the current kernels: a record whose
    `sources_sha` equals the current sources' wins; among equals the one taken last (`taken_unix`,
    written by tools/prof_summary.py since round 6), then the file name.  (The file name alone
    misorders: a round-5 `sq_cfg5_r05sq.json` sorts after the newer `sq_cfg5_r05am.json`.)"""
    best, best_key = (None, None), None
    for path in files:
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        key = (rec.get("sources_sha") == sha_now, float(rec.get("taken_unix") or 0.0), os.path.basename(path))
        if best_key is None or key > best_key:
            best, best_key = (path, rec), key
    return best


def reference_config(ctx, reps=10, cpu=True):
    """The reference's own shipped configuration, timed beside its recorded number: N = 125,
    3 agents on the Highway map (planner/scripts/config_files/config_LPV.py:13-24), through the
    PlannerLPV drop-in (host arrays in and out, LPV scheduling + planes + QP build + the
    stage-wise Riccati IPM on the GPU).  Inputs: the reference-captured steps 0 and 1 of
    tests/golden/lpv_n125_a3.npz; map table tests/golden/track_highway.npz.  The reference
    records 111.9 ms per agent solve on an i7-13700H
    (experiments_paper/LPV3r_agent_laptop/settings.csv), its agents solved one after another."""
    import types

    import cmpc

    gold = os.path.join(ROOT, "tests", "golden")
    d = np.load(os.path.join(gold, "lpv_n125_a3.npz"), allow_pickle=False)
    t = np.load(os.path.join(gold, "track_highway.npz"), allow_pickle=False)
    track = types.SimpleNamespace(PointAndTangent=t["PointAndTangent"], halfWidth=t["halfWidth"], lane=int(t["lane"]))
    # config_LPV.py:6-11 gains; "SCALED CAR" model and limits (base_class.py:20-41)
    Q = np.diag([10.0, 0.0, 0.0, 25.0, 10.0, 0.0, 0.0, 0.0, 0.0])
    model = dict(lf=0.125, lr=0.125, m=1.98, I=0.09, Cf=70.0, Cr=70.0, mu=0.05)
    lim = dict(vx_ref=float(d["vx_ref"]), min_dist=0.25, max_vel=5.5, min_vel=0.0, max_rs=0.3, max_ls=0.3,
               max_ac=5.0, max_dc=10.0, sm=0.9)
    N = int(d["N"])
    bp = cmpc.PlannerLPVBatch(Q, 1e7 * np.eye(3), 0.0 * np.eye(2), 50.0 * np.eye(2), N, float(d["dt"]), track, 5.0,
                              model, lim, ctx=ctx)
    steps = []
    for step in sorted(set(d["step"].tolist())):
        sel = [j for j in range(len(d["step"])) if d["step"][j] == step]
        args = (d["x0"][sel], np.stack([d[f"x_last_{j}"] for j in sel]), np.stack([d[f"u_last_{j}"] for j in sel]),
                d["u_old"][sel], d["x_agents"][sel], d["pose"][sel])
        res = bp.solve(*args)
        t0 = time.perf_counter()
        for _ in range(reps):
            res = bp.solve(*args)
        ms = (time.perf_counter() - t0) / reps * 1e3
        row = {"step": int(step), "agents": len(sel), "ms_per_step": ms,
               "ipm_iters": res["iters"].tolist(), "status": res["status"].tolist(),
               "max_abs_err_vs_certified_optimum": float(np.abs(res["z"] - d["z"][sel]).max())}
        if cpu:
            row["cpu"] = reference_config_cpu(bp, args, res, d["z"][sel])
        steps.append(row)
    ref_ms = 111.9
    worst = max(s_["ms_per_step"] for s_ in steps)
    out = {"workload": "reference config_LPV.py: N=125, 3 agents, Highway, nx=9 nu=2 nb=2, fp64 (PlannerLPV drop-in, "
                       "host arrays)", "steps": steps,
           "reference_ms_per_agent_solve": ref_ms, "reference_ms_per_step_3_agents_sequential": 3 * ref_ms,
           "speedup_vs_reference_step": 3 * ref_ms / worst, "reps": reps}
    if cpu:
        model_name, nproc, usable = host_cpu()
        out["cpu_baseline"] = {
            "kind": "port", "cores": 1, "cpu_model": model_name, "nproc": nproc,
            "ms_per_step_sequential": [sum(s_["cpu"]["ms_per_agent"]) for s_ in steps],
            "sample": "the same six N=125 agent-QPs (GPU builder's problems read back), solved one after another on "
                      "one core by oracle/cmpc_oracle.c with the stage-wise Riccati method in the kernel's "
                      "double-double mode (newton 3, the method the GPU runs at this horizon), best of 3"}
    return out


def reference_config_cpu(bp, args, res, z_cert):
    """One control step of the reference configuration on the host: the structured problems the GPU
    builder made (read back), each agent solved by the C restatement of the same stage-wise Riccati
    method (oracle/cmpc_oracle.c, newton 3) on one thread, as the reference solves its agents one
    after another; per-agent wall time (best of 3) and z against the certified optimum and the GPU."""
    from oracle import cmpc_oracle as CO

    x0, x_last, u_last, u_old, x_agents, pose = args
    b = bp.build(x_last, u_last, x_agents, pose)
    prm, nb = bp.prm, x_agents.shape[2]
    ms, errs, errg, st = [], [], [], []
    for a in range(x0.shape[0]):
        P = dict(nx=9, nu=2, N=bp.N, ns=3, mc=4 + nb, Q=np.array(prm.Q[:]).reshape(9, 9),
                 R=np.array(prm.R[:]).reshape(2, 2), dR=np.array(prm.dR[:]).reshape(2, 2), Qs=np.array(prm.Qs[:]),
                 u_ub=np.array([prm.max_rs, prm.max_ac]), u_lb=np.array([-prm.max_ls, -prm.max_dc]),
                 row_slack=np.array([-1, 0, 1, 1] + [2] * nb), row_sign=np.array([1, 1, 1, 1] + [-1] * nb),
                 **{k: b[k][a:a + 1] for k in ("A", "B", "qlin", "C", "h")}, x0=x0[a:a + 1], u_prev=u_old[a:a + 1])
        best = np.inf
        for _ in range(3):
            t0 = time.perf_counter()
            zc, _, _, sc = CO.solve_batch(P, nthreads=1, newton=3)
            best = min(best, time.perf_counter() - t0)
        ms.append(best * 1e3)
        st.append(int(sc[0]))
        errs.append(float(np.abs(zc[0] - z_cert[a]).max()))
        errg.append(float(np.abs(zc[0] - res["z"][a]).max()))
    return {"ms_per_agent": ms, "status": st, "max_abs_err_vs_certified_optimum": max(errs),
            "max_abs_err_vs_gpu": max(errg)}


def lpv_population(ctx, replicas=341, rescue=True, finish=False, riccati=False):
    """The population of the `lpv_rounds` line: `replicas` copies of the reference's 3-agent
    Highway scenario at its captured step 0 (tests/golden/lpv_n30_a3: x0, Last_xPredicted, uPred,
    OldSteering/OldAccelera, positions), each copy's initial v_x scaled by a seeded factor in
    [0.98, 1.02]; an agent's neighbours are the other two agents of its copy
    (LPV_HP_N_main.py:82-85).  Returns (PlannerLPVBatch, LPVRounds constructor arguments)."""
    import types

    import cmpc
    from cmpc import _lib as L

    d = np.load(os.path.join(ROOT, "tests", "golden", "lpv_n30_a3.npz"), allow_pickle=False)
    t = np.load(os.path.join(ROOT, "tests", "golden", "track_highway.npz"), allow_pickle=False)
    track = types.SimpleNamespace(PointAndTangent=t["PointAndTangent"], halfWidth=t["halfWidth"], lane=int(t["lane"]))
    N, dt = int(d["N"]), float(d["dt"])
    sel = [j for j in range(len(d["step"])) if d["step"][j] == 0]
    order = np.argsort(d["agent"][sel])
    sel = [sel[i] for i in order]
    x0 = np.tile(d["x0"][sel], (replicas, 1))
    x0[:, 0] *= np.repeat(1.0 + 0.02 * np.random.default_rng(5).uniform(-1, 1, replicas), 3)
    x_last = np.tile(np.stack([d[f"x_last_{j}"] for j in sel]), (replicas, 1, 1))
    u_last = np.tile(np.stack([d[f"u_last_{j}"] for j in sel]), (replicas, 1, 1))
    u_old = np.tile(d["u_old"][sel], (replicas, 1))
    traj = np.tile(d["pose"][sel], (replicas, 1, 1))
    g = np.arange(3 * replicas) // 3 * 3
    nbr = np.stack([g + (np.arange(3 * replicas) + 1) % 3, g + (np.arange(3 * replicas) + 2) % 3], 1)
    nbr = np.sort(nbr, 1)   # the reference's ns[i]: the other agents in index order
    Q = np.diag([10.0, 0.0, 0.0, 25.0, 10.0, 0.0, 0.0, 0.0, 0.0])
    model = dict(lf=0.125, lr=0.125, m=1.98, I=0.09, Cf=70.0, Cr=70.0, mu=0.05)
    lim = dict(vx_ref=float(d["vx_ref"]), min_dist=0.25, max_vel=5.5, min_vel=0.0, max_rs=0.3, max_ls=0.3,
               max_ac=5.0, max_dc=10.0, sm=0.9)
    bp = cmpc.PlannerLPVBatch(Q, 1e7 * np.eye(3), 0.0 * np.eye(2), 50.0 * np.eye(2), N, dt, track, 5.0, model, lim,
                              ctx=ctx)
    if riccati:
        bp.opts = L.opts(flags=L.CMPC_FLAG_RICCATI)
    elif not rescue:
        bp.opts = L.opts()
    elif finish:
        bp.opts = L.opts(flags=L.CMPC_FLAG_RESCUE | L.CMPC_FLAG_FINISH)
    return bp, (x0, x_last, u_last, nbr), dict(u_old=u_old, traj=traj)


def lpv_check_round(bp, R, sample):
    """The current round's problems of the `sample` agents (the GPU builder's A, B, qlin, C, h,
    read back) solved by the C restatement with the product's rescue policy
    (oracle.cmpc_oracle.solve_batch_rescue); returns (z_cpu, status_cpu) of the sample."""
    from oracle import cmpc_oracle as CO

    rows = R.last_rows
    xl = R.x_last.cpu().numpy().reshape(-1)[: R.B * rows * 9].reshape(R.B, rows, 9)[sample]
    b = bp.build(xl, R.u_last.cpu().numpy()[sample], R.x_agents.cpu().numpy()[sample], R.pose.cpu().numpy()[sample])
    prm = bp.prm
    P = dict(nx=9, nu=2, N=bp.N, ns=3, mc=4 + R.nb, Q=np.array(prm.Q[:]).reshape(9, 9), R=np.array(prm.R[:]).reshape(2, 2),
             dR=np.array(prm.dR[:]).reshape(2, 2), Qs=np.array(prm.Qs[:]), u_ub=np.array([prm.max_rs, prm.max_ac]),
             u_lb=np.array([-prm.max_ls, -prm.max_dc]), row_slack=np.array([-1, 0, 1, 1] + [2] * R.nb),
             row_sign=np.array([1, 1, 1, 1] + [-1] * R.nb), A=b["A"], B=b["B"], x0=R.x0.cpu().numpy()[sample],
             u_prev=R.u_old.cpu().numpy()[sample], qlin=b["qlin"], C=b["C"], h=b["h"])
    finish = bool(bp.opts.flags & 64)   # CMPC_FLAG_FINISH
    polish = bool(bp.opts.flags & 256)  # CMPC_FLAG_POLISH
    amax = None
    if polish:  # the polish kernel's active-set capacity for this shape (both sides polish the same agents)
        from cmpc.solver import plan

        amax = plan(P, 1, rescue=True, polish=True)["polish_max_active"]
    zc, _, _, sc = CO.solve_batch_rescue(P, nthreads=min(16, os.cpu_count() or 1), finish=finish, polish=polish,
                                         polish_amax=amax)
    return zc, sc, P


def reference_certificate(P, a, z):
    """Reference-form (OSQP-form, LPV_Planner.py:222-233) KKT residual of agent a's primal z with its
    best sign-feasible multipliers (oracle.qp_ipm.kkt_of_primal), and its objective value."""
    from oracle import qp_ipm
    from oracle import synth

    Pm, q, A, l, u = synth.reference_form(P, a)
    cert, _ = qp_ipm.kkt_of_primal(Pm, q, A, l, u, z)
    return max(cert["stat_rel"], cert["prim"], cert["comp"]), float(0.5 * z @ Pm @ z + q @ z)


def lpv_rounds(ctx, replicas=341, rounds=20, warmup=2, rescue=True, check=True, sample=128, finish=False,
               riccati=False):
    """The reference's own agent model in device-resident consensus rounds (cmpc.rounds.LPVRounds:
    gather -> LPV scheduling + planes + QP build + solve -> advance -> exchange, all in HBM), at
    N = 30 (nx 9, nu 2, 2 neighbours: the v3 kernel), on lpv_population's 1023 agents.  Timed
    over `rounds` rounds after `warmup`; then (``check``) the same rounds are replayed from the
    start (the GPU path is deterministic) and each round's `sample` seeded agents are re-solved by
    the C restatement with the same rescue policy: max |z - z_cpu| over the agents both solve to
    tolerance, and the max scaled KKT residual over every agent of every round."""
    import torch

    from cmpc.rounds import LPVRounds

    bp, args, kw = lpv_population(ctx, replicas, rescue, finish, riccati)
    N = bp.N
    R = LPVRounds(bp, *args, **kw)
    dev = R.dev
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(rounds)]
    for _ in range(warmup):
        R.step(halt=False)
    torch.cuda.synchronize(dev)
    st, it, kk = [], [], []
    t0 = time.perf_counter()
    for k in range(rounds):
        R.step(timer=ev[k], halt=False)   # (no per-round host check: the statuses are tallied after the loop)
        st.append(R.status.clone())
        it.append(R.iters.clone())
        kk.append(R.kkt.clone())
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    st = torch.stack(st).cpu().numpy()
    it = torch.stack(it).cpu().numpy()
    kk = torch.stack(kk).cpu().numpy()
    B = 3 * replicas
    out = {"workload": f"device-resident LPV rounds: {B} agents ({replicas} copies of the reference's 3-agent "
                       f"Highway scenario, lpv_n30_a3 step 0, v_x0 x U[0.98, 1.02]), N={N}, nx=9 nu=2 nb=2, fp64; "
                       f"round = gather + LPV build + solve + advance + exchange",
           "agent_qp_per_s": B * rounds / el, "ms_per_round": el / rounds * 1e3,
           "build_solve_ms": sum(a.elapsed_time(b) for a, b in ev) / rounds, "rounds": rounds, "warmup": warmup,
           "rescue": rescue, "finish": finish, "riccati": riccati, "polish": bool(bp.opts.flags & 256), "mean_ipm_iters": float(it.mean()), "max_ipm_iters": int(it.max()),
           "max_ipm_iters_per_round": it.max(1).tolist(), "max_kkt": float(kk.max()),
           "status_counts": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}}
    if check:
        R = LPVRounds(bp, *args, **kw)
        rng = np.random.default_rng(11)
        err, err_nd, both, n = 0.0, 0.0, 0, 0
        # agents both sides solve whose z differ by more than 1e-6: an interior-point endpoint against a
        # polished one on a degenerate optimum (a weakly active row: the IPM approaches it like sqrt(mu));
        # each is certified in addition by the GPU point's reference-form KKT residual and objective, and
        # counted; max_abs_err_vs_cpu stays over every both-solved agent
        deg = {"count": 0, "max_ref_kkt_gpu": 0.0, "max_ref_kkt_cpu": 0.0, "max_obj_gap_rel": -np.inf,
               "max_abs_err": 0.0}
        for k in range(warmup + rounds):
            R.gather()
            R.solve()
            torch.cuda.synchronize(dev)
            if k >= warmup:
                smp = np.sort(rng.choice(B, sample, replace=False))
                zc, sc, Pc = lpv_check_round(bp, R, smp)
                zg, sg = R.z.cpu().numpy()[smp], R.status.cpu().numpy()[smp]
                ok = (sc == 1) & (sg == 1)
                e = np.abs(zg - zc).max(1)
                if ok.any():
                    err = max(err, float(e[ok].max()))
                for a in np.flatnonzero(ok & (e > 1e-6)):
                    kg, fg = reference_certificate(Pc, a, zg[a])
                    kc, fc = reference_certificate(Pc, a, zc[a])
                    deg["count"] += 1
                    deg["max_ref_kkt_gpu"] = max(deg["max_ref_kkt_gpu"], kg)
                    deg["max_ref_kkt_cpu"] = max(deg["max_ref_kkt_cpu"], kc)
                    deg["max_obj_gap_rel"] = max(deg["max_obj_gap_rel"], (fg - fc) / max(1.0, abs(fc)))
                    deg["max_abs_err"] = max(deg["max_abs_err"], float(e[a]))
                    ok[a] = False
                if ok.any():
                    err_nd = max(err_nd, float(e[ok].max()))
                both += int(((sc == 1) & (sg == 1)).sum())
                n += sample
            R.advance()
            R.exchange()
        out["oracle_sample"] = {"agents_per_round": sample, "checked": n, "both_solved": both,
                                "max_abs_err_vs_cpu": err, "max_abs_err_vs_cpu_non_degenerate": err_nd,
                                "degenerate": deg}
    return out


def osqp_dropin(ctx, reps=20, cpu=True):
    """The literal reference boundary, osqp_solve_qp(P, q, G, h, A, b) (LPV_Planner.py:192-249),
    timed on the reference-captured N=30 QPs of tests/golden/lpv_n30_a3.npz (3 agents, several
    closed-loop steps): csr matrices in, (res, feasible) out, as PlannerLPV.solve calls it
    (LPV_Planner.py:156-157).  One call per QP (host arrays, structure recognition, one
    structured launch each) and all QPs in one osqp_solve_qp_batch call; z against the
    KKT-certified optimum."""
    import scipy.sparse as sp

    import cmpc

    d = np.load(os.path.join(ROOT, "tests", "golden", "lpv_n30_a3.npz"), allow_pickle=False)

    def mat(nm, j):
        shp = tuple(int(v) for v in d[f"{nm}_{j}_shape"])
        return sp.csr_matrix((d[f"{nm}_{j}_data"], (d[f"{nm}_{j}_row"], d[f"{nm}_{j}_col"])), shape=shp)

    qps = []
    for j in range(len(d["step"])):
        Aall, l, u = mat("A", j), d["l"][j], d["u"][j]
        eq = np.isfinite(l) & (l == u)
        qps.append((mat("P", j), d["q"][j], Aall[np.flatnonzero(~eq)], u[~eq], Aall[np.flatnonzero(eq)], u[eq]))
    out = [cmpc.osqp_solve_qp(*qp, ctx=ctx) for qp in qps]
    t0 = time.perf_counter()
    for _ in range(reps):
        out = [cmpc.osqp_solve_qp(*qp, ctx=ctx) for qp in qps]
    one_ms = (time.perf_counter() - t0) / (reps * len(qps)) * 1e3
    cmpc.osqp_solve_qp_batch(qps, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(reps):
        bat = cmpc.osqp_solve_qp_batch(qps, ctx=ctx)
    bat_ms = (time.perf_counter() - t0) / reps * 1e3
    err = max(float(np.abs(r.x - d["z"][j]).max()) for j, (r, _) in enumerate(out))
    berr = max(float(np.abs(r.x - d["z"][j]).max()) for j, (r, _) in enumerate(bat))
    res = {"workload": f"osqp_solve_qp drop-in on the {len(qps)} reference-captured N=30 agent QPs of "
                       f"lpv_n30_a3 (nx=9 nu=2, n={qps[0][0].shape[0]} vars, "
                       f"{qps[0][2].shape[0] + qps[0][4].shape[0]} rows, csr in)",
           "ms_per_call": one_ms, "batch_call_ms": bat_ms, "qps": len(qps),
           "status_val": sorted({int(r.info.status_val) for r, _ in out}),
           "max_kkt": max(float(r.info.kkt) for r, _ in out),
           "max_abs_err_vs_certified_optimum": err, "batch_max_abs_err_vs_certified_optimum": berr,
           "reps": reps}
    if cpu:
        res["cpu"] = osqp_dropin_cpu(qps, d["z"])
    return res


def osqp_dropin_cpu(qps, z_cert, reps=3):
    """The CPU figure beside the literal boundary: each of the same QPs, recognised into the structured
    form the GPU path solves (cmpc.structure.recognize), solved by the C restatement of the same
    policy (oracle/cmpc_oracle.c: the condensed IPM, rescue hand-over and polish; solve_batch_rescue) on
    ONE thread, one QP after another as PlannerLPV.solve calls osqp_solve_qp; per-QP wall time, best of
    `reps` (the recognition is the GPU call's too and is not timed here)."""
    from cmpc import structure as St
    from cmpc.solver import plan
    from oracle import cmpc_oracle as CO

    ms, errs, st = [], [], []
    for j, qp in enumerate(qps):
        P = St.recognize(*qp[:6])
        amax = plan(P, 1, rescue=True, polish=True)["polish_max_active"]
        best = np.inf
        for _ in range(reps):
            t0 = time.perf_counter()
            zc, _, _, sc = CO.solve_batch_rescue(P, nthreads=1, polish=True, polish_amax=amax)
            best = min(best, time.perf_counter() - t0)
        ms.append(best * 1e3)
        st.append(int(sc[0]))
        errs.append(float(np.abs(zc[0] - z_cert[j]).max()))
    model_name, nproc, _ = host_cpu()
    return {"kind": "port", "cores": 1, "cpu_model": model_name, "nproc": nproc,
            "ms_per_call_mean": float(np.mean(ms)), "ms_per_call_max": float(np.max(ms)), "status": sorted(set(st)),
            "max_abs_err_vs_certified_optimum": max(errs),
            "sample": "the same QPs in structured form, the C restatement (rescue + polish policy) on one thread, "
                      "best of 3 per QP"}


def fp32_vs_fp64(R):
    """BASELINE cfg5's tolerance check of the fp32 path: the next round's problem solved by the fp32
    path (this DIRounds) and by the fp64 stage-wise Riccati kernel, every agent: statuses and the
    largest |z32 - z64| / max(1, |z64|)."""
    import torch

    import cmpc

    R.build()
    R.solve()
    torch.cuda.synchronize()
    z32, st32 = R.z.cpu().numpy().copy(), R.status.cpu().numpy().copy()
    p = R.snapshot()
    z64, _, _, st64 = cmpc.solve_mpc(p, R.ctx, riccati=True)
    err = np.abs(z32 - z64) / np.maximum(1.0, np.abs(z64))
    both = (st32 == cmpc.CMPC_SOLVED) & (st64 == cmpc.CMPC_SOLVED)
    return {"agents": int(len(st32)), "fp32_solved": float(np.mean(st32 == cmpc.CMPC_SOLVED)),
            "fp32_status_counts": {int(k): int(v) for k, v in zip(*np.unique(st32, return_counts=True))},
            "fp64_solved": float(np.mean(st64 == cmpc.CMPC_SOLVED)),
            "max_rel_err": float(err.max()), "p99_rel_err": float(np.quantile(err.max(1), 0.99)),
            "max_rel_err_both_solved": float(err[both].max()) if both.any() else None,
            "reference": "fp64 stage-wise Riccati kernel (double-double near the solution), same problems"}


def pmc_traffic(kind=None):
    """HBM bytes per solver launch from the newest committed PMC summary (profiles/pmc_r*.json;
    cfg5 lines: profiles/pmc_{kind}_r*.json,
    FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes, tools/prof_summary.py).  PMC
    counters cannot be collected inside this process, so the figure carries its provenance:
    the commit it was measured at, and "stale" = whether the kernel sources (sha256 over
    csrc/ and cmpc.h) differ from the ones that were profiled."""
    import glob

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from prof_summary import solver_sources_sha

    path, rec = select_profile(glob.glob(os.path.join(ROOT, "profiles", f"pmc_{kind}_r*.json" if kind else "pmc_r*.json")),
                               solver_sources_sha())
    if rec is None:
        return None, None
    traffic = rec.get("solve_kernel", {}).get("hbm_bytes_per_launch")
    sha = rec.get("sources_sha")
    return traffic, {"file": os.path.relpath(path, ROOT), "commit": rec.get("commit"),
                     "stale": None if sha is None else sha != solver_sources_sha()}


def host_cpu():
    """(model name, nproc, usable CPUs) of this host."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    return model, nproc, usable


def cpu_baseline(R, seconds, rounds=4, newton=0, label="cfg3"):
    """The oracle's plain-C restatement (oracle/cmpc_oracle.c, OpenMP, one agent-QP per
    thread) timed on this host over whole rounds of the SAME workload the GPU solves:
    `rounds` consecutive consensus rounds are built and solved on the device, each round's
    full structured problem (every agent of this rank) is copied to the host, and the CPU
    solves all of them, repeated until about `seconds` of CPU time.  Threads: every CPU this
    process may use, capped by OMP_NUM_THREADS when it is set (the GPU box grants each job a
    16-CPU share of a larger host, so nproc there is not the usable count).  `newton` selects the
    restated method: 0 the condensed IPM of the v3 kernel (cfg3), 3 the stage-wise Riccati IPM
    with the kernel's double-double mode (cfg5)."""
    import torch

    from oracle import cmpc_oracle as CO

    model, nproc, usable = host_cpu()
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(usable, env) if env > 0 else usable
    probs, zs = [], []
    for _ in range(rounds):
        R.build()
        probs.append(R.snapshot())
        R.solve()
        torch.cuda.synchronize()
        zs.append(R.z.cpu().numpy().copy())
        R.advance()
        R.exchange()
    B = probs[0]["A"].shape[0]
    err = 0.0
    t = time.perf_counter()
    passes = 0
    while True:
        for p, zg in zip(probs, zs):
            zc, _, _, _ = CO.solve_batch(p, nthreads=threads, newton=newton)
            if passes == 0:
                err = max(err, float(np.abs(zg - zc).max()))
        passes += 1
        el = time.perf_counter() - t
        if el >= seconds:
            break
    solved = passes * rounds * B
    return ({"value": solved / el, "unit": "agent-QP/s", "cores": threads, "kind": "port",
             "nproc": nproc, "cpu_model": model,
             "cores_note": f"{threads}-thread job share (affinity mask) of a {nproc}-thread host: a baseline "
                           f"against those threads, not against the whole node",
             "sample": f"{passes} pass(es) over {rounds} consecutive full {label} rounds of {B} agents "
                       f"(device-built problems copied to the host), oracle/cmpc_oracle.c fp64, OpenMP "
                       f"{threads} threads, {el:.1f} s"}, err)


if __name__ == "__main__":
    main()
