#!/usr/bin/env python3
"""MIDASPOM posterior-grid benchmark (BASELINE.json metric).

A "step" = one pass of the hot path over one (e, c) grid slab per rank: the
per-c coefficient kernels plus the forward-recursion kernel over every grid
point.  Grid points are independent, so steps need no exchange; with N > 1
ranks the job's single RCCL gather of the log-likelihood slabs to rank 0
(main_MIDASPOM_MPI.c:482-506) runs once, after the last step, inside the
timed region.  Units = grid points x year transitions = s^2 (tmax - 1) per
rank; value = units over all ranks / max-over-ranks wall time (weak scaling:
each rank owns an s x s slab of an (N s) x s grid).
Other modes: --config 3 (256 x 200, 1024^2), --config 4 (dieoff 256^3),
--config 5 (future, 10^6 replicates), --config 6 (a 200-year survey with
~4 states a year: the chunked forward path); --backend gloo rehearses N
ranks on fewer GPUs (collectives through host memory).

Workload: 64 patches x 50 years (synthetic,
Appendix C generator, md5-checked), 512 x 512 grid, -m 400 -d 100, FP64.
Launch:  python bench.py [--gpus N --steps K --warmup W]   (N > 1: starts N ranks itself)
         torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import subprocess
import tempfile
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import midaspom_amd as mdp  # noqa: E402
from midaspom_amd import synth  # noqa: E402

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (= FP64 matrix) peak, AMD datasheet
HBM_PEAK_GBS = 8000.0
LOG_DBL_MIN = float(np.log(np.finfo(np.float64).tiny))

CONFIGS = {
    2: dict(gen=synth.CONFIG2, s=512, name="config2: 64 patches x 50 years, 512x512 (e,c) grid"),
    3: dict(gen=synth.CONFIG3, s=1024, name="config3: 256 patches x 200 years, 1024x1024 (e,c) grid"),
    # not a BASELINE config: a 200-year survey with ~4 states a year (3 086
    # forward uses, past one specialised kernel: the chunked forward path)
    6: dict(gen=synth.LONG200, s=1024, name="long200: 64 patches x 200 years, 20% unvisited, 1024x1024 (e,c) grid"),
}


def _pmc_traffic(cfg):
    """HBM bytes per launch of the config's dominant kernel from the committed
    rocprofv3 PMC passes (scripts/gpu_measure.sh, scripts/pmc_traffic.py):
    FETCH_SIZE x2 + WRITE_SIZE; null when no profile of this config exists."""
    tf = ROOT / "profiles" / f"pmc_traffic_cfg{cfg}.json"
    if not tf.exists():
        return {"traffic": None}
    return {"traffic": json.loads(tf.read_text())["hbm_bytes_per_launch"],
            "traffic_unit": "bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": str(tf.relative_to(ROOT))}


def host_info():
    """The host's CPUs as SURVEY §8(d) asks them stated: the model, logical
    CPUs and physical cores of the machine, the CPUs this process may run on
    (affinity) and the CPU time it may use (the cgroup quota: on the GPU
    pool a one-GPU job gets 16 CPUs' worth of a 2 x 64-core EPYC, whatever
    its affinity says)."""
    model, phys = "unknown", set()
    try:
        cur = {}
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name") and model == "unknown":
                model = ln.split(":", 1)[1].strip()
            elif ln.startswith("physical id"):
                cur["p"] = ln.split(":", 1)[1].strip()
            elif ln.startswith("core id"):
                phys.add((cur.get("p"), ln.split(":", 1)[1].strip()))
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count() or 1, "logical_cpus": os.cpu_count() or 1,
            "physical_cores": len(phys) or None, "usable_cores": usable, "cgroup_cpu_quota": quota,
            "cpu_model": model}


def _all_threads():
    """Every CPU this job can use: the affinity set, capped by the cgroup
    CPU quota (threads past the quota only time-share it)."""
    h = host_info()
    n = h["usable_cores"]
    if h["cgroup_cpu_quota"]:
        n = min(n, max(1, int(h["cgroup_cpu_quota"])))
    return max(1, n)


def _oracle_leg(om, g_e, g_c, lik_gpu, ltot_gpu, tmax, threads, budget_s, per_pt):
    """Time the oracle on an evenly strided sample of the grid sized for
    ~budget_s of wall on `threads` threads; parity of the GPU run there."""
    ne, nc = lik_gpu.shape
    npts = int(min(ne * nc, max(threads * 8, budget_s * threads / per_pt)))
    stride = max(1, int(np.ceil(np.sqrt(ne * nc / npts))))
    ee, cc = np.meshgrid(np.arange(0, ne, stride), np.arange(0, nc, stride), indexing="ij")
    ee, cc = ee.ravel(), cc.ravel()
    t0 = time.perf_counter()
    ref = om.loglik_points(g_e[ee], g_c[cc], threads=threads)
    wall = time.perf_counter() - t0
    got = lik_gpu[ee, cc]
    with np.errstate(invalid="ignore", over="ignore"):
        pg, pr = np.exp(got - ltot_gpu), np.exp(ref - ltot_gpu)
    fin = np.isfinite(pr) & np.isfinite(pg)
    big = fin & (pr > 1e-14)
    fl = (got >= LOG_DBL_MIN) & (ref >= LOG_DBL_MIN)
    parity = {"max_abs_dposterior": float(np.abs(pg[fin] - pr[fin]).max()) if fin.any() else 0.0,
              "max_rel_dposterior": float((np.abs(pg[big] - pr[big]) / pr[big]).max()) if big.any() else 0.0,
              "max_abs_dloglik": float(np.abs(got[fl] - ref[fl]).max()) if fl.any() else 0.0,
              "points_checked": int(ee.size),
              # L subnormal or 0 (log L < log DBL_MIN) at the same points: in
              # that range two summation orders round differently (the tests'
              # rule, tests/test_gpu_parity.py assert_loglik_close)
              "underflow_positions_match": bool(np.array_equal(got < LOG_DBL_MIN, ref < LOG_DBL_MIN))}
    return {"value": ee.size * (tmax - 1) / wall, "cores": threads, "wall_s": wall,
            "sample": f"{ee.size} grid points (every {stride}th e and c of the {ne}x{nc} grid)"}, parity


def cli_walls(cfg_inputs, tmpdir):
    """End-to-end wall time of the drop-in CLI (parse -> hipRTC -> grid -> Ltot
    -> write; main_MIDASPOM.c:330,437-439 time the same span) with cold
    (fresh) caches, on the first run with caches on, and warm (steady state),
    and of the oracle's own CLI
    (the reference formulation, naive dgemm, 1 core) on config 1."""
    from midaspom_amd import _lib
    out = {}
    cache = Path(tempfile.mkdtemp(prefix="mdp_jitcache_", dir=tmpdir))
    for name, (inp, s) in cfg_inputs.items():
        for leg in ("cold", "warm_first", "warm"):
            # cold: an empty code-object cache and no compiler-side cache
            # (ROCm's comgr keeps its own, which this process has warmed).
            # warm_first: the first run with both caches on.  Besides our
            # code object, the HIP runtime's own first kernel launch goes
            # through comgr, 0.15 s with its cache cold even for a one-kernel
            # program (scripts/ubench/tiny_launch, scripts/jitcache_probe.py),
            # and comgr's cache keeps that across processes: warm is the
            # steady state after it
            env = dict(os.environ, MDP_JIT_CACHE=str(cache / name), MIDASPOM_TIMING="1",
                       **({"AMD_COMGR_CACHE": "0"} if leg == "cold" else {}))
            t0 = time.monotonic()
            r = subprocess.run([str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", str(s), "-i", str(inp),
                                "-o", str(Path(tmpdir) / f"{name}.post")], env=env, capture_output=True, text=True)
            t1 = time.monotonic()
            out[f"{name}_cli_{leg}_s"] = t1 - t0 if r.returncode == 0 else None
            # the CLI's own split (MIDASPOM_TIMING): parse, HIP start-up,
            # engine set-up (hipRTC), grid, Ltot, write
            for ln in r.stderr.splitlines():
                if ln.startswith("midaspom timing (s):"):
                    v = ln.split(":", 1)[1].split()
                    out[f"{name}_cli_{leg}_split_s"] = {v[i]: float(v[i + 1]) for i in range(0, len(v) - 1, 2)}
                # main's entry and return on this process's clock (CLOCK_MONOTONIC):
                # the wall before main (spawn, exec, loader, library
                # constructors) and after it (exit handlers, runtime teardown)
                if ln.startswith("midaspom clock (s):"):
                    v = ln.split(":", 1)[1].split()
                    st = {v[i]: float(v[i + 1]) for i in range(0, len(v) - 1, 2)}
                    out[f"{name}_cli_{leg}_outside_s"] = {"before_main": st["main_entry"] - t0,
                                                          "after_main": t1 - st["main_return"]}
    orc = ROOT / "oracle" / "_build" / "orc_main"
    if orc.exists() and "config1" in cfg_inputs:
        inp, s = cfg_inputs["config1"]
        t0 = time.perf_counter()
        r = subprocess.run([str(orc), "-m", "400", "-d", "100", "-s", str(s), "-i", str(inp),
                            "-o", str(Path(tmpdir) / "orc.post")], capture_output=True,
                           env=dict(os.environ, OMP_NUM_THREADS="1"))
        out["config1_oracle_cli_1core_s"] = time.perf_counter() - t0 if r.returncode == 0 else None
    return out


def e2e_walls(input_path, tmpdir):
    """cli_walls on configs 1-3 (the config-2 input is the bench's own)."""
    cfg1 = ROOT / "tests" / "golden" / "occupancies.txt"
    return cli_walls({"config1": (cfg1, 50), "config2": (input_path, 512),
                      "config3": (synth.write(Path(tmpdir) / "config3.txt", **synth.CONFIG3), 1024)}, tmpdir)


def cpu_baseline(input_path, g_e, g_c, lik_gpu, ltot_gpu, tmax, tmpdir, budget_s=10.0, end_to_end=None):
    """The oracle (oracle/spom_oracle.c: the reference's dense CBLAS
    formulation restated in C with a naive row-major dgemm) on the host
    cores: a 1-core leg and an all-cores leg over bounded strided samples of
    the same grid, plus end-to-end CLI walls (configs 1 and 2)."""
    import oracle
    om = oracle.OracleModel.load(input_path, 400.0, 0.5, 100.0)
    t0 = time.perf_counter()
    om.loglik_points(g_e[:4], g_c[:4], threads=1)
    per_pt = (time.perf_counter() - t0) / 4
    threads = _all_threads()
    one, _ = _oracle_leg(om, g_e, g_c, lik_gpu, ltot_gpu, tmax, 1, budget_s, per_pt)
    allc, parity = _oracle_leg(om, g_e, g_c, lik_gpu, ltot_gpu, tmax, threads, budget_s, per_pt)
    cfg1 = ROOT / "tests" / "golden" / "occupancies.txt"
    hi = host_info()
    res = {
        "value": allc["value"], "unit": "grid-point-timestep evals/s", "cores": threads, "kind": "port",
        "sample": f"{allc['sample']}, {threads} threads (all this job may use: affinity {hi['usable_cores']}, "
                  f"cgroup quota {hi['cgroup_cpu_quota']} CPUs), {allc['wall_s']:.1f} s",
        "one_core": {"value": one["value"], "sample": f"{one['sample']}, 1 thread, {one['wall_s']:.1f} s"},
        # not measured: what the whole machine's physical cores would give at
        # the measured one-core rate (an upper estimate for a node-wide CPU run)
        "whole_host_estimate": {"value": one["value"] * (hi["physical_cores"] or 1),
                                "basis": f"one-core rate x {hi['physical_cores']} physical cores (extrapolated)"},
        "dgemm": "naive row-major triple loop (oracle/spom_oracle.c); the reference itself needs CBLAS, "
                 "which this image lacks (DESIGN.md §7)",
        **host_info(),
        "end_to_end": end_to_end if end_to_end is not None else e2e_walls(input_path, tmpdir),
    }
    return res, parity


def _coll_name(args):
    """The collective library a multi-rank line used: RCCL for the nccl
    backend (ROCm), else the rehearsal backend's own name."""
    return "RCCL" if args.backend == "nccl" else args.backend


def _coll_tensor(t, args):
    """The tensor a collective runs on: itself under RCCL, a host copy under
    a rehearsal backend (gloo moves host tensors only)."""
    return t if args.backend == "nccl" else t.cpu()


def bench_future(args, world, rank, dev):
    """Config 5: MIDASPOM_future on examples/input with the
    config-1 posterior (s = 101, computed by the GPU engine before timing),
    `-a 50 -m 400 -d 100`, 10^6 replicates split over the ranks (strong
    scaling) + one sum-reduce of the per-year counts over RCCL.  A step = the
    whole ensemble; units = replicate-years."""
    inp = ROOT / "tests" / "golden" / "occupancies.txt"
    tfut, nsim, seed = 50, args.replicates, 20161014
    post_lik, ltot = mdp.run_file(inp, None, m=400.0, d=100.0, s=101, devices=[dev.index])
    post = mdp.posterior(post_lik, ltot)
    _, _, row = mdp.read_survey(inp)
    fut = mdp.Future(row, post, m=400.0, d=100.0, device=dev.index)
    from midaspom_amd import dist as mdist
    r0, r1 = mdist.replicate_range(rank, world, nsim)
    counts = torch.zeros(tfut, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        fut.simulate_device(counts.data_ptr(), r1 - r0, tfut, seed=seed, rep0=r0, stream=stream)
        if world > 1:
            dist.reduce(_coll_tensor(counts, args), dst=0, op=dist.ReduceOp.SUM)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    fut.check(stream)  # no replicate overflowed the posterior look-back
    kms = fut.time_kernel(r1 - r0, tfut, seed=seed, reps=args.steps)
    if world > 1:
        t = _coll_tensor(torch.tensor([dt], dtype=torch.float64, device=dev), args)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # The kernel is bound by VALU issue (Philox4x32-10: 4 calls per
    # replicate-year, 19 v_mad_u64_u32 each), not by FP64.  Its roofline is
    # SIMD issue cycles: the VALU instructions per launch counted by
    # rocprofv3 per class (profiles/pmc_valu_cfg5.json) priced at their
    # measured issue cost (v_mad_u64_u32 8 cycles, FP64 4, 32-bit 2:
    # scripts/ubench/int_rates.hip, scripts/pmc_valu.py), against 256 CUs x
    # 4 SIMDs x 2.4 GHz.  The plain instruction count against one wave64
    # instruction per 2 cycles (what round 1 reported) and the FP64 work the
    # model itself needs (n^2 colonisation-sum adds + n source adds + n
    # products c*s1 per replicate-year, simpij future.c:64-110) are reported
    # beside it.
    n = row.size
    flop_per_ry = n * n + 2 * n + n
    issue_peak = 256 * 4 * 2.4e9 / 1e9  # G SIMD issue cycles/s
    valu_issue_peak = issue_peak / 2  # G wave-instructions/s at 2 cycles each
    achieved = insts = None
    valu_src = None
    vf = ROOT / "profiles" / "pmc_valu_cfg5.json"
    if vf.exists():
        pv = json.loads(vf.read_text())
        if pv.get("replicates") == r1 - r0 and pv.get("years") == tfut and "issue_cycles_per_launch" in pv:
            achieved = pv["issue_cycles_per_launch"] / (kms * 1e-3) / 1e9
            insts = pv["valu_insts_per_launch"] / (kms * 1e-3) / 1e9
            valu_src = str(vf.relative_to(ROOT))
    result = {
        "metric": "replicate-year simulations/sec (MIDASPOM_future ensemble)",
        "value": nsim * tfut * args.steps / dt,
        "unit": "replicate-years/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "examples/input (shipped), posterior from the GPU engine at s=101",
        "config": {"workload": "config5: MIDASPOM_future, 10^6 replicates x 50 years, examples/input",
                   "patches": int(n), "replicates": nsim, "years": tfut,
                   "parallelism": f"replicate ranges x{world}" + (f", {_coll_name(args)} reduce" if world > 1 else ""),
                   "backend": args.backend if world > 1 else None},
        "kernel_ms": {"k_future": kms},
        "roofline": {"kernel": "k_future", "bound": "valu-issue",
                     "compute_unit": "VALU issue cycles (Philox integer work), instructions priced by class",
                     "achieved": achieved, "peak": issue_peak, "unit": "G SIMD issue cycles/s",
                     "frac": achieved / issue_peak if achieved else None, **_pmc_traffic(5),
                     "valu_source": valu_src,
                     "valu_insts_rate": insts, "valu_insts_peak": valu_issue_peak,
                     "valu_insts_frac": insts / valu_issue_peak if insts else None,
                     "fp64_tflops": flop_per_ry * (r1 - r0) * tfut / (kms * 1e-3) / 1e12,
                     "flop_per_replicate_year": flop_per_ry},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        threads = _all_threads()
        t0 = time.perf_counter()
        oracle.future_counts(row, post, tfut=tfut, nrep=2000, m=400.0, d=100.0, seed=seed, threads=1)
        per = (time.perf_counter() - t0) / 2000
        nref = int(min(nsim, max(threads * 100, 12.0 * threads / per)))
        t0 = time.perf_counter()
        ref = oracle.future_counts(row, post, tfut=tfut, nrep=nref, m=400.0, d=100.0, seed=seed, threads=threads)
        wall = time.perf_counter() - t0
        got = fut.simulate(nref, tfut, seed=seed)
        result["cpu_baseline"] = {
            "value": nref * tfut / wall, "unit": "replicate-years/s", "cores": threads, "kind": "port",
            "sample": f"replicates [0, {nref}) of the same stream, oracle/spom_future_oracle.c, {threads} threads, "
                      f"{wall:.1f} s"}
        result["parity"] = {"replicates_checked": nref, "counts_identical": bool(np.array_equal(got, ref))}
    fut.close()
    return result


def bench_dieoff(args, world, rank, dev):
    """Config 4: MIDASPOM_dieoff likelihood over a 3-D
    (e, c, K_D) = 256^3 grid -- e, c on [0, 1], K_D log-spaced on [0.1, 100]
    -- for the first survey row of examples/input (n = 8, 2^8 states),
    `-b 20 -a 10 -m 400 -d 100`.  The e rows are split into contiguous slabs
    over the ranks (strong scaling: the grid is fixed) and gathered to rank 0
    in one RCCL collective.  Units = grid points x (ts + tdis) year
    transitions."""
    from midaspom_amd import dist as mdist
    inp = ROOT / "tests" / "golden" / "occupancies.txt"
    s, ts, tdis = args.grid4, 20, 10
    g, _ = mdp.grid(s, 0.0, 1.0)
    K = mdp.kgrid(s, 0.1, 100.0)
    r0, r1 = mdist.row_slab(rank, world, s)
    cap = s // world + s % world
    row = mdp.first_row(inp)
    sc = mdp.Scenario(row, "dieoff", m=400.0, d=100.0, device=dev.index)
    sc.set_grid(g[r0:r1], g, K, ts=ts, tdis=tdis)
    out = torch.zeros((cap, s, s), dtype=torch.float64, device=dev)
    gathered = [torch.empty_like(out) for _ in range(world)] if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        sc.run(out.data_ptr(), stream)

    def gather():  # the job's one gather, after the last pass (as configs 2/3)
        if world > 1:
            src = _coll_tensor(out, args)
            dist.gather(src, [_coll_tensor(g, args) for g in gathered] if gathered else None, dst=0)

    for _ in range(args.warmup):
        step()
    gather()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    gather()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    job_ms = time_job(step, gather, dev, world, reps=1)
    kms = sc.time_kernels(out.data_ptr(), stream, reps=max(1, min(args.steps, 5)))
    torch.cuda.synchronize(dev)
    if world > 1:
        t = _coll_tensor(torch.tensor([dt], dtype=torch.float64, device=dev), args)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    n = row.size
    ns = 1 << n
    # FP64 work per point per year in the vector-propagation form: the Pc
    # application (3^n FMAs) + n Pe passes over 2^(n-1) pairs (3 flop each)
    flop_year = 2 * 3 ** n + 3 * n * (ns // 2)
    nloc = (r1 - r0) * s * s
    achieved = flop_year * nloc * ts / (kms["k_scn_lik"] * 1e-3) / 1e12
    result = {
        "metric": "grid-point x timestep likelihood evals/sec (MIDASPOM_dieoff 3-D grid)",
        "value": s ** 3 * (ts + tdis) * args.steps / dt,
        "unit": "grid-point-timestep evals/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "examples/input first survey row (shipped)",
        "config": {"workload": f"config4: MIDASPOM_dieoff (e,c,K_D) {s}^3 grid, ts=20, tdis=10, n=8",
                   "grid": [s, s, s], "patches": int(n), "states": ns,
                   "parallelism": f"e-row slabs x{world}" + (f", {_coll_name(args)} gather" if world > 1 else ""),
                   "backend": args.backend if world > 1 else None},
        "job": {"ms": job_ms, "what": "one pass + one gather to rank 0" if world > 1 else "one pass"},
        "kernel_ms": kms,
        "roofline": {"kernel": "k_scn_lik", "bound": "fp64-valu", "compute_unit": "FP64 VALU",
                     "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, **_pmc_traffic(4), "flop_per_point_year": flop_year},
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_projection:
        result["projection"] = projection_block(args, dev, stream, [4])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        rng = np.random.default_rng(0)
        lik = out[: r1 - r0].cpu().numpy()
        t0 = time.perf_counter()
        pts, worst = 0, 0.0
        while time.perf_counter() - t0 < 10.0:
            ie, ic = int(rng.integers(0, s)), int(rng.integers(0, s))
            iK = rng.choice(s, size=4, replace=False)
            ref = oracle.dieoff_lik(row, K[iK], g[ie], g[ic], ts=ts, tdis=tdis, m=400.0, d=100.0)
            got = lik[ie, ic, iK]
            big = ref > 1e-14
            if big.any():
                worst = max(worst, float((np.abs(got[big] - ref[big]) / ref[big]).max()))
            worst = max(worst, float(np.abs(got[~big] - ref[~big]).max(initial=0.0)) * 1e6)
            pts += iK.size
        wall = time.perf_counter() - t0
        result["cpu_baseline"] = {
            "value": pts * (ts + tdis) / wall, "unit": "grid-point-timestep evals/s", "cores": 1, "kind": "port",
            "sample": f"{pts} random (e,c,K) points, oracle/spom_dieoff_oracle.c dense matpow formulation, "
                      f"1 thread, {wall:.1f} s"}
        result["parity"] = {"points_checked": pts, "max_rel_dlik": worst}
    sc.close()
    return result


def time_job(step, gather, dev, world, reps=3):
    """Median wall (ms) of the reference's job shape: one pass of the path
    plus the single gather, bracketed by barrier + synchronize."""
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        step()
        gather()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        ts.append(time.perf_counter() - t0)
    ms = float(np.median(ts)) * 1e3
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    return ms


def strong_scaling(model, s, tmax, rank, world, dev, args):
    """The reference's MPI job on a FIXED grid (main_MIDASPOM_MPI.c:361-368,
    482-506) as the drop-in runs it (midaspom_amd/dist.py): the s x s grid
    split into `world` c-column slabs (remainder to rank 0; each rank forms
    only its own columns' per-c tables, for the whole grid's |c| bound), each
    rank one pass over its slab in the product's [c][e] layout, then ONE
    gather of the padded slabs to rank 0 (RCCL over xGMI).  Timed as that job
    (median of 10, barrier + synchronize either side, max over ranks) and as
    K passes + one gather; value = s^2 (tmax - 1) units over the time.  Work
    per rank shrinks as N grows, so this is the strong-scaling figure
    ("scaling": "strong")."""
    from midaspom_amd import dist as mdist
    g, _ = mdp.grid(s, 0.0, 1.0)
    c0, c1 = mdist.row_slab(rank, world, s)
    cap = s // world + s % world
    eng = mdp.Engine(model, devices=[dev.index])
    eng.set_cbound(float(np.abs(g).max()))
    eng.set_grid(g, g[c0:c1])
    eng.set_layout("ce")
    out = torch.zeros((cap, s), dtype=torch.float64, device=dev)
    # the gather's targets on rank 0 (host tensors under a rehearsal backend)
    gathered = [_coll_tensor(torch.empty_like(out), args) for _ in range(world)] if rank == 0 else None
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        eng.run(out.data_ptr(), s, stream)

    def gather():
        dist.gather(_coll_tensor(out, args), gathered, dst=0)

    for _ in range(max(1, args.warmup)):
        step()
    gather()
    job_ms = time_job(step, gather, dev, world, reps=10)
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    gather()
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    t = _coll_tensor(torch.tensor([dt], dtype=torch.float64, device=dev), args)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    same = None
    if rank == 0:
        # the gathered grid (the last pass's slabs, [c][e] each) against the
        # whole grid computed by this one rank: the same bits, as the
        # reference's MPI build gives the same file for any rank count
        full = np.empty((s, s), dtype=np.float64)  # [c][e]
        for r in range(world):
            a, b = mdist.row_slab(r, world, s)
            full[a:b] = gathered[r][: b - a].cpu().numpy()
        eng.set_grid(g, g)
        one = torch.empty((s, s), dtype=torch.float64, device=dev)
        eng.run(one.data_ptr(), s, stream)
        torch.cuda.synchronize(dev)
        same = bool(np.array_equal(full, one.cpu().numpy(), equal_nan=True))
    eng.close()
    units = s * s * (tmax - 1)
    return {"scaling": "strong", "grid": [s, s], "split": "c-column slabs (dist.py)",
            "cols_per_rank": {"rank0": cap, "others": s // world},
            "gathered_equals_one_rank": same, "backend": args.backend,
            "job_ms": job_ms, "value": units / (job_ms * 1e-3),
            "what": "fixed s x s grid in N c-column slabs: one pass per rank + one gather to rank 0",
            "steps_ms_per_step": dt / args.steps * 1e3, "steps_value": units * args.steps / dt,
            "steps_what": f"{args.steps} passes + one gather (the gather amortised)"}


def _ms_per_pass(run, dev, reps):
    """Mean wall (ms) of `reps` back-to-back passes after two warm ones,
    bracketed by synchronize (the bench step's own timing)."""
    run()
    run()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / reps * 1e3


PROJ_NS = (2, 4, 8)


def _project(t1_ms, slab_ms, nbytes):
    """Projection record of one split: per N the slowest rank's pass against
    the one-GPU pass, and the bytes rank 0 receives in the job's one gather
    (((N - 1) / N of the grid, padded slabs), which only a multi-GPU run
    times."""
    out = {}
    for n, ms in slab_ms.items():
        worst = max(ms)
        out[str(n)] = {"slab_ms": ms, "max_slab_ms": worst, "projected_speedup": t1_ms / worst,
                       "gather_bytes_to_rank0": int(nbytes * (n - 1) / n)}
    return out


def project_likelihood(model, s, dev, stream, reps, splits=("e", "c")):
    """Strong-scaling projection measured on ONE GPU: the fixed
    s x s grid split over N = 2, 4, 8 ranks, each rank's exact slab timed
    alone on this GPU as one pass of the path (the engine picks its kernels
    for the slab's shape, as a rank would); projected_speedup = one-GPU pass /
    slowest slab.  Splits: "e" -- e-row slabs (main_MIDASPOM_MPI.c:361-368,
    remainder to rank 0); "c" -- c-column slabs (each rank then forms only
    its own columns' per-c tables; in the [c][e] layout a c-slab is one
    contiguous block for the gather, and the posterior file does not depend
    on the split).  The slab kernel times name the term that bounds it."""
    from midaspom_amd import dist as mdist
    g, _ = mdp.grid(s, 0.0, 1.0)
    eng = mdp.Engine(model, devices=[dev.index])
    eng.set_layout("ce")
    eng.set_cbound(float(np.abs(g).max()))  # as a column-slab rank builds its tables (dist.py)
    out = torch.empty((s, s), dtype=torch.float64, device=dev)

    def timed(e, c, kernels=False):
        eng.set_grid(e, c)
        ms = _ms_per_pass(lambda: eng.run(out.data_ptr(), len(e), stream), dev, reps)
        return ms, (eng.time_kernels(out.data_ptr(), len(e), stream, reps=reps) if kernels else None)

    t1, k1 = timed(g, g, True)
    res = {"one_gpu_ms": t1, "one_gpu_kernel_ms": k1, "reps": reps}
    for split in splits:
        slab_ms, kslab = {}, {}
        for n in PROJ_NS:
            slab_ms[n] = []
            for r in range(n):
                a, b = mdist.row_slab(r, n, s)
                ms, km = timed(*((g[a:b], g) if split == "e" else (g, g[a:b])), kernels=(r == 0))
                slab_ms[n].append(ms)
                if km is not None:
                    kslab[n] = km  # rank 0's slab (the largest: the remainder is its)
        proj = _project(t1, slab_ms, s * s * 8)
        for n in PROJ_NS:
            proj[str(n)]["rank0_kernel_ms"] = kslab[n]
        res[f"split_{split}"] = proj
    eng.close()
    return res


def project_dieoff(s, dev, stream, reps):
    """The same projection for config 4 (die-off (e, c, K_D) = s^3): e-row
    slabs, each rank's slab timed alone on this GPU."""
    from midaspom_amd import dist as mdist
    inp = ROOT / "tests" / "golden" / "occupancies.txt"
    g, _ = mdp.grid(s, 0.0, 1.0)
    K = mdp.kgrid(s, 0.1, 100.0)
    sc = mdp.Scenario(mdp.first_row(inp), "dieoff", m=400.0, d=100.0, device=dev.index)
    out = torch.empty((s, s, s), dtype=torch.float64, device=dev)

    def timed(e):
        sc.set_grid(e, g, K, ts=20, tdis=10)
        return _ms_per_pass(lambda: sc.run(out.data_ptr(), stream), dev, reps)

    t1 = timed(g)
    slab_ms = {n: [timed(g[a:b]) for a, b in (mdist.row_slab(r, n, s) for r in range(n))] for n in PROJ_NS}
    sc.close()
    return {"one_gpu_ms": t1, "reps": reps, "split_e": _project(t1, slab_ms, s ** 3 * 8)}


def projection_block(args, dev, stream, cfgs):
    """The projections of `cfgs` (each guarded: a failing leg reports its
    error instead of costing the bench line)."""
    res = {}
    for c in cfgs:
        try:
            if c == 4:
                res["config4"] = project_dieoff(args.grid4, dev, stream, reps=2)
            else:
                gen = CONFIGS[c]
                m = mdp.Model.load(synth.write(Path(tempfile.mkdtemp(prefix="mdp_proj_")) / "in.txt", **gen["gen"]),
                                   m=400.0, p=0.5, d=100.0)
                res[f"config{c}"] = project_likelihood(m, gen["s"], dev, stream, reps=20 if c == 2 else 10)
        except Exception as exc:  # noqa: BLE001 -- reported, not fatal
            res[f"config{c}"] = {"error": repr(exc)}
    res["what"] = ("strong scaling of the fixed grid projected from ONE GPU: each rank's exact slab timed alone "
                   "(one pass); projected_speedup = one-GPU pass / slowest slab; the job's one gather is not in "
                   "it (gather_bytes_to_rank0; the N-GPU lines time it)")
    return res


def resolve_world(args, env=None):
    """(world, rank, local, spawn): the job's shape from the launcher's
    environment (torchrun: WORLD_SIZE / RANK / LOCAL_RANK) or, when no
    launcher set it, from --gpus (spawn = True: this process starts --gpus
    ranks itself).  A launcher world that contradicts an explicit --gpus is
    an error: the line would name one GPU count and time another."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher's WORLD_SIZE is {world}")
        return world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0")), False
    world = args.gpus if args.gpus is not None else 1
    if world < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return world, 0, 0, world > 1


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _spawned_rank(local, argv, world, port):
    """Entry of a rank started by bench.py itself (--gpus N, no launcher): the
    launcher's environment, then the ordinary path.  Started with the spawn
    method, so it is a fresh interpreter: the parent never touched the GPU."""
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(local), "LOCAL_RANK": str(local),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.argv = [sys.argv[0]] + list(argv)
    main()


def dry_run(args, world, rank):
    """--dry-run: the multi-rank plumbing without a GPU (CPU tests): the
    process group over gloo, each rank's e-row slabs of the weak (N s x s)
    and strong (s x s, configs 2 and 3) grids, gathered to rank 0."""
    from midaspom_amd import dist as mdist
    if world > 1:
        dist.init_process_group("gloo")
    s = CONFIGS[args.config]["s"]
    mine = {"rank": rank, "weak_rows": [rank * s, (rank + 1) * s],
            "strong_cols": {str(c): list(mdist.row_slab(rank, world, CONFIGS[c]["s"])) for c in (2, 3)}}
    allr = [None] * world
    if world > 1:
        dist.all_gather_object(allr, mine)
        dist.destroy_process_group()
    else:
        allr = [mine]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": allr}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; under a launcher it must equal WORLD_SIZE, without one "
                         "bench.py starts that many ranks itself (default 1)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS) + [4, 5])
    ap.add_argument("--grid4", type=int, default=256, help="config 4 grid points per axis")
    ap.add_argument("--replicates", type=int, default=1_000_000, help="config 5 ensemble size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-strong", action="store_true", help="N > 1: skip the fixed-grid (strong) blocks")
    ap.add_argument("--layout", default="ce", choices=["ce", "ec"],
                    help="device layout of log L: ce = [c][e] (coalesced stores, default), ec = [e][c] rows")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--dry-run", action="store_true", help="multi-rank plumbing only, no GPU (tests)")
    ap.add_argument("--no-projection", action="store_true",
                    help="N = 1: skip the one-GPU strong-scaling projection of configs 2, 3, 4 and 6")
    args = ap.parse_args()

    world, rank, local, spawn = resolve_world(args)
    if spawn:
        # no launcher: start the ranks here, before this process makes any
        # GPU call (they are fresh interpreters; this one only waits)
        import torch.multiprocessing as tmp
        argv = [a for a in sys.argv[1:]]
        tmp.start_processes(_spawned_rank, args=(argv, world, _free_port()), nprocs=world, join=True,
                            start_method="spawn")
        return
    if args.dry_run:
        dry_run(args, world, rank)
        return
    # the drop-in CLI's end-to-end walls (cpu_baseline.end_to_end) are taken
    # first, while this process holds no GPU context: a user's CLI run does
    # not share the device with a live bench process either (round 3 took
    # them after the timed loop, beside this process's own context)
    e2e, tmpdir = None, Path(tempfile.mkdtemp(prefix="mdp_bench_"))
    if world == 1 and not args.no_cpu_baseline and args.config in CONFIGS:
        e2e = e2e_walls(synth.write(tmpdir / "e2e_input.txt", **CONFIGS[2]["gen"]), tmpdir)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dev_index = local % max(1, torch.cuda.device_count())  # == local on a full node
        torch.cuda.set_device(dev_index)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:  # rehearsal of the multi-rank logic (e.g. 2 ranks on a 1-GPU box)
            dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.config in (4, 5):
        result = (bench_future if args.config == 5 else bench_dieoff)(args, world, rank, dev)
        if rank == 0:
            print(json.dumps(result))
        if world > 1:
            dist.destroy_process_group()
        return

    cfg = CONFIGS[args.config]
    s = cfg["s"]
    inp = tmpdir / "occupancies.txt"
    synth.write(inp, **cfg["gen"])
    model = mdp.Model.load(inp, m=400.0, p=0.5, d=100.0)
    tmax = model.tmax

    # weak scaling: rank r owns e-rows [r*s, (r+1)*s) of an (world*s) x s grid
    # (N > 1 lines also carry "strong": the fixed s x s grids of configs 2
    # and 3 split over the N ranks)
    g_all, _ = mdp.grid(world * s, 0.0, 1.0)
    g_e = g_all[rank * s:(rank + 1) * s].copy()
    g_c, win = mdp.grid(s, 0.0, 1.0)

    eng = mdp.Engine(model, devices=[dev.index])
    eng.set_grid(g_e, g_c)
    # the slab's log L in HBM: [c][e] by default (each workgroup's e values of
    # one column contiguous, so its stores coalesce; mdp_engine_set_layout),
    # or the reference's [e][c] rows; the slab is s x s either way
    eng.set_layout(args.layout)
    out = torch.empty((s, s), dtype=torch.float64, device=dev)
    # the gather's targets on rank 0 (host tensors under a rehearsal backend)
    gathered = [_coll_tensor(torch.empty_like(out), args) for _ in range(world)] if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream(dev).cuda_stream

    # A step = one pass of the hot path over this rank's slab (no exchange:
    # grid points are independent).  The job's single gather of the slabs to
    # rank 0 (main_MIDASPOM_MPI.c:482-506; RCCL over xGMI) runs once, at the
    # end of the timed region, on the last pass's output.
    def step():
        eng.run(out.data_ptr(), s, stream)

    def gather():
        if world > 1:
            dist.gather(_coll_tensor(out, args), gathered, dst=0)

    for _ in range(args.warmup):
        step()
    gather()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    gather()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    weak_same = None
    if world > 1 and rank == 0:
        # the gathered (N s) x s grid against the same grid computed by this
        # one rank alone: the same bits (each point's arithmetic is its own)
        one_eng = mdp.Engine(model, devices=[dev.index])
        one_eng.set_grid(g_all, g_c)
        one_eng.set_layout(args.layout)
        one = torch.empty((s, world * s) if args.layout == "ce" else (world * s, s), dtype=torch.float64, device=dev)
        one_eng.run(one.data_ptr(), one.shape[1], stream)
        torch.cuda.synchronize(dev)
        one_eng.close()
        parts = [x.cpu().numpy() for x in gathered]
        full = np.concatenate(parts, axis=1 if args.layout == "ce" else 0)
        weak_same = bool(np.array_equal(full, one.cpu().numpy(), equal_nan=True))
    job_ms = time_job(step, gather, dev, world)
    strong = None
    if world > 1 and not args.no_strong:
        strong = {}
        for sc in (2, 3):
            if sc == args.config:
                m_sc = model
            else:
                m_sc = mdp.Model.load(synth.write(tmpdir / f"strong_cfg{sc}.txt", **CONFIGS[sc]["gen"]),
                                      m=400.0, p=0.5, d=100.0)
            strong[f"config{sc}"] = strong_scaling(m_sc, CONFIGS[sc]["s"], m_sc.tmax, rank, world, dev, args)
    # Kernel durations, measured live with HIP events on the stream the path
    # runs on (torch's current stream):
    # each kernel of the path launched K times back to back between two
    # events (mdp_engine_time_kernels; no per-launch events, whose completion
    # signals would add microseconds to every launch).  They agree with
    # rocprofv3 --kernel-trace --stats of the same command (profiles/).
    kms = eng.time_kernels(out.data_ptr(), s, stream, reps=args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        t = _coll_tensor(torch.tensor([dt], dtype=torch.float64, device=dev), args)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # HBM traffic of the forward kernel per launch, from the committed
    # rocprofv3 PMC passes of this workload (scripts/gpu_pmc.sh,
    # scripts/pmc_traffic.py); null when no profile of this config exists
    traffic, traffic_src = None, None
    tf = ROOT / "profiles" / f"pmc_traffic_cfg{args.config}.json"
    if tf.exists():
        traffic = json.loads(tf.read_text())["hbm_bytes_per_launch"]
        traffic_src = str(tf.relative_to(ROOT))
    units = world * s * s * (tmax - 1) * args.steps
    work = eng.work(s, s)
    fact = eng.work_fact(s, s)
    info = eng.info()
    fwd_ms = kms.get("k_forward", float("nan"))
    fused = "k_qrows" not in kms  # the fused forward kernel does the per-c work too
    # numerator: the algorithmic minimum of the ratio forms the kernels
    # evaluate (mdp_engine_work_fact flop_min, ABI 8): each distinct Q
    # group's Horner chain once per point, g^d once per distinct (group, d)
    # on s-form points, every year's state update, the pre-scales, flushes,
    # set-up and prior sum (+ the per-c tables when the fused kernel forms
    # them); a transition that recurs is algorithmic reuse, not work.  The
    # round-4 direct-form counts (with the weight table the ratio forms no
    # longer build) are reported beside it as legacy figures.
    flop_fwd = fact["flop_min"] if fused else s * s * fact["pt_min"]
    flop_direct = fact["flop_min_direct"] if fused else s * s * (fact["weight_pt"] + fact["use_pt_min"]
                                                                  + fact["final_pt"])
    flop_every = fact["flop"] if fused else s * s * (fact["weight_pt"] + fact["use_pt"] + fact["final_pt"])
    achieved_tf = flop_fwd / (fwd_ms * 1e-3) / 1e12
    result = {
        "metric": "grid-point x timestep likelihood evals/sec",
        "value": units / dt,
        "unit": "grid-point-timestep evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        # value: each rank its own s x s slab (per-GPU work fixed as N grows);
        # N > 1 lines carry the fixed-grid figures of configs 2 and 3 in "strong"
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md Appendix C generator, md5-checked input)",
        "config": {"workload": cfg["name"], "patches": model.n, "years": tmax, "grid": [world * s, s],
                   "per_rank_grid": [s, s], "nvar": model.nvar, "nstates": model.nstates,
                   "nextid": model.nextid,
                   "parallelism": f"e-row slabs x{world}" + (f", {_coll_name(args)} gather" if world > 1 else ""),
                   "backend": args.backend if world > 1 else None,
                   # [c][e] is the product's layout: the CLIs (mdp_loglik_grid_layout), the torchrun
                   # drop-in (dist.gather_cols) and the normaliser / writer views all use it
                   "layout": "[c][e] (MDP_LAYOUT_CE, the drop-ins' layout)" if args.layout == "ce"
                             else "[e][c] (reference lik[i][j] order)"},
        # the reference's job shape: ONE pass over the grid plus the single
        # gather of the slabs (main_MIDASPOM_MPI.c:361-368, 482-506), median of 3
        "job": {"ms": job_ms, "value": world * s * s * (tmax - 1) / (job_ms * 1e-3),
                "what": "one pass + one gather to rank 0" if world > 1 else "one pass"},
        **({"strong": strong} if strong else {}),
        **({"gathered_equals_one_rank": weak_same} if world > 1 else {}),
        "kernel_ms": kms,
        "roofline": {
            "kernel": "k_forward",
            "bound": "fp64-valu",
            "compute_unit": "FP64 VALU (MI355X FP64 vector peak = FP64 matrix peak)",
            "achieved": achieved_tf,
            "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tf / FP64_PEAK_TFLOPS,
            "traffic": traffic,
            "traffic_unit": "bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": traffic_src,
            # closed-form factorised count from the plan's dimensions
            # (mdp_engine_work_fact): the kernel's share of it
            "flop_per_launch": flop_fwd,
            "flop_basis": "closed-form minimum of the ratio forms (each distinct Q group once per point), "
                          + ("per-c + per-point terms (fused kernel)" if fused
                             else "per-point terms (k_qrows does the per-c work)"),
            "flop_per_launch_direct_form": flop_direct,
            "frac_direct_form": flop_direct / (fwd_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
            "flop_per_launch_every_use": flop_every,
            "work_fact": fact,
            # the whole step's minimum (per-c tables + per-point work) over the step time
            "step_tflops_fact": fact["flop_min"] / (dt / args.steps) / 1e12,
            # the hipRTC generator's count of the code it emitted (transition caching included)
            "flop_per_launch_generated": work["flop_impl"],
            # SURVEY §8(d) F_alg (dense-in-j form): exceeds the FP64 peak as a
            # rate because the factorised path never performs most of it
            "flop_per_launch_survey_dense": work["flop_survey"],
            "falg_step_equiv_tflops": work["flop_survey"] / (dt / args.steps) / 1e12,
            "uses_per_point": info["nuses"],
            # forward-kernel time per (grid point x forward use): compares
            # series of different lengths (config 3 vs the chunked config 6)
            "fwd_ps_per_point_use": fwd_ms * 1e9 / (s * s * max(1, info["nuses"])),
        },
    }
    if world == 1 and not args.no_projection:
        result["projection"] = projection_block(args, dev, stream, [2, 3, 4, 6] if args.config == 2 else [args.config])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        lik = torch.empty((s, s), dtype=torch.float64, device=dev)
        eng.run(lik.data_ptr(), s, stream)
        torch.cuda.synchronize(dev)
        lik_h = lik.cpu().numpy()
        if args.layout == "ce":  # [c][e] -> the reference's lik[e][c]
            lik_h = np.ascontiguousarray(lik_h.T)
        ltot = mdp.log_total(lik_h, win)
        cpu, parity = cpu_baseline(inp, g_e, g_c, lik_h, ltot, tmax, tmpdir, end_to_end=e2e)
        result["cpu_baseline"] = cpu
        result["parity"] = parity
    else:
        result["cpu_baseline"] = None
    eng.close()
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
