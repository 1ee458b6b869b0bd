"""Time the paths for years with more than 16 states on survey-like series
(the Appendix C generator with many unvisited patches per year): the
specialised kernel with its states in LDS (default up to 64 states; two waves per
64 points splitting each year's new states, or one with MDP_VSPLIT=1) and the
wide kernels (MDP_WIDE=1).  Prints one JSON line per case and path: kernel
times, step time, the FP64 rate of the generated / wide work, and the
oracle's per-point CPU cost on a small sample (1 thread)."""
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch

if os.environ.get("WIDE_DIAG") == "1":  # measurement-only knobs (MDP_HS_PROBE) need the diag library
    os.environ["MIDASPOM_DIAG_LIB"] = "1"

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp  # noqa: E402
import oracle  # noqa: E402
from midaspom_amd import synth  # noqa: E402

tmp = Path(tempfile.mkdtemp())
PATHS = {  # path name -> engine knobs
    "default": {}, "nosplit": {"MDP_VSPLIT": "1"}, "split2": {"MDP_VSPLIT": "2"}, "split4": {"MDP_VSPLIT": "4"},
    "wide": {"MDP_WIDE": "1"}, "wideplain": {"MDP_WIDE": "1", "MDP_WIDE_MMA": "0"},
    "mma5": {"MDP_WIDE": "1", "MDP_WIDE_MMA": "1"},
    "hs": {"MDP_WIDE": "1", "MDP_WIDE_MMA": "3"},
    "mmt": {"MDP_WIDE": "1", "MDP_WIDE_MMA": "2"},
    "hs8": {"MDP_WIDE": "1", "MDP_WIDE_MMA": "3", "MDP_HS_WAVES": "8"},
    "epl2": {"MDP_VLDS_EPL": "2"},
}
# (pmiss, years, grid, path, variable patches): the config-2 generator with
# 8 variable patches (years of up to 64 / 128 / 256 states) and, round 6,
# with 9 and 10 (up to 512 / 1 024 states)
CASES = [(0.45, 30, 512, p, 8) for p in os.environ.get("WIDE_PATHS", "default,nosplit,wide").split(",") if p]
CASES += [(0.6, 50, 256, p, 8) for p in os.environ.get("WIDE60_PATHS", "default").split(",") if p]
CASES += [(0.75, 30, 256, p, 8) for p in os.environ.get("WIDE75_PATHS", "default").split(",") if p]
CASES += [(0.75, 30, 256, p, 9) for p in os.environ.get("WIDE9_PATHS", "").split(",") if p]
CASES += [(0.6, 30, 256, p, 10) for p in os.environ.get("WIDE10_PATHS", "").split(",") if p]
for pmiss, T, s, path, nvar in CASES:
    for k in [k for k in os.environ if k.startswith("MDP_")]:
        os.environ.pop(k, None)
    # "name" or "name:KNOB=V:KNOB=V" (extra engine knobs on top of the path's)
    name, *extra = path.split(":")
    os.environ.update(PATHS[name])
    os.environ.update(dict(kv.split("=") for kv in extra))
    cfg = dict(synth.CONFIG2, pmiss=pmiss, seed=5, T=T, nvar=nvar)
    f = synth.write(tmp / f"w{pmiss}_{nvar}.txt", **cfg)
    model = mdp.Model.load(f)
    g, _ = mdp.grid(s)
    t0 = time.perf_counter()
    eng = mdp.Engine(model, devices=[0])
    t_create = time.perf_counter() - t0
    eng.set_grid(g, g)
    out = torch.empty((s, s), dtype=torch.float64, device="cuda")
    for _ in range(2):
        eng.run(out.data_ptr(), s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        eng.run(out.data_ptr(), s)
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / 5
    kms = eng.time_kernels(out.data_ptr(), s, 0, reps=3)
    om = oracle.OracleModel.load(f, 400.0, 0.5, 100.0)
    t0 = time.perf_counter()
    om.loglik_points(g[1:9], g[1:9], threads=1)
    per_pt = (time.perf_counter() - t0) / 8
    w = eng.work(s, s)
    fa = eng.work_fact(s, s)  # the algorithmic minimum (each distinct transition once per point)
    fwd = [v for k, v in kms.items() if k in ("k_forward", "k_fwd_wide", "k_fwd_mma", "k_fwd_mmt", "k_fwd_hs")]
    print(json.dumps({"pmiss": pmiss, "nvar": nvar, "years": T, "grid": s, "path": path, "npstates_max": int(model.npstates.max()),
                      "nuses": eng.info()["nuses"], "variant": eng.info()["variant"], "create_s": t_create,
                      "launched": sorted(eng.launched()), "step_ms": step * 1e3,
                      "kernel_ms": kms, "fwd_tflops": w["flop_impl"] / (fwd[0] * 1e-3) / 1e12 if fwd else None,
                      "fwd_frac_fp64": w["flop_impl"] / (fwd[0] * 1e-3) / 78.6e12 if fwd else None,
                      "fwd_frac_min": s * s * (fa["weight_pt"] + fa["use_pt_min"] + fa["final_pt"]) / (fwd[0] * 1e-3)
                      / 78.6e12 if fwd else None,
                      "fwd_frac_min_ratio": s * s * fa["pt_min"] / (fwd[0] * 1e-3) / 78.6e12 if fwd else None,
                      "flop_impl_pt": w["flop_impl"] / (s * s), "pt_min": fa["pt_min"],
                      "gpu_points_per_s": s * s / step, "oracle_points_per_s_1core": 1 / per_pt}),
          flush=True)
    eng.close()
