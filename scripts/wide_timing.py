"""Time the wide forward path (years with more than 16 states) on survey-like
series: the Appendix C generator with many unvisited patches per year.
Prints one JSON line per case: kernel times, step time, and the oracle's
per-point CPU cost on a small sample (1 thread)."""
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp  # noqa: E402
import oracle  # noqa: E402
from midaspom_amd import synth  # noqa: E402

tmp = Path(tempfile.mkdtemp())
for pmiss, T, s in [(0.45, 30, 512), (0.6, 50, 256)]:
    cfg = dict(synth.CONFIG2, pmiss=pmiss, seed=5, T=T)
    f = synth.write(tmp / f"w{pmiss}.txt", **cfg)
    model = mdp.Model.load(f)
    g, _ = mdp.grid(s)
    eng = mdp.Engine(model, devices=[0])
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
    print(json.dumps({"pmiss": pmiss, "years": T, "grid": s, "npstates_max": int(model.npstates.max()),
                      "nuses": eng.info()["nuses"], "variant": eng.info()["variant"], "step_ms": step * 1e3,
                      "kernel_ms": kms, "gpu_points_per_s": s * s / step, "oracle_points_per_s_1core": 1 / per_pt}),
          flush=True)
    eng.close()
