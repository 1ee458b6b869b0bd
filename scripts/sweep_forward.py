"""Time the engine's kernels under environment variants on configs 2, 3 and 6
(LONG200).

Usage (GPU box):
  python scripts/sweep_forward.py [--steps K] [--configs 2,3] [--diag]
         [--variants 'MDP_JIT=1,MDP_EPL=2;MDP_JIT=0,MDP_EPL=2']
Each variant is a comma-separated list of environment assignments applied
before the engine is created.  Prints one JSON line per (config, variant).
"""
import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp  # noqa: E402
from midaspom_amd import synth  # noqa: E402

DEFAULT_VARIANTS = ";".join([
    "MDP_JIT=1",
    "MDP_JIT=1,MDP_EPL=1",
    "MDP_JIT=1,MDP_JIT_WINDOW=16",
    "MDP_JIT=0,MDP_EPL=2",
])

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--configs", default="2,3")
ap.add_argument("--variants", default=DEFAULT_VARIANTS)
ap.add_argument("--diag", action="store_true")
ap.add_argument("--layout", default="ce", choices=["ce", "ec"], help="device layout of log L (bench.py's default: ce)")
args = ap.parse_args()
# phase stamps and the measurement-only options need the diag library
if args.diag or "MDP_JIT_HACK" in args.variants or "MDP_JIT_WPE" in args.variants:
    os.environ["MIDASPOM_DIAG_LIB"] = "1"
torch.cuda.set_device(0)
tmp = Path(tempfile.mkdtemp())
KEYS = ("MDP_JIT", "MDP_EPL", "MDP_QROWS_XCD", "MDP_JIT_EFAST", "MDP_JIT_CHUNK", "MDP_JIT_GATHER", "MDP_QGLOBAL", "MDP_JIT_WINDOW", "MDP_FWD", "MDP_DIAG", "MDP_JIT_SLOTS", "MDP_JIT_XCD", "MDP_FUSED",
        "MDP_JIT_SMEM", "MDP_FUSED_COLS", "MDP_JIT_WPE", "MDP_JIT_HACK", "MDP_JIT_STORE")
for cfgid in [int(x) for x in args.configs.split(",")]:
    gen, s = {2: (synth.CONFIG2, 512), 3: (synth.CONFIG3, 1024), 6: (synth.LONG200, 512)}[cfgid]
    f = synth.write(tmp / f"c{cfgid}.txt", **gen)
    model = mdp.Model.load(f)
    g, _ = mdp.grid(s)
    ref = None
    for var in [v for v in args.variants.split(";") if v]:
        for k in [k for k in os.environ if k.startswith("MDP_")]:  # every engine knob, not only KEYS
            os.environ.pop(k, None)
        env = dict(kv.split("=") for kv in var.split(","))
        if args.diag:
            env["MDP_DIAG"] = "1"
        os.environ.update(env)
        t0 = time.perf_counter()
        eng = mdp.Engine(model, devices=[0])
        t_create = time.perf_counter() - t0
        eng.set_grid(g, g)
        eng.set_layout(args.layout)
        out = torch.empty((s, s), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            eng.run(out.data_ptr(), s, st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.run(out.data_ptr(), s, st)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.steps
        # kernel durations without per-launch events (bench.py's measure)
        ms = eng.time_kernels(out.data_ptr(), s, st, reps=args.steps)
        torch.cuda.synchronize()
        w = eng.work(s, s)
        o = out.cpu().numpy()
        if ref is None:
            ref = o
        fin = np.isfinite(ref) & np.isfinite(o)
        r = {"config": cfgid, "variant": var, "create_s": round(t_create, 3),
             **{k: round(v * 1e3, 2) for k, v in ms.items()},
             "step_us": round(wall * 1e6, 1),
             "fwd_tflops": round(w["flop_impl"] / (ms["k_forward"] * 1e-3) / 1e12, 2),
             "same_inf": bool(np.array_equal(np.isinf(ref), np.isinf(o))),
             "max_dlog_vs_first": float(np.abs(o[fin] - ref[fin]).max()) if fin.any() else 0.0,
             "info": eng.info()}
        print(json.dumps(r), flush=True)
        if args.diag:
            eng.run(out.data_ptr(), s, st)
            torch.cuda.synchronize()
            print("after idle:", eng.diag_report(), flush=True)
            for _ in range(20):  # steady state: the report shows the last of 20 back-to-back runs
                eng.run(out.data_ptr(), s, st)
            torch.cuda.synchronize()
            print("back to back:", eng.diag_report(), flush=True)
        eng.close()
