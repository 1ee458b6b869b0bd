"""Time k_zpv / k_coefs / k_forward variants (MDP_EPL) on configs 2 and 3.
Usage (GPU box): python scripts/sweep_forward.py [--steps K]"""
import argparse
import json
import os
import sys
import tempfile
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp  # noqa: E402
from midaspom_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--epl", default="1,2,4")
ap.add_argument("--configs", default="2,3")
args = ap.parse_args()
torch.cuda.set_device(0)
tmp = Path(tempfile.mkdtemp())
res = []
for cfgid in [int(x) for x in args.configs.split(",")]:
    gen, s = (synth.CONFIG2, 512) if cfgid == 2 else (synth.CONFIG3, 1024)
    f = synth.write(tmp / f"c{cfgid}.txt", **gen)
    model = mdp.Model.load(f)
    g, _ = mdp.grid(s)
    ref = None
    for epl in [int(x) for x in args.epl.split(",")]:
        os.environ["MDP_EPL"] = str(epl)
        eng = mdp.Engine(model, devices=[0])
        eng.set_grid(g, g)
        out = torch.empty((s, s), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            eng.run(out.data_ptr(), s, st)
        torch.cuda.synchronize()
        eng.set_profiling(True)
        for _ in range(args.steps):
            eng.run(out.data_ptr(), s, st)
        torch.cuda.synchronize()
        ms = eng.kernel_ms()
        w = eng.work(s, s)
        o = out.cpu().numpy()
        if ref is None:
            ref = o
        same = bool(((o == ref) | (torch.isnan(torch.from_numpy(o)).numpy())).all())
        r = {"config": cfgid, "epl": epl, **{k: round(v * 1e3, 2) for k, v in ms.items()},
             "fwd_tflops": round(w["flop_impl"] / (ms["k_forward"] * 1e-3) / 1e12, 2),
             "bitwise_same_as_first": same, "info": eng.info()}
        print(json.dumps(r), flush=True)
        eng.close()
