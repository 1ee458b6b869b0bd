"""Split config 4's k_scn likelihood pass into its per-workgroup fixed cost
(tables, initial states, final sum) and its per-year cost: time the pass at
ts = 0, 1, 5, 20 years on the 256^3 grid (tdis = 10).  Usage (GPU box):
python scripts/scenario_years.py"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp  # noqa: E402

row = mdp.first_row(ROOT / "tests" / "golden" / "occupancies.txt")
g, _ = mdp.grid(256)
K = mdp.kgrid(256, 0.1, 100.0)
res = {}
for ts in (0, 1, 5, 20):
    with mdp.Scenario(row, "dieoff", m=400.0, d=100.0) as sc:
        shape = sc.set_grid(g, g, K, ts=ts, tdis=10)
        out = torch.empty(shape, dtype=torch.float64, device="cuda")
        ms = sc.time_kernels(out.data_ptr(), 0, reps=3)
        res[f"ts{ts}"] = ms
        print(json.dumps({"ts": ts, **ms}), flush=True)
