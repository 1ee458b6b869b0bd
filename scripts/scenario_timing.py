"""Scenario kernel times against n: k_scn (n <= 8, LDS, lanes over e),
k_scn_row (n <= 12, a workgroup per point, threads over rows; MDP_SCN_ROW=1)
and k_scn_big (n <= 16, states in HBM; MDP_SCN_BIG=1), die-off, on an
(e, c, K) grid of G^3 points, ts = 20, tdis = 10.  Prints the kernel time and
the FP64 rate of the factorised algorithm (2 3^n + 3 n 2^(n-1) flop per
point-year).  GPU box: python scripts/scenario_timing.py"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import midaspom_amd as mdp  # noqa: E402

torch.cuda.set_device(0)
G = int(sys.argv[1]) if len(sys.argv) > 1 else 32
rng = np.random.default_rng(3)
for n, kern in ((8, "k_scn"), (8, "k_scn_row"), (8, "k_scn_big"), (9, "k_scn_row"), (9, "k_scn_big"),
                (10, "k_scn_row"), (10, "k_scn_big"), (11, "k_scn_row"), (12, "k_scn_row"), (12, "k_scn_big")):
    os.environ["MDP_SCN_BIG"] = "1" if kern == "k_scn_big" else "0"
    os.environ["MDP_SCN_ROW"] = "1" if kern == "k_scn_row" else "0"
    big = kern == "k_scn_big"
    row = (rng.random(n) < 0.5).astype(np.int32)
    row[0] = 1
    g = np.linspace(0.0, 1.0, G)
    K = mdp.kgrid(G, 0.1, 100.0)
    gg = G if (n <= 10 or not big) else max(4, G // 4)  # keep the k_scn_big cases short
    with mdp.Scenario(row, "dieoff", m=400.0, d=100.0) as sc:
        shape = sc.set_grid(g[:gg], g[:gg], K[:gg], ts=20, tdis=10)
        out = torch.empty(int(np.prod(shape)), dtype=torch.float64, device="cuda")
        sc.run(out.data_ptr())
        torch.cuda.synchronize()
        ms = sc.time_kernels(out.data_ptr(), reps=3)
    pts = gg ** 3
    flop = (2 * 3 ** n + 3 * n * 2 ** (n - 1)) * pts * 30
    t = ms["k_scn_lik"] * 1e-3
    print(f"n {n:2d} {kern:9s} grid {gg}^3  lik {ms['k_scn_lik']:.3f} ms  "
          f"v {ms['k_scn_v']:.3f} ms  {flop / t / 1e12:.2f} TF/s", flush=True)
