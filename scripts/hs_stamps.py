"""Phase stamps of k_fwd_hs (diag library, MDP_HS_PROBE=4): workgroup 0's
wave 0 records the shader clock at each phase of each year -- year start,
first v Pe pass issued, passes done, its U Pc loop done, the barrier after
it, its stores done, the year's last barrier -- on the survey-like series
of scripts/wide_timing.py.  Prints per series the clock spent in each phase
summed over the years (the results are not stored in this mode)."""
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

os.environ["MIDASPOM_DIAG_LIB"] = "1"
import torch  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp  # noqa: E402
from midaspom_amd import synth  # noqa: E402

tmp = Path(tempfile.mkdtemp())
PH = ["to_pass0", "passes", "mfma_own", "mfma_barrier", "stores", "year_barrier"]
for pmiss, T, nvar in [(0.6, 50, 8), (0.75, 30, 8), (0.75, 30, 9), (0.6, 30, 10)]:
    f = synth.write(tmp / f"s{pmiss}_{nvar}.txt", **dict(synth.CONFIG2, pmiss=pmiss, seed=5, T=T, nvar=nvar))
    model = mdp.Model.load(f)
    g, _ = mdp.grid(256)
    with mdp.Engine(model, options="MDP_WIDE=1;MDP_WIDE_MMA=3;MDP_HS_PROBE=4") as eng:
        eng.set_grid(g, g)
        out = torch.zeros((256, 256), dtype=torch.float64, device="cuda")
        for _ in range(3):
            eng.run(out.data_ptr(), 256)
        torch.cuda.synchronize()
        st = out.flatten()[: 8 * T].cpu().numpy().reshape(T, 8)[1:, :7]
    d = np.diff(st, axis=1)  # per year: phases 0-1 .. 5-6
    tot = d.sum(axis=0)
    rec = {"pmiss": pmiss, "nvar": nvar, "npstates_max": int(model.npstates.max()), "years": T - 1,
           "clk_per_year": float(tot.sum() / (T - 1)), **{k: float(v) for k, v in zip(PH, tot)},
           "per_year": {str(int(t + 1)): [int(x) for x in d[t]] for t in range(T - 1) if model.npstates[t + 1] >= 64}}
    print(json.dumps(rec), flush=True)
