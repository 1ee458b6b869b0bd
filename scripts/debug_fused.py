"""Compare the fused direct path against k_qrows (MDP_FUSED=0) and the oracle
on small inputs; print mismatch statistics (GPU debugging aid)."""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import midaspom_amd as mdp  # noqa: E402
import oracle  # noqa: E402

G = Path(__file__).resolve().parents[1] / "tests" / "golden"
for fname, s in [("occupancies.txt", 50), ("config2_64x50.txt", 64)]:
    model = mdp.Model.load(G / fname)
    g, _ = mdp.grid(s)
    ref = oracle.OracleModel.load(G / fname, 400.0, 0.5, 100.0).loglik_grid(g, g)
    for env in ("MDP_FUSED=1,MDP_JIT_GLDS=1", "MDP_FUSED=1,MDP_JIT_GLDS=0", "MDP_FUSED=0"):
        for k in ("MDP_FUSED", "MDP_JIT_GLDS"):
            os.environ.pop(k, None)
        os.environ.update(dict(kv.split("=") for kv in env.split(",")))
        with mdp.Engine(model) as eng:
            got = eng.loglik_grid(g, g)
        bad = np.isneginf(got) != np.isneginf(ref)
        fin = np.isfinite(got) & np.isfinite(ref)
        print(fname, env, "inf-mismatch", int(bad.sum()), "max|d|",
              float(np.abs(got[fin] - ref[fin]).max()) if fin.any() else None,
              "sample", got[bad][:3], ref[bad][:3], flush=True)
