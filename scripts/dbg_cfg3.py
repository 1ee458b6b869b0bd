"""Debug: config 3 on the 1024^2 grid at the parity test's sampled points,
engine variants against the oracle (prints max |dlogL| per variant and the
worst points)."""
import os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np
import midaspom_amd as mdp
import oracle

golden = ROOT / "tests" / "golden"
model = mdp.Model.load(golden / "config3_256x200.txt")
g, win = mdp.grid(1024)
rng = np.random.default_rng(7)
ie, ic = rng.integers(0, 1024, 160), rng.integers(0, 1024, 160)
ie[:4], ic[:4] = [0, 1023, 0, 1023], [0, 0, 1023, 1023]
om = oracle.OracleModel.load(golden / "config3_256x200.txt")
ref = om.loglik_points(g[ie], g[ic], threads=16)
fin = np.isfinite(ref)
print("finite ref points", fin.sum(), flush=True)
for var in sys.argv[1:]:
    opts = dict(kv.split("=") for kv in var.split(",")) if var != "default" else {}
    with mdp.Engine(model, devices=[0], options=opts) as eng:
        got = eng.loglik_grid(g, g)[ie, ic]
        launched = eng.launched()
    err = np.abs(got - ref)
    err[~fin] = 0
    w = np.argsort(-err)[:5]
    print(var, sorted(launched), "max", err.max(), "neginf match", np.array_equal(np.isneginf(got), np.isneginf(ref)), flush=True)
    for k in w:
        print("   ie", ie[k], "ic", ic[k], "e", g[ie[k]], "c", g[ic[k]], "got", got[k], "ref", ref[k])
