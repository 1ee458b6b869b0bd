"""Debug: config-1 grid after an unrelated engine ran in the same process."""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp
import oracle
import torch
torch.cuda.set_device(0)
golden = ROOT / "tests" / "golden"
if len(sys.argv) > 1 and sys.argv[1] == "pollute":
    # allocate, fill with garbage and free device memory through torch and the future engine
    x = torch.full((64 << 20,), float("nan"), dtype=torch.float64, device="cuda")
    del x
    torch.cuda.empty_cache()
model = mdp.Model.load(golden / "occupancies.txt", m=400, d=100)
g, win = mdp.grid(50)
with mdp.Engine(model, devices=[0]) as eng:
    lik = eng.loglik_grid(g, g)
    print(eng.info())
ref = oracle.OracleModel.load(golden / "occupancies.txt", 400, 0.5, 100).loglik_grid(g, g)
bad = np.isneginf(lik) != np.isneginf(ref)
print("mismatch cells", int(bad.sum()), "of", bad.size)
idx = np.argwhere(bad)[:10]
for i, j in idx:
    print(i, j, lik[i, j], ref[i, j])
fin = np.isfinite(ref) & np.isfinite(lik)
print("max dlog", float(np.abs(lik[fin] - ref[fin]).max()) if fin.any() else None)
