"""Forward-kernel time against grid size on config 3 (fixed nc): the steps of
T(blocks) show how many workgroups of the reading-variant forward kernel run
concurrently per CU.  GPU box: python scripts/occupancy_probe.py"""
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp  # noqa: E402
from midaspom_amd import synth  # noqa: E402

torch.cuda.set_device(0)
tmp = Path(tempfile.mkdtemp())
path = synth.write(str(tmp / "in3.txt"), **synth.CONFIG3)
model = mdp.Model.load(path)
nc = int(sys.argv[1]) if len(sys.argv) > 1 else 256
with mdp.Engine(model, devices=[0]) as eng:
    for ne in (512, 1024, 2048, 3072, 4096, 6144, 8192):
        e = np.linspace(0.0, 1.0, ne)
        c = np.linspace(0.0, 1.0, nc)
        eng.set_grid(e, c)
        out = torch.empty(nc * ne, dtype=torch.float64, device="cuda")
        eng.run(out.data_ptr(), nc)  # out[e][c]: ld = nc
        torch.cuda.synchronize()
        ms = eng.time_kernels(out.data_ptr(), nc, reps=20)
        blocks = nc * ((ne + 511) // 512)
        print(f"nc {nc} ne {ne} blocks {blocks} per-CU {blocks / 256:.1f} fwd_us {ms.get('k_forward', 0) * 1e3:.2f}",
              flush=True)
