"""Would config 3's k_qrows overlap with the forward kernel of other columns?

Times one engine over the whole 1024 x 1024 grid against the same grid cut
into K column ranges, each its own engine (k_qrows + forward) launched on its
own stream, all K issued before any is waited for: if the latency-bound
k_qrows of one range runs under the FP64-bound forward of another, the K-range
step is shorter than the one-engine step.  Prints one JSON line per K.
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import midaspom_amd as mdp  # noqa: E402
from midaspom_amd import synth  # noqa: E402

s, steps = 1024, 50
f = synth.write("/tmp/ovl_c3.txt", **synth.CONFIG3)
model = mdp.Model.load(f)
g, _ = mdp.grid(s)
for k in (1, 2, 4):
    edges = np.linspace(0, s, k + 1).astype(int)
    engs, outs, streams = [], [], []
    for i in range(k):
        c = g[edges[i]:edges[i + 1]]
        eng = mdp.Engine(model, devices=[0])
        eng.set_grid(g, c)
        eng.set_layout("ce")
        engs.append(eng)
        outs.append(torch.empty((c.size, s), dtype=torch.float64, device="cuda"))
        streams.append(torch.cuda.Stream())

    def step():
        for eng, out, st in zip(engs, outs, streams):
            eng.run(out.data_ptr(), s, st.cuda_stream)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(json.dumps({"ranges": k, "step_us": dt * 1e6}), flush=True)
    for eng in engs:
        eng.close()
