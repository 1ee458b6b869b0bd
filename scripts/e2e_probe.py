"""Where the drop-in CLI's wall goes (GPU box): configs 1 (s = 50) and 2
(s = 512) interleaved, warm (a filled code-object cache), each run timed
from spawn to exit on CLOCK_MONOTONIC beside the CLI's own split
(MIDASPOM_TIMING=1: parse, HIP start-up, set-up, grid, Ltot, write) and its
main entry / return stamps -- the wall before main (exec, loader, library
constructors) and after it (exit) -- with the default quick exit and with
MIDASPOM_FULL_EXIT=1 (the HIP runtime's exit-time teardown).  One JSON line."""
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from midaspom_amd import _lib, synth  # noqa: E402

tmp = Path(tempfile.mkdtemp())
inputs = {"config1": (ROOT / "tests" / "golden" / "occupancies.txt", 50),
          "config2": (synth.write(tmp / "c2.txt", **synth.CONFIG2), 512)}
env = dict(os.environ, MDP_JIT_CACHE=str(tmp / "jit"), MIDASPOM_TIMING="1")


def run(name, extra):
    inp, s = inputs[name]
    cmd = [str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", str(s), "-i", str(inp), "-o", str(tmp / "p.txt")]
    t0 = time.monotonic()
    r = subprocess.run(cmd, env=dict(env, **extra), capture_output=True, text=True)
    t1 = time.monotonic()
    assert r.returncode == 0, r.stderr[-800:]
    out = {"wall": round(t1 - t0, 4)}
    for ln in r.stderr.splitlines():
        if ln.startswith("midaspom timing (s):"):
            v = ln.split(":", 1)[1].split()
            out["split"] = {v[i]: float(v[i + 1]) for i in range(0, len(v) - 1, 2)}
        if ln.startswith("midaspom clock (s):"):
            v = ln.split(":", 1)[1].split()
            st = {v[i]: float(v[i + 1]) for i in range(0, len(v) - 1, 2)}
            out["before_main"] = round(st["main_entry"] - t0, 4)
            out["after_main"] = round(t1 - st["main_return"], 4)
    return out


res = {}
for name in ("config1", "config2"):  # fill the caches
    run(name, {})
for rep in range(3):
    for name in ("config1", "config2"):
        for mode, extra in (("quick", {}), ("full", {"MIDASPOM_FULL_EXIT": "1"})):
            res.setdefault(f"{name}_{mode}", []).append(run(name, extra))
print(json.dumps(res))
