"""End-to-end wall of the compiled drop-in CLI on small grids: cold and warm
hipRTC cache, the generic (precompiled) kernels (MDP_JIT=0), and the HIP
start-up alone (mdp_device_count through ctypes in a fresh process).  Median
of 3 per leg.  Usage (GPU box): python scripts/cli_timing.py"""
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from midaspom_amd import _lib  # noqa: E402

tmp = Path(tempfile.mkdtemp())
inp = ROOT / "tests" / "golden" / "occupancies.txt"


def wall(cmd, env):
    t0 = time.perf_counter()
    r = subprocess.run(cmd, env=env, capture_output=True)
    assert r.returncode == 0, r.stderr.decode()[-500:]
    return time.perf_counter() - t0


res = {}
probe = [sys.executable, "-c", f"import ctypes; l = ctypes.CDLL({str(_lib.LIB_PATH)!r}); print(l.mdp_device_count())"]
res["python_ctypes_device_count_s"] = sorted(wall(probe, dict(os.environ)) for _ in range(3))[1]
res["python_start_s"] = sorted(wall([sys.executable, "-c", "pass"], dict(os.environ)) for _ in range(3))[1]
for s in (50, 101):
    cmd = [str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", str(s), "-i", str(inp), "-o", str(tmp / "p.txt")]
    cold = []
    for i in range(3):
        cold.append(wall(cmd, dict(os.environ, MDP_JIT_CACHE=str(tmp / f"c{s}_{i}"))))
    res[f"s{s}_cold_s"] = sorted(cold)[1]
    res[f"s{s}_warm_s"] = sorted(wall(cmd, dict(os.environ, MDP_JIT_CACHE=str(tmp / f"c{s}_0"))) for _ in range(3))[1]
    res[f"s{s}_generic_s"] = sorted(wall(cmd, dict(os.environ, MDP_JIT="0")) for _ in range(3))[1]
print(json.dumps(res))
