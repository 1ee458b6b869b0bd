"""Where the config-1 drop-in CLI's wall goes (GPU box): the bare HIP floor
(scripts/ubench/hipinit_probe: device count, a context, normal exit or
_exit), then the CLI cold (empty hipRTC cache) once and warm 5 times, with
the CLI's own split (MIDASPOM_TIMING=1), normally and with
MIDASPOM_FAST_EXIT=1 (no exit-time runtime teardown).  One JSON line."""
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
s = int(sys.argv[1]) if len(sys.argv) > 1 else 50
res = {"s": s}


def run(cmd, env):
    t0 = time.perf_counter()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True)
    w = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr[-800:]
    split = None
    for ln in r.stderr.splitlines():
        if ln.startswith("midaspom timing (s):") or ln.startswith("hipinit_probe:"):
            split = ln.split(":", 1)[1].strip()
    return round(w, 4), split


probe = str(ROOT / "scripts" / "ubench" / "hipinit_probe")
for args in ([], ["fast"], ["ctx"], ["ctx", "fast"]):
    res["probe_" + ("_".join(args) or "plain")] = [run([probe] + args, dict(os.environ)) for _ in range(3)]
cmd = [str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", str(s), "-i", str(inp), "-o", str(tmp / "p.txt")]
cache = tmp / "jit"
env = dict(os.environ, MDP_JIT_CACHE=str(cache), MIDASPOM_TIMING="1")
res["cold"] = run(cmd, dict(env, AMD_COMGR_CACHE="0"))
res["warm"] = [run(cmd, env) for _ in range(5)]
res["warm_fast_exit"] = [run(cmd, dict(env, MIDASPOM_FAST_EXIT="1")) for _ in range(5)]
print(json.dumps(res))
