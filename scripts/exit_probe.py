"""Where the drop-in CLI's exit remainder on small grids goes (cli_exit.h).
Times, from the parent on CLOCK_MONOTONIC, the wall after main returns for
scripts/ubench/hipinit_probe (device count + a 1 MiB context touch, then
_exit; variants: sleep before the exit, one thread, pools of busy threads)
and for the CLI on config 1 at s = 50 and 512 with and without its
pre-exit core warm-up (MIDASPOM_EXIT_WARM) -- 5 runs each, interleaved.  One
JSON line per case (rounds 5-6: profiles/r06/analysis/exit_probe_*.jsonl)."""
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

PROBE = ROOT / "scripts" / "ubench" / "hipinit_probe"
tmp = Path(tempfile.mkdtemp())
env = dict(os.environ, MDP_JIT_CACHE=str(tmp / "jit"), MIDASPOM_TIMING="1")
inp = ROOT / "tests" / "golden" / "occupancies.txt"


def stamps(err, key):
    for ln in err.splitlines():
        if ln.startswith(key):
            v = ln.split(":", 1)[1].split()
            return {v[i]: float(v[i + 1]) for i in range(0, len(v) - 1, 2)}
    return None


def run(cmd, key, extra=None):
    t0 = time.monotonic()
    r = subprocess.run(cmd, env=dict(env, **(extra or {})), capture_output=True, text=True)
    t1 = time.monotonic()
    assert r.returncode == 0, r.stderr[-500:]
    st = stamps(r.stderr, key)
    return {"wall": round(t1 - t0, 4), "before_main": round(st["main_entry"] - t0, 4),
            "main": round(st["main_return"] - st["main_entry"], 4), "after_main": round(t1 - st["main_return"], 4)}


cases = {f"probe_sleep{ms}": ([str(PROBE), "ctx", "fast", f"sleep={ms}"], "hipinit_probe clock:", None) for ms in (0,)}
cases["probe_pool16"] = ([str(PROBE), "ctx", "fast", "pool=16"], "hipinit_probe clock:", None)
cli = lambda s: [str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", str(s), "-i", str(inp), "-o", str(tmp / "p.txt")]
for s in (50, 512):
    cases[f"cli_s{s}"] = (cli(s), "midaspom clock (s):", None)  # default: 16 cores warmed 2 ms before _exit
    cases[f"cli_s{s}_nowarm"] = (cli(s), "midaspom clock (s):", {"MIDASPOM_EXIT_WARM": "0"})
for w in ("16,500", "8,2000", "4,2000"):
    cases[f"cli_s50_warm{w}"] = (cli(50), "midaspom clock (s):", {"MIDASPOM_EXIT_WARM": w})
run(*cases["cli_s50"][:2])  # fill the code-object cache
res = {k: [] for k in cases}
for _ in range(5):
    for k, (cmd, key, extra) in cases.items():
        res[k].append(run(cmd, key, extra))
for k, v in res.items():
    med = {f: sorted(x[f] for x in v)[len(v) // 2] for f in v[0]}
    print(json.dumps({"case": k, "median": med, "runs": v}), flush=True)
