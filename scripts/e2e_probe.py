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
c2 = synth.write(tmp / "c2.txt", **synth.CONFIG2)
inputs = {"config1": (ROOT / "tests" / "golden" / "occupancies.txt", 50),
          "config2": (c2, 512),
          # the same programs on the other grid size: is the exit cost the
          # problem's or the grid's?
          "config1_s512": (ROOT / "tests" / "golden" / "occupancies.txt", 512),
          "config2_s50": (c2, 50)}
env = dict(os.environ, MDP_JIT_CACHE=str(tmp / "jit"), MIDASPOM_TIMING="1")


def run(name, extra, files=False):
    """(files: stdout / stderr to files instead of pipes -- a process that
    holds an inherited pipe open past the CLI's exit would delay a pipe's
    EOF, not the exit)"""
    inp, s = inputs[name]
    cmd = [str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", str(s), "-i", str(inp), "-o", str(tmp / "p.txt")]
    t0 = time.monotonic()
    if files:
        with open(tmp / "o.txt", "w") as fo, open(tmp / "e.txt", "w") as fe:
            rc = subprocess.run(cmd, env=dict(env, **extra), stdout=fo, stderr=fe).returncode
        t1 = time.monotonic()
        err = (tmp / "e.txt").read_text()
    else:
        r = subprocess.run(cmd, env=dict(env, **extra), capture_output=True, text=True)
        t1 = time.monotonic()
        rc, err = r.returncode, r.stderr
    assert rc == 0, err[-800:]
    out = {"wall": round(t1 - t0, 4)}
    for ln in err.splitlines():
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
for name in inputs:  # fill the caches
    run(name, {})
if os.environ.get("E2E_MALLOC"):
    # E2E_MALLOC=1: the exit cost against where glibc puts the output buffer
    # (mmap threshold forced low: every buffer mmapped and unmapped by free;
    # forced high: every buffer on the brk heap)
    for sz in (50, 200, 512):
        inputs[f"config1_s{sz}x"] = (inputs["config1"][0], sz)
    for rep in range(3):
        for sz in (50, 200, 512):
            for vn, extra in (("default", {}), ("mmap4k", {"MALLOC_MMAP_THRESHOLD_": "4096"}),
                              ("heap", {"MALLOC_MMAP_THRESHOLD_": "1073741824"})):
                res.setdefault(f"config1_s{sz}_{vn}", []).append(run(f"config1_s{sz}x", extra))
    print(json.dumps(res))
    sys.exit(0)
if os.environ.get("E2E_SIZES"):
    # E2E_SIZES=1: config 1's problem over grid sizes (where does the exit cost start?)
    for sz in (50, 100, 150, 200, 300, 512):
        inputs[f"config1_s{sz}x"] = (inputs["config1"][0], sz)
        run(f"config1_s{sz}x", {})
    for rep in range(3):
        for sz in (50, 100, 150, 200, 300, 512):
            res.setdefault(f"config1_s{sz}", []).append(run(f"config1_s{sz}x", {}))
    print(json.dumps(res))
    sys.exit(0)
if os.environ.get("E2E_VARIANTS"):
    # E2E_VARIANTS=1: configs 1 at s = 50 and 512 under runtime settings that
    # could make the exit's cost (copy engines off, one hardware queue)
    variants = {"base": {}, "sdma0": {"HSA_ENABLE_SDMA": "0"}, "hwq1": {"GPU_MAX_HW_QUEUES": "1"},
                "sdma0_hwq1": {"HSA_ENABLE_SDMA": "0", "GPU_MAX_HW_QUEUES": "1"}}
    for rep in range(3):
        for vn, extra in variants.items():
            for name in ("config1", "config1_s512"):
                res.setdefault(f"{name}_{vn}", []).append(run(name, extra))
    print(json.dumps(res))
    sys.exit(0)
for rep in range(3):
    for name in inputs:
        for mode, extra in (("quick", {}), ("full", {"MIDASPOM_FULL_EXIT": "1"})):
            res.setdefault(f"{name}_{mode}", []).append(run(name, extra))
        res.setdefault(f"{name}_quick_files", []).append(run(name, {}, files=True))
print(json.dumps(res))
