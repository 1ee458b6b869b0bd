"""Config-1 CLI warm set-up probe (GPU box): cold, then warm runs with the
compiler-side cache on and off, listing the hipRTC code-object cache after
each run -- does the warm run hit the engine's own cache?  One line per run."""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from midaspom_amd import _lib  # noqa: E402

tmp = Path(tempfile.mkdtemp())
inp = ROOT / "tests" / "golden" / (sys.argv[1] if len(sys.argv) > 1 else "occupancies.txt")
s = sys.argv[2] if len(sys.argv) > 2 else "50"
cache = tmp / "cache" / "config1"
cmd = [str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", s, "-i", str(inp), "-o", str(tmp / "p.txt")]
cdir = str(tmp / "comgr")
for leg, extra in [("cold", {"AMD_COMGR_CACHE": "0"}), ("warm", {}), ("warm_nocomgr", {"AMD_COMGR_CACHE": "0"}),
                   ("warm", {}), ("nocache", {"MDP_JIT_NOCACHE": "1", "AMD_COMGR_CACHE": "0"}),
                   ("warm_newcomgrdir", {"AMD_COMGR_CACHE_DIR": cdir}), ("warm_newcomgrdir", {"AMD_COMGR_CACHE_DIR": cdir}),
                   ("warm_newcomgrdir", {"AMD_COMGR_CACHE_DIR": cdir}),
                   ("warm_rtunbundle", {"AMD_COMGR_CACHE_DIR": cdir + "2", "HIP_USE_RUNTIME_UNBUNDLER": "1"}),
                   ("warm_rtunbundle", {"AMD_COMGR_CACHE_DIR": cdir + "2", "HIP_USE_RUNTIME_UNBUNDLER": "1"}),
                   ("warm_nocomgr_rtunbundle", {"AMD_COMGR_CACHE": "0", "HIP_USE_RUNTIME_UNBUNDLER": "1"})]:
    env = dict(os.environ, MDP_JIT_CACHE=str(cache), MIDASPOM_TIMING="1", MDP_SETUP_TIMING="1", **extra)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True)
    split = [ln for ln in r.stderr.splitlines() if ln.startswith("midaspom timing") or ln.startswith("mdp setup")]
    files = sorted((p.name, p.stat().st_size) for p in cache.glob("*")) if cache.exists() else []
    cfiles = sum(1 for _ in Path(cdir).rglob("*")) if Path(cdir).exists() else 0
    print(leg, r.returncode, split, files, "comgr-dir entries", cfiles, flush=True)

# the same first-use cost for a one-kernel program (scripts/ubench/tiny_launch)
tiny = str(ROOT / "scripts" / "ubench" / "tiny_launch")
for leg, extra in [("tiny_newcomgrdir", {"AMD_COMGR_CACHE_DIR": cdir + "3"}), ("tiny_newcomgrdir", {"AMD_COMGR_CACHE_DIR": cdir + "3"}),
                   ("tiny_nocomgr", {"AMD_COMGR_CACHE": "0"})]:
    r = subprocess.run([tiny], env=dict(os.environ, **extra), capture_output=True, text=True)
    print(leg, r.returncode, [ln for ln in r.stderr.splitlines() if ln.startswith("tiny_launch")], flush=True)
