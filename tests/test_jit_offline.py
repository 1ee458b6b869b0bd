"""The problem-specialised forward kernels (csrc/spom_jit.cpp) compile for
gfx950 on a CPU-only host: with MDP_JIT_CHECK=1 and no HIP device,
mdp_engine_create plans the problem, generates both forward variants (fused
and Q-row reading) and compiles them with hipRTC, then reports MDP_ENODEV.
Catches generator bugs (e.g. zero-sized LDS arrays when every column is
variable) before a GPU run.  Runs in a subprocess so the environment knobs do
not leak into other tests."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

from conftest import gpu_available

ROOT = Path(__file__).resolve().parents[1]

SCRIPT = r"""
import sys
sys.path.insert(0, {root!r})
import midaspom_amd as mdp
from midaspom_amd import synth
src = {src!r}
if src.startswith("synth:"):
    name = src.split(":", 1)[1]
    path = synth.write({tmp!r} + "/in.txt", **getattr(synth, name))
else:
    path = src
model = mdp.Model.load(path)
try:
    mdp.Engine(model, devices=[0])
except mdp.MidaspomError as ex:
    msg = str(ex)
    assert "forward kernels compiled" in msg, msg
    print("ok")
else:
    raise SystemExit("engine creation succeeded without a device")
"""

CASES = [
    str(ROOT / "tests" / "golden" / "occupancies.txt"),   # n = nvar = 8: no always-zero column
    str(ROOT / "tests" / "golden" / "manual_p3_obs.txt"),
    "synth:CONFIG2",
    "synth:CONFIG3",
]


@pytest.mark.skipif(gpu_available(), reason="offline compile check runs on CPU-only hosts")
@pytest.mark.parametrize("src", CASES, ids=[Path(c).name for c in CASES])
def test_forward_kernels_compile_offline(src, tmp_path):
    env = dict(os.environ, MDP_JIT_CHECK="1", MDP_JIT_NOCACHE="1")
    code = SCRIPT.format(root=str(ROOT), src=src, tmp=str(tmp_path))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(gpu_available(), reason="offline planning check runs on CPU-only hosts")
@pytest.mark.parametrize("row0,wide,expect", [
    ([1, -1, -1, -1, -1, -1, -1, 1], "", "forward kernels compiled"),   # 64 states: LDS-state kernel
    ([1, -1, -1, -1, -1, -1, -1, 1], "1", "wide path planned"),         # forced onto the wide kernels
    ([-1, -1, -1, -1, -1, -1, -1, 1], "", "wide path planned"),         # 128 states: the wide kernels
])
def test_wide_years_plan_offline(row0, wide, expect):
    """Years with 6-7 missing patches (64 / 128 states) plan instead of
    being refused (main_MIDASPOM.c:225-251 takes any count): up to 64
    states on the specialised kernel with its states in LDS, beyond that
    (or with MDP_WIDE=1) on the wide kernels."""
    code = (f"import sys; sys.path.insert(0, {str(ROOT)!r})\n"
            "import numpy as np, midaspom_amd as mdp\n"
            f"obs = np.array([{row0!r}, [1, 1, 0, 1, 0, 1, 1, 0], [1, 0, 0, 1, 1, 1, 0, 1]])\n"
            "try:\n    mdp.Engine(mdp.Model.from_obs(obs), devices=[0])\n"
            f"except mdp.MidaspomError as ex:\n    assert {expect!r} in str(ex), str(ex); print('ok')\n")
    env = dict(os.environ, MDP_JIT_CHECK="1")
    env.pop("MDP_WIDE", None)
    if wide:
        env["MDP_WIDE"] = wide
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(gpu_available(), reason="offline planning check runs on CPU-only hosts")
def test_qrows_slot_colouring_offline(tmp_path):
    """k_qrows' Pc slots (spom_engine.hip build_direct_plan): coloured so the
    phase-3 gathers (16-lane groups, slots distinct mod 16) and the phase-2
    stores (8 consecutive items, distinct mod 8) meet few bank conflicts, in
    about as many slots as items.  Config 3: 416 gather groups, 236 store
    groups; the plan reports the extra cycles the colouring leaves."""
    import re
    env = dict(os.environ, MDP_JIT_CHECK="1")
    code = SCRIPT.format(root=str(ROOT), src="synth:CONFIG3", tmp=str(tmp_path)).replace(
        '    assert "forward kernels compiled" in msg, msg\n    print("ok")',
        '    print(msg)')
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    m = re.search(r"nitems (\d+) .*qrows slots (\d+) conflicts (\d+) \+ (\d+)", r.stdout)
    assert m, r.stdout + r.stderr
    nitems, slots, gather, store = map(int, m.groups())
    assert nitems == 1881
    assert slots <= nitems + 16 + 64          # 16 zero slots, little slack
    assert gather <= 32 and store <= 96       # of 416 / 236 groups
