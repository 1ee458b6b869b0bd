"""Engine options (ABI 7) and the hipRTC code-object cache, on a CPU host.

* The library reads no tuning knob from the environment: kernel variants are
  chosen by mdp_engine_create_opts' options string.  Unknown names and the
  measurement-only names (MDP_DIAG, MDP_JIT_HACK, MDP_JIT_WPE) are refused by
  the default library; the diag library (libmidaspom_diag.so) accepts them.
* A cached code object is used only if its trailer names the cache key of
  the source being compiled (source, compile options, hipRTC version): a
  stale, corrupted or foreign file under the key is rebuilt, not loaded (a
  staleness / corruption check).  The cache directory itself is used only
  while it is private to this user (0700-created, owned by the user, not
  group- or world-writable), which is what keeps other users' objects out.

Each case runs in a subprocess (the library is loaded once per process)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

from conftest import gpu_available

ROOT = Path(__file__).resolve().parents[1]
BUILD = ROOT / "midaspom_amd" / "_build"

PRELUDE = r"""
import ctypes, sys
sys.path.insert(0, {root!r})
import midaspom_amd as mdp
from midaspom_amd import _lib
model = mdp.Model.load({root!r} + "/tests/golden/occupancies.txt")
L = _lib.lib()
def create(opts, c_plain=False):
    h = ctypes.c_void_p()
    if c_plain:
        rc = L.mdp_engine_create(ctypes.byref(model.problem), None, 0, ctypes.byref(h))
    else:
        rc = L.mdp_engine_create_opts(ctypes.byref(model.problem), None, 0, opts, ctypes.byref(h))
    return rc, L.mdp_last_error().decode()
"""


def run(code, env_extra=None):
    env = {k: v for k, v in os.environ.items() if not k.startswith("MDP_") and k != "MIDASPOM_DIAG_LIB"}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, "-c", PRELUDE.format(root=str(ROOT)) + code], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.skipif(gpu_available(), reason="checks option parsing up to the device probe (CPU hosts)")
def test_options_parsed_and_environment_ignored():
    out = run(r"""
rc, msg = create(b"MDP_NO_SUCH=1")
assert rc == -1 and "unknown engine option" in msg, (rc, msg)
for bad in (b"MDP_JIT_HACK=1", b"MDP_DIAG=1", b"MDP_JIT_WPE=3"):
    rc, msg = create(bad)
    assert rc == -1 and "measurement-only" in msg, (bad, rc, msg)
# variant options pass the parser (then: no device)
rc, msg = create(b"MDP_FUSED=1;MDP_JIT_CHUNK=64, MDP_EPL=1")
assert rc == -5, (rc, msg)
# MDP_JIT_HACK in the environment is not read by the library
rc, msg = create(None, c_plain=True)
assert rc == -5, (rc, msg)
# ... and the Python layer does not forward it from the environment to the
# default library (a warning, then the plain engine: no device here) ...
import warnings
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    try:
        mdp.Engine(model)
    except mdp.MidaspomError as ex:
        assert "MDP_ENODEV" in str(ex), ex
    else:
        raise SystemExit("no device, yet created")
assert any("measurement-only" in str(x.message) for x in w), [str(x.message) for x in w]
# ... while an explicit option of that name is refused
try:
    mdp.Engine(model, options="MDP_JIT_HACK=1")
except mdp.MidaspomError as ex:
    assert "measurement-only" in str(ex), ex
else:
    raise SystemExit("accepted")
print("ok")
""", {"MDP_JIT_HACK": "1"})
    assert "ok" in out


@pytest.mark.skipif(gpu_available(), reason="CPU hosts")
@pytest.mark.skipif(not (BUILD / "libmidaspom_diag.so").exists(), reason="diag library not built")
def test_diag_library_accepts_measurement_options():
    out = run(r"""
assert "diag" in L._name
rc, msg = create(b"MDP_JIT_HACK=1;MDP_DIAG=1")
assert rc == -5, (rc, msg)
print("ok")
""", {"MIDASPOM_DIAG_LIB": "1"})
    assert "ok" in out


@pytest.mark.skipif(gpu_available(), reason="offline compile check runs on CPU-only hosts")
def test_jit_cache_rejects_stale_and_foreign_objects(tmp_path):
    """Compile config 1's forward kernels into an empty cache; then replace
    every cached file by garbage, by a bare gfx950 ELF without our trailer,
    and by another key's (valid) file: each time the engine recompiles, and
    the cache again holds trailer-stamped objects."""
    cache = tmp_path / "jit"
    code = r"""
import os
os.environ.pop("MDP_JIT_NOCACHE", None)
rc, msg = create(b"MDP_JIT_CHECK=1")
assert rc == -5 and "forward kernels compiled" in msg, msg
print("ok")
"""
    env = {"MDP_JIT_CACHE": str(cache)}
    assert "ok" in run(code, env)
    files = sorted(cache.glob("fwd_*.co"))
    assert len(files) == 2, files  # fused + reading variants
    good = {f: f.read_bytes() for f in files}
    for f, b in good.items():
        assert b[:4] == b"\x7fELF" and b[-16:-12] == b"MDPJ"
    plants = [
        lambda f: b"not a code object" * 10,
        lambda f: good[f][:-16],                   # a bare ELF: no trailer naming the key
        lambda f: good[files[1 - files.index(f)]],  # another key's stamped object
    ]
    for plant in plants:
        for f in files:
            f.write_bytes(plant(f))
        assert "ok" in run(code, env)
        for f in files:
            assert f.read_bytes() == good[f], f.name


def _gpu_option_cases():
    import ast
    tree = ast.parse((ROOT / "tests" / "test_gpu_options.py").read_text())
    vals = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and isinstance(node.targets[0], ast.Name) \
                and node.targets[0].id in ("VARIANTS", "TOOLING"):
            vals[node.targets[0].id] = ast.literal_eval(node.value)
    return vals["VARIANTS"], vals["TOOLING"]


def test_every_accepted_option_has_a_parity_case():
    """Every option name the default library accepts (the Python mirror
    ENGINE_OPTION_NAMES, checked against the C list below) is set by some
    case of tests/test_gpu_options.py (oracle parity on the GPU), or is a
    tooling option that selects no kernel."""
    from midaspom_amd import _lib
    variants, tooling = _gpu_option_cases()
    used = set()
    for opts, _ in variants:
        for kv in opts.split(";"):
            used.add(kv.split("=")[0])
    accepted = [n for n in _lib.ENGINE_OPTION_NAMES if n not in _lib.DIAG_OPTION_NAMES]
    missing = [n for n in accepted if n not in used and n not in tooling]
    assert not missing, f"options with no GPU parity case: {missing}"
    assert used <= set(accepted), used - set(accepted)


@pytest.mark.skipif(gpu_available(), reason="checks option parsing up to the device probe (CPU hosts)")
def test_c_library_accepts_exactly_the_python_list():
    """The C library's option list equals _lib.ENGINE_OPTION_NAMES: each
    name passes the parser (then: no device), and the round-4 measured-off
    variants (removed in round 5) are unknown."""
    out = run(r"""
for name in _lib.ENGINE_OPTION_NAMES:
    if name in _lib.DIAG_OPTION_NAMES:
        continue
    rc, msg = create((name + "=1").encode())
    assert rc == -5, (name, rc, msg)
for name in ("MDP_FUSED_SBUILD", "MDP_FUSED_BAL", "MDP_FUSED_PH2FLAT", "MDP_FUSED_CMERGE", "MDP_FUSED_DIRECT",
             "MDP_JIT_EARLYW", "MDP_FUSED_QFLAT"):
    rc, msg = create((name + "=1").encode())
    assert rc == -1 and "unknown engine option" in msg, (name, rc, msg)
print("ok")
""")
    assert "ok" in out


@pytest.mark.skipif(gpu_available(), reason="offline compile check runs on CPU-only hosts")
def test_jit_cache_ignores_a_shared_directory(tmp_path):
    """A cache directory that others can write to is neither read nor
    written: the engine compiles, the directory stays empty; made private
    again, the cache fills."""
    cache = tmp_path / "shared"
    cache.mkdir()
    os.chmod(cache, 0o777)
    code = r"""
import os
os.environ.pop("MDP_JIT_NOCACHE", None)
rc, msg = create(b"MDP_JIT_CHECK=1")
assert rc == -5 and "forward kernels compiled" in msg, msg
print("ok")
"""
    env = {"MDP_JIT_CACHE": str(cache)}
    assert "ok" in run(code, env)
    assert not list(cache.iterdir())
    os.chmod(cache, 0o700)
    assert "ok" in run(code, env)
    assert len(list(cache.glob("fwd_*.co"))) == 2


def test_integration_option_table():
    """INTEGRATION.md §4 names only options the default library accepts (the
    Python mirror, itself checked against the C list above), the scenario
    options, the environment-read cache / timing variables, the diag-only
    names (said to be diag-only) and the round-4 names it says were deleted
    (which the library refuses)."""
    import re
    from midaspom_amd import _lib
    text = (ROOT / "INTEGRATION.md").read_text()
    sec = text[text.index("## 4. Engine options"):text.index("## 5.")]
    names = set(re.findall(r"MDP_[A-Z0-9_]+", sec))
    accepted = set(_lib.ENGINE_OPTION_NAMES) - set(_lib.DIAG_OPTION_NAMES)
    env_read = {"MDP_JIT_CACHE", "MDP_JIT_NOCACHE", "MDP_SETUP_TIMING"}
    diag = set(_lib.DIAG_OPTION_NAMES)
    deleted = {"MDP_FUSED_SBUILD", "MDP_FUSED_BAL", "MDP_FUSED_PH2FLAT", "MDP_FUSED_CMERGE", "MDP_FUSED_DIRECT",
               "MDP_JIT_EARLYW"}
    unknown = names - accepted - set(_lib.SCENARIO_OPTION_NAMES) - env_read - diag - deleted - {"MDP_EINVAL"}
    assert not unknown, f"INTEGRATION.md §4 names options the library does not accept: {sorted(unknown)}"
    for sentence in re.split(r"(?<=[.;])\s", sec):
        if any(n in sentence for n in deleted):
            assert "deleted" in sentence and "refuses" in sentence, sentence
        if any(n in sentence for n in diag):
            assert "diag" in sentence, sentence
    assert "MDP_WIDE_MMA" in names and "k_fwd_mmt" in sec
