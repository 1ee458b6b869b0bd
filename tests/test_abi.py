"""The C-ABI library loads and exports every symbol include/*.h declares; the
CLI binary links against it.  No compute calls (CPU host)."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from midaspom_amd import _lib

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    names = []
    for h in sorted((ROOT / "include").glob("*.h")):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names += re.findall(r"\b(mdp_\w+)\s*\(", text)
    return sorted(set(names))


def test_header_declares_abi():
    names = declared_functions()
    assert "mdp_engine_create" in names and "mdp_loglik_grid" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert set(declared_functions()) == bound


def test_abi_version():
    assert _lib.lib().mdp_abi_version() == 9


def test_engine_library_is_gfx950():
    """The fat binary embedded in the library carries a gfx950 code object."""
    blob = _lib.LIB_PATH.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_cli_links(tmp_path):
    r = subprocess.run(["ldd", str(_lib.CLI_PATH)], capture_output=True, text=True)
    assert "libmidaspom.so" in r.stdout and "not found" not in r.stdout.split("libmidaspom.so")[1].splitlines()[0]


def test_cli_unknown_option():
    r = subprocess.run([str(_lib.CLI_PATH), "-z"], capture_output=True, text=True)
    assert r.returncode == 1
    assert "Unknown option `-z'." in r.stderr
    assert r.stdout.startswith("------ MIDASPOM, beta version ------\n")


def test_scenario_and_future_cli_argument_errors(tmp_path):
    """The other drop-ins' argument handling (no GPU needed): unknown option
    -> the getopt message and exit 1; dieoff / loss without -a -e -c -> exit 1
    (quirk Q11); a missing input file -> exit 1 with its name."""
    for exe in (_lib.DIEOFF_CLI_PATH, _lib.LOSS_CLI_PATH, _lib.FUTURE_CLI_PATH):
        r = subprocess.run([str(exe), "-z"], capture_output=True, text=True)
        assert r.returncode == 1 and "Unknown option `-z'." in r.stderr, exe
        assert "beta" in r.stdout.splitlines()[0]
    for exe in (_lib.DIEOFF_CLI_PATH, _lib.LOSS_CLI_PATH):
        r = subprocess.run([str(exe), "-e", "0.3", "-c", "0.4"], capture_output=True, text=True)
        assert r.returncode == 1 and "-a" in r.stderr
        r = subprocess.run([str(exe), "-a", "1", "-e", "0.3", "-c", "0.4", "-i", str(tmp_path / "none.txt")],
                           capture_output=True, text=True)
        assert r.returncode == 1 and "none.txt" in r.stderr
    r = subprocess.run([str(_lib.FUTURE_CLI_PATH), "-i", str(tmp_path / "none.txt")], capture_output=True, text=True)
    assert r.returncode == 1
