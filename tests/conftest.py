"""Shared fixtures.  GPU tests are marked ``@pytest.mark.gpu``; everything
else runs on a CPU-only host (`pytest -m "not gpu"`)."""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running parity case")


def _ensure_built():
    """Build the oracle and the engine in-tree if a fresh checkout lacks them
    (make is incremental; on the GPU box the prebuilt files travel)."""
    if not (ROOT / "oracle" / "_build" / "liboracle.so").exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    if not (ROOT / "midaspom_amd" / "_build" / "libmidaspom.so").exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "midaspom_amd" / "csrc")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(scope="session")
def anchors():
    return json.loads((GOLDEN / "anchors.json").read_text())


def run_by_name(anchors, name):
    for r in anchors["runs"]:
        if r["name"] == name:
            return r
    raise KeyError(name)


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
