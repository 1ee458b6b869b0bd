"""bench.py's multi-rank plumbing on the CPU (gloo): how the job's world is
resolved from --gpus and the launcher's environment, the ranks bench.py
starts itself when no launcher did, and each rank's e-row slabs
(main_MIDASPOM_MPI.c:361-368: the remainder rows go to rank 0)."""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _bench():
    import bench
    return bench


def _args(gpus):
    return argparse.Namespace(gpus=gpus)


def test_resolve_world():
    b = _bench()
    assert b.resolve_world(_args(None), {}) == (1, 0, 0, False)
    assert b.resolve_world(_args(1), {}) == (1, 0, 0, False)
    assert b.resolve_world(_args(4), {}) == (4, 0, 0, True)  # no launcher: bench.py starts the ranks
    env = {"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"}
    assert b.resolve_world(_args(8), env) == (8, 5, 5, False)
    assert b.resolve_world(_args(None), env) == (8, 5, 5, False)
    with pytest.raises(SystemExit):
        b.resolve_world(_args(2), env)  # --gpus contradicts the launcher
    with pytest.raises(SystemExit):
        b.resolve_world(_args(0), {})


def _clean_env():
    return {k: v for k, v in os.environ.items()
            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _check_slabs(res, n):
    assert res["n_gpus"] == n and [r["rank"] for r in res["ranks"]] == list(range(n))
    for cfg, s in (("2", 512), ("3", 1024)):
        rows = [r["strong_rows"][cfg] for r in res["ranks"]]
        assert rows[0][0] == 0 and rows[-1][1] == s
        assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))  # contiguous, in rank order
        assert rows[0][1] - rows[0][0] == s // n + s % n      # the remainder on rank 0
        assert all(r[1] - r[0] == s // n for r in rows[1:])
    assert [r["weak_rows"] for r in res["ranks"]] == [[512 * i, 512 * (i + 1)] for i in range(n)]


def test_gpus_n_starts_n_ranks():
    """`bench.py --gpus 3` with no launcher: three ranks, one process group."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3", "--dry-run", "--backend", "gloo"],
                       capture_output=True, text=True, timeout=240, env=_clean_env(), cwd=str(ROOT))
    assert r.returncode == 0, r.stderr
    _check_slabs(_json_line(r.stdout), 3)


def test_torchrun_launch_unchanged():
    """Under torchrun the launcher's ranks are the job (no second spawn)."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29731", str(ROOT / "bench.py"),
                        "--gpus", "2", "--dry-run", "--backend", "gloo"],
                       capture_output=True, text=True, timeout=240, env=_clean_env(), cwd=str(ROOT))
    assert r.returncode == 0, r.stderr
    _check_slabs(_json_line(r.stdout), 2)
