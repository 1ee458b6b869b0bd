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
        rows = [r["strong_cols"][cfg] for r in res["ranks"]]
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


def test_projection_record():
    """The one-GPU strong-scaling projection (bench.project_likelihood /
    project_dieoff): per N the slowest rank's slab against the one-GPU pass,
    and the bytes rank 0 receives in the job's one gather."""
    b = _bench()
    p = b._project(10.0, {2: [5.5, 5.0], 4: [3.0, 2.5, 2.5, 2.5], 8: [2.0] + [1.25] * 7}, 1024 * 1024 * 8)
    assert set(p) == {"2", "4", "8"}
    assert p["2"]["max_slab_ms"] == 5.5 and p["2"]["projected_speedup"] == pytest.approx(10 / 5.5)
    assert p["8"]["projected_speedup"] == pytest.approx(5.0)
    assert p["4"]["gather_bytes_to_rank0"] == 1024 * 1024 * 8 * 3 // 4
    assert b.PROJ_NS == (2, 4, 8)


def test_coll_name():
    b = _bench()
    assert b._coll_name(argparse.Namespace(backend="nccl")) == "RCCL"
    assert b._coll_name(argparse.Namespace(backend="gloo")) == "gloo"


@pytest.mark.gpu
def test_projection_legs_on_gpu():
    """The projection legs the default N = 1 line carries, on config 2 (both
    splits) and a small die-off grid: every rank's slab timed, speedups > 0."""
    import torch
    b = _bench()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    res = b.projection_block(argparse.Namespace(grid4=32), dev, stream, [2, 4])
    for key, splits in (("config2", ("split_e", "split_c")), ("config4", ("split_e",))):
        r = res[key]
        assert "error" not in r, r
        assert r["one_gpu_ms"] > 0
        for sp in splits:
            for n in b.PROJ_NS:
                rec = r[sp][str(n)]
                assert len(rec["slab_ms"]) == n and rec["projected_speedup"] > 0
