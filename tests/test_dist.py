"""Multi-process path on CPU: world_size-2/3 gloo ranks shard the grid --
the e rows as main_MIDASPOM_MPI.c:361-368 does, and the c columns as the
drop-in does (dist.py, round 6) -- and gather the slabs to rank 0 in one
collective; the slab compute here is the CPU oracle (the GPU engine is
exercised by the -m gpu tests)."""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

from midaspom_amd import dist as mdist

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("s", [2, 5, 17, 101, 512])
def test_row_slabs_partition(world, s):
    if world > s:
        pytest.skip("more ranks than rows")
    spans = [mdist.row_slab(r, world, s) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == s
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0
    sizes = [b - a for a, b in spans]
    assert sizes[0] == s // world + s % world
    assert all(x == s // world for x in sizes[1:])


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, inp, s, outdir):
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    import oracle
    from midaspom_amd import dist as md
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    om = oracle.OracleModel.load(inp, 400.0, 0.5, 100.0)
    g, win = oracle.grid(s)
    full = md.distributed_loglik(g, g, rank, world, lambda e, c: om.loglik_grid(e, c, threads=1))
    if rank == 0:
        np.save(os.path.join(outdir, "full.npy"), full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_matches_single_process(golden, tmp_path, world):
    import oracle
    s = 9
    inp = str(golden / "config2_64x50.txt")
    mp.spawn(_worker, args=(world, _free_port(), inp, s, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "full.npy")
    om = oracle.OracleModel.load(inp)
    g, _ = oracle.grid(s)
    ref = om.loglik_grid(g, g, threads=1)
    assert np.array_equal(got, ref)


def _ce_worker(rank, world, port, inp, s, outdir):
    """The drop-in's device layout: each rank's slab as [c][e] columns
    (gather_cols), exactly what gpu_slab_compute leaves in HBM."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    import oracle
    from midaspom_amd import dist as md
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    om = oracle.OracleModel.load(inp, 400.0, 0.5, 100.0)
    g, win = oracle.grid(s)
    r0, r1 = md.row_slab(rank, world, s)
    slab = om.loglik_grid(g[r0:r1], g, threads=1)              # [rows][c]
    local = torch.from_numpy(np.ascontiguousarray(slab.T))   # [c][rows]
    full = md.gather_cols(local, rank, world, s, s)
    if rank == 0:
        assert full.shape == (s, s) and full.T.flags.c_contiguous
        np.save(os.path.join(outdir, "full.npy"), np.ascontiguousarray(full))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_cols_matches_single_process(golden, tmp_path, world):
    """[c][e] slabs gathered in one collective give the single-process grid
    (as its transposed view), bit for bit."""
    import oracle
    s = 11
    inp = str(golden / "config2_64x50.txt")
    mp.spawn(_ce_worker, args=(world, _free_port(), inp, s, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "full.npy")
    om = oracle.OracleModel.load(inp)
    g, _ = oracle.grid(s)
    assert np.array_equal(got, om.loglik_grid(g, g, threads=1))


def _colslab_worker(rank, world, port, inp, ne, nc, outdir):
    """The drop-in's split (dist.py, round 6): each rank the c columns
    [c0, c1) for every e, as [cols][e] -- what gpu_slab_compute leaves in
    HBM -- gathered in one collective (gather_colslabs)."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    import oracle
    from midaspom_amd import dist as md
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    om = oracle.OracleModel.load(inp, 400.0, 0.5, 100.0)
    ge, _ = oracle.grid(ne)
    gc, _ = oracle.grid(nc)
    c0, c1 = md.row_slab(rank, world, nc)
    slab = om.loglik_grid(ge, gc[c0:c1], threads=1)           # [e][cols]
    local = torch.from_numpy(np.ascontiguousarray(slab.T))    # [cols][e]
    full = md.gather_colslabs(local, rank, world, ne, nc)
    if rank == 0:
        assert full.shape == (ne, nc) and full.T.flags.c_contiguous
        np.save(os.path.join(outdir, "full.npy"), np.ascontiguousarray(full))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_colslabs_matches_single_process(golden, tmp_path, world):
    """Column slabs (remainder columns on rank 0) gathered in one collective
    give the single-process grid, as its [ie][ic] view, bit for bit."""
    import oracle
    ne, nc = 7, 11
    inp = str(golden / "config2_64x50.txt")
    mp.spawn(_colslab_worker, args=(world, _free_port(), inp, ne, nc, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "full.npy")
    om = oracle.OracleModel.load(inp)
    ge, _ = oracle.grid(ne)
    gc, _ = oracle.grid(nc)
    assert np.array_equal(got, om.loglik_grid(ge, gc, threads=1))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("nsimul", [1, 7, 10000])
def test_replicate_ranges_partition(world, nsimul):
    spans = [mdist.replicate_range(r, world, nsimul) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == nsimul
    assert all(a1 == b0 for (_, a1), (b0, _) in zip(spans, spans[1:]))


def _future_worker(rank, world, port, inp, outdir):
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    import oracle
    from midaspom_amd import dist as md
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _, _, row = oracle.last_row(inp)
    post = np.load(os.path.join(outdir, "post.npy"))
    tot = md.distributed_future_counts(
        5000, rank, world,
        lambda r0, nr: oracle.future_counts(row, post, tfut=20, nrep=nr, rep0=r0, seed=9, m=400, d=100,
                                            KS=0.5, threads=1))
    if rank == 0:
        np.save(os.path.join(outdir, "tot.npy"), tot)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_future_reduce_matches_single_process(golden, tmp_path, world):
    """Replicate ranges per rank + one sum-reduce (future_MPI.c:376-383,
    :432-444) give the single-process counts exactly."""
    import oracle
    inp = str(golden / "occupancies.txt")
    oracle.run(inp, tmp_path / "post.txt", m=400, d=100, s=21)
    post = oracle.read_posterior(tmp_path / "post.txt") * 0.7  # exercise the carry-over across ranks
    np.save(tmp_path / "post.npy", post)
    mp.spawn(_future_worker, args=(world, _free_port(), inp, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "tot.npy")
    _, _, row = oracle.last_row(inp)
    ref = oracle.future_counts(row, post, tfut=20, nrep=5000, seed=9, m=400, d=100, KS=0.5, threads=1)
    assert np.array_equal(got, ref)
