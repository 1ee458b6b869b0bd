"""One process per GPU: grid slabs + a single gather (the MIDASPOM_MPI.out
job shape, sources/main_MIDASPOM_MPI.c:361-368 and :482-506).

The reference splits the s x s grid into e-row slabs (remainder to rank 0).
Every rank then forms all s columns' per-c coefficient tables, a fixed cost
that does not shrink with the rank count, so the GPU drop-in splits the c
columns instead (round 6): rank r computes columns [c0, c1) -- the same
partition function, row_slab, on the c axis -- for every e, in the devices'
[c][e] layout, where a column slab is one contiguous block; the slabs meet on
rank 0 in ONE collective (torch.distributed gather: RCCL over xGMI with the
"nccl" backend, gloo on CPU), padded to equal size because collectives move
equal-sized buffers.  Every rank builds its tables for the whole grid's max
|c| (mdp_engine_set_cbound), so the gathered grid has the bits of a one-rank
run and the posterior file does not depend on the rank count.  Rank 0
normalises and writes.  The e-row helpers stay for the row-split callers.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import numpy as np


def row_slab(rank: int, world: int, s: int):
    """[r0, r1) rows of rank `rank`: floor(s/N) each, the remainder on rank 0
    (main_MIDASPOM_MPI.c:361-368)."""
    avg, rem = divmod(s, world)
    if rank == 0:
        return 0, avg + rem
    return rank * avg + rem, (rank + 1) * avg + rem


def gather_rows(local, rank: int, world: int, s: int, nc: int, device=None):
    """Gather every rank's row slab (torch tensor [rows, nc], float64) to rank
    0 in one collective.  Returns the full [s, nc] numpy grid on rank 0, None
    elsewhere."""
    import torch
    import torch.distributed as dist

    avg, rem = divmod(s, world)
    cap = avg + rem  # the largest slab (rank 0's)
    dev = local.device if device is None else device
    buf = torch.zeros((cap, nc), dtype=torch.float64, device=dev)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    full = np.empty((s, nc), dtype=np.float64)
    for r in range(world):
        r0, r1 = row_slab(r, world, s)
        full[r0:r1] = parts[r][: r1 - r0].cpu().numpy()
    return full


def gather_cols(local, rank: int, world: int, s: int, nc: int, device=None):
    """The same single gather for slabs in the devices' native [c][e] layout
    (torch tensor [nc, rows], float64: rank r's e rows are its columns).
    Returns on rank 0 the transposed view of the full [nc, s] array -- indexed
    [ie][ic] like gather_rows' result; log_total / write_posterior read it in
    place -- and None elsewhere."""
    import torch
    import torch.distributed as dist

    avg, rem = divmod(s, world)
    cap = avg + rem
    dev = local.device if device is None else device
    buf = torch.zeros((nc, cap), dtype=torch.float64, device=dev)
    buf[:, : local.shape[1]] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    full = np.empty((nc, s), dtype=np.float64)
    for r in range(world):
        r0, r1 = row_slab(r, world, s)
        full[:, r0:r1] = parts[r][:, : r1 - r0].cpu().numpy()
    return full.T


def gather_colslabs(local, rank: int, world: int, ne: int, nc: int, device=None):
    """Gather every rank's column slab (torch tensor [cols, ne], float64: the
    [c][e] layout) to rank 0 in one collective.  Returns on rank 0 the
    transposed view of the full [nc, ne] array -- indexed [ie][ic] like
    gather_rows' result; log_total / write_posterior read it in place -- and
    None elsewhere."""
    import torch
    import torch.distributed as dist

    avg, rem = divmod(nc, world)
    cap = avg + rem
    dev = local.device if device is None else device
    buf = torch.zeros((cap, ne), dtype=torch.float64, device=dev)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    full = np.empty((nc, ne), dtype=np.float64)
    for r in range(world):
        c0, c1 = row_slab(r, world, nc)
        full[c0:c1] = parts[r][: c1 - c0].cpu().numpy()
    return full.T


def distributed_loglik(e, c, rank: int, world: int,
                       compute: Callable[[np.ndarray, np.ndarray], object], device=None):
    """Each rank computes its slab with `compute(e_slab, c)` (a torch tensor
    or numpy array [rows, nc]) and the slabs are gathered to rank 0."""
    import torch

    r0, r1 = row_slab(rank, world, len(e))
    local = compute(np.ascontiguousarray(e[r0:r1]), np.ascontiguousarray(c))
    if not torch.is_tensor(local):
        local = torch.from_numpy(np.asarray(local, dtype=np.float64))
    if device is not None:
        local = local.to(device)
    return gather_rows(local, rank, world, len(e), len(c), device)


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def under_launcher() -> bool:
    """Started by torchrun (the `mpirun -np N` of the _MPI programs): the
    drop-ins then behave as the MPI builds even for N = 1 (banner, per-rank
    lines, the gather), as `mpirun -np 1 MIDASPOM_MPI.out` does."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def gpu_slab_compute(model, device_index: int):
    """compute(e_slab, c) on this rank's GPU through the C ABI; the result
    stays in HBM (a torch tensor [nc, rows]: the [c][e] layout the kernels
    store fastest, MDP_LAYOUT_CE) until the gather (gather_cols)."""
    import torch

    import midaspom_amd as mdp

    eng = mdp.Engine(model, devices=[device_index])
    eng.set_layout("ce")

    def compute(e_slab, c, cbound=0.0):
        """log L of e_slab x c as [len(c), len(e_slab)]; cbound: the whole
        grid's max |c| when c is a column slab of it."""
        out = torch.empty((len(c), len(e_slab)), dtype=torch.float64, device=f"cuda:{device_index}")
        if len(e_slab) and len(c):
            eng.set_cbound(cbound)
            eng.set_grid(e_slab, c)
            eng.run(out.data_ptr(), len(e_slab), torch.cuda.current_stream(device_index).cuda_stream)
        return out

    compute.engine = eng
    return compute


# ---------------------------------------------------------------------------
# forward simulation: replicate ranges + one sum-reduce (future_MPI.c)
# ---------------------------------------------------------------------------
def replicate_range(rank: int, world: int, nsimul: int):
    """[r0, r1) replicates of rank `rank`: floor(nsimul/N) each, the
    remainder on rank 0 (main_MIDASPOM_future_MPI.c:376-383)."""
    return row_slab(rank, world, nsimul)


def reduce_counts(local, rank: int, world: int):
    """Sum every rank's per-year counts (torch int64 tensor [tfut]) onto rank
    0 in ONE collective (the root's MPI_Recv accumulate,
    future_MPI.c:432-444); returns the numpy totals on rank 0, None elsewhere."""
    import torch.distributed as dist

    dist.reduce(local, dst=0, op=dist.ReduceOp.SUM)
    return local.cpu().numpy().astype(np.uint64) if rank == 0 else None


def distributed_future_counts(nsimul: int, rank: int, world: int,
                              compute: Callable[[int, int], object], device=None):
    """Each rank simulates its replicate range with `compute(rep0, nrep)` (a
    torch int64 tensor or numpy array [tfut]) and the counts are summed on
    rank 0.  Replicate r draws from the same addressed stream wherever it runs,
    so the totals do not depend on the world size."""
    import torch

    r0, r1 = replicate_range(rank, world, nsimul)
    local = compute(r0, r1 - r0)
    if not torch.is_tensor(local):
        local = torch.from_numpy(np.asarray(local).astype(np.int64))
    if device is not None:
        local = local.to(device)
    return reduce_counts(local, rank, world)


def gpu_future_compute(fut, tfut: int, seed: int, device_index: int):
    """compute(rep0, nrep) on this rank's GPU through the C ABI; the counts
    stay in HBM (a torch int64 tensor) until the reduce."""
    import torch

    def compute(rep0, nrep):
        out = torch.zeros(tfut, dtype=torch.int64, device=f"cuda:{device_index}")
        if nrep:
            st = torch.cuda.current_stream(device_index).cuda_stream
            fut.simulate_device(out.data_ptr(), nrep, tfut, seed=seed, rep0=rep0, stream=st)
            fut.check(st)  # raises if a draw overflowed the posterior look-back
        return out

    return compute
