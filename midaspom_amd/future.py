"""`python -m midaspom_amd.future [flags]` -- MIDASPOM_future over the GPU
replicate engine.

Single process: the same flags, code defaults, stdout lines and output file
as the compiled drop-in `midaspom_future` (midaspom_amd/csrc/midaspom_future_cli.c;
reference sources/main_MIDASPOM_future.c:113-415).  Extensions as there:
`-r <seed>` (default $MIDASPOM_SEED or time(NULL)) and `-g N` (or
MIDASPOM_GPUS=N): the replicates in N contiguous ranges, one thread and
engine per range, the ranges dealt round-robin over the visible GPUs.

Under torchrun (WORLD_SIZE > 1, one process per GPU): the drop-in for
`mpirun -np N MIDASPOM_future_MPI.out` -- the replicates split into
contiguous ranges (remainder to rank 0, main_MIDASPOM_future_MPI.c:376-383),
one sum-reduce of the per-year counts to rank 0 (:429-446), and that
program's per-rank stdout lines (`npstates =` :320, start / end :372, :427,
send / gather :430-445).  Rank 0 writes the file.

Replicate r draws from the Philox stream addressed by (seed, r) wherever it
runs, so the file does not depend on N or on the split (rank 0's seed is
broadcast).  The reference's rand() stream is matched statistically only
(DESIGN.md §12).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

BANNER = "------MIDASPOM, beta MPI version -------\n-> N. Alcala, E. M. Cole, N. A. Rosenberg  <-\n"


def parse_args(argv):
    # getopt "n:a:m:p:q:d:i:o:S:s:D:" and the code defaults (future.c:123-140)
    ap = argparse.ArgumentParser(prog="midaspom_future")
    ap.add_argument("-n", type=int, default=10000, help="replicates")
    ap.add_argument("-a", type=int, default=50, help="years in the future")
    ap.add_argument("-m", type=float, default=400.0, help="mean dispersal distance")
    ap.add_argument("-p", type=float, default=0.5, help="prior occupancy of missing patches")
    ap.add_argument("-q", default="posterior.txt", help="posterior of (e, c)")
    ap.add_argument("-d", type=float, default=200.0, help="segment length")
    ap.add_argument("-i", default="input.txt", help="occupancy file (last row used)")
    ap.add_argument("-o", default="pext_future.txt")
    ap.add_argument("-S", type=float, default=0.0, help="source strength K_S")
    ap.add_argument("-s", type=float, default=200.0, help="distance to the source")
    ap.add_argument("-D", type=float, default=1.0, help="K_D (the code's default, not the manual's 0)")
    ap.add_argument("-r", default=None, help="seed (default $MIDASPOM_SEED or time(NULL))")
    ap.add_argument("-g", type=int, default=None,
                    help="GPUs (single process): replicate ranges, one thread each (default MIDASPOM_GPUS or 1)")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default nccl)")
    return ap.parse_args(argv)


def _completions(row, p):
    """The last survey's completions and their priors as the drop-in prints
    them (future.c:286-332): missing patches in order, the first missing the
    most significant bit; pr in float arithmetic times a double."""
    n = row.size
    miss = [j for j in range(n) if row[j] == -1]
    nm = len(miss)
    np_ = 1 << nm if nm < 31 else 0
    out = []
    for k in range(np_):
        pr = 1.0
        q = 0
        vals = []
        for j in range(n):
            v = int(row[j])
            if v == -1:
                bit = (k >> (nm - 1 - q)) & 1
                q += 1
                v = bit
                pr *= float(np.float32(np.float32(bit) * np.float32(p)) +
                            np.float32(np.float32(1 - bit) * np.float32(1 - np.float32(p))))
            vals.append(v)
        out.append((vals, pr))
    return np_, out


def _simulate_threads(mdp, mdist, row, post, a, seed, ngpu):
    """Single-process -g N: replicate ranges (the MPI partition), one thread
    and engine each, dealt round-robin over the visible GPUs; the ctypes
    calls release the GIL, so the ranges run together."""
    import threading

    ndev = max(1, mdp.device_count())
    parts = [None] * ngpu
    errs = []

    def run(r):
        r0, r1 = mdist.replicate_range(r, ngpu, a.n)
        try:
            with mdp.Future(row, post, m=a.m, d=a.d, KD=a.D, KS=a.S, dS=a.s, device=r % ndev) as f:
                parts[r] = f.simulate(r1 - r0, a.a, seed=seed, rep0=r0) if r1 > r0 else np.zeros(a.a, np.uint64)
        except Exception as exc:  # re-raised on the main thread
            errs.append(exc)

    th = [threading.Thread(target=run, args=(r,)) for r in range(1, ngpu)]
    for t in th:
        t.start()
    run(0)
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return np.sum(np.stack(parts), axis=0, dtype=np.uint64)


def main(argv=None) -> int:
    import midaspom_amd as mdp
    from midaspom_amd import dist as mdist

    argv = sys.argv[1:] if argv is None else argv
    rank, world, local = mdist.env_rank_world()
    root = rank == 0
    mpi = world > 1 or mdist.under_launcher()

    def out(text, all_ranks=False):
        if root or all_ranks:
            sys.stdout.write(text)
            sys.stdout.flush()

    out(BANNER)  # root-only in the MPI build (:128-129)
    try:
        a = parse_args(argv)
    except SystemExit as ex:
        return int(ex.code or 0)
    seed_txt = a.r if a.r is not None else os.environ.get("MIDASPOM_SEED")
    seed = int(seed_txt, 0) if seed_txt is not None else int(time.time())
    out(f"{a.a} years in the future\n")
    out(f"Reading observations from file {a.i}... ")
    try:
        n, tmax, row = mdp.read_survey(a.i)
    except mdp.MidaspomError as ex:
        sys.stderr.write(f"{ex}\n")
        return 1
    out("Last occupancy survey:\n" + "".join(f"{int(v)} " for v in row) + "\n")
    out("\n done\n")
    out(f"Number of habitat patches: {n}\nNumber of sampled years: {tmax}\n")
    out(f"Reading posterior distribution from file {a.q}... ")
    try:
        post = mdp.read_posterior(a.q)
    except mdp.MidaspomError as ex:
        sys.stderr.write(f"{ex}\n")
        return 1
    out(f"{post.shape[0]}X{post.shape[0]} posterior distribution\n")
    inv = 1.0 / a.m
    out("Migration matrix:\n")
    for i in range(n + 1):
        cells = []
        for j in range(n):
            if i == n:
                v = np.exp(-inv * (j + 1) * a.s)
            elif i == j:
                v = 0.0
            else:
                v = np.exp(-inv * abs(i - j) * a.d)
            cells.append(f"{v:.3f} ")
        out("".join(cells) + "\n")
    np_, comps = _completions(row, a.p)
    out(f"npstates = {np_}\n", all_ranks=True)  # unguarded in the MPI build (:320)
    out("Last occupancy survey:\n")
    for vals, pr in comps:
        out("\t" + "".join(f"{v} " for v in vals) + f"; pr={pr:.6f}\n")
    start = int(time.time())
    if not mpi:
        out("Starting likelihood computation\n")
        ngpu = a.g if a.g is not None else int(os.environ.get("MIDASPOM_GPUS", "1"))
        ngpu = max(1, min(ngpu, a.n)) if a.n > 0 else 1
        if a.a > 0 and a.n > 0:
            counts = _simulate_threads(mdp, mdist, row, post, a, seed, ngpu)
        else:
            counts = np.zeros(max(a.a, 0), np.uint64)
        out("end likelihood computation\n")
    else:
        import torch
        import torch.distributed as dist

        backend = a.backend or "nccl"
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            tdev = torch.device("cuda", dev)
        else:
            dist.init_process_group(backend)
            tdev = torch.device("cpu")
        s = torch.tensor([seed], dtype=torch.int64, device=tdev)
        dist.broadcast(s, src=0)  # one stream for all ranks (the reference seeds each rank by time, Q12)
        seed = int(s.item())
        out(f"Starting parallel likelihood computation process {rank + 1}/{world}\n", all_ranks=True)
        r0, r1 = mdist.replicate_range(rank, world, a.n)
        local_counts = np.zeros(max(a.a, 0), np.uint64)
        if a.a > 0 and r1 > r0:
            with mdp.Future(row, post, m=a.m, d=a.d, KD=a.D, KS=a.S, dS=a.s, device=dev) as f:
                local_counts = f.simulate(r1 - r0, a.a, seed=seed, rep0=r0)
        out(f"end likelihood computation process {rank + 1}/{world}\n", all_ranks=True)
        if not root:
            out(f"Sending data (proc {rank})... ", all_ranks=True)
        else:
            out(f"Gathering data from {world - 1} proc... ")
        t = torch.from_numpy(local_counts.astype(np.int64)).to(tdev)
        counts = mdist.reduce_counts(t, rank, world)
        if not root:
            out("done\n", all_ranks=True)
        else:
            out("done\n" * (world - 1))  # one per received rank (:445)
        dist.destroy_process_group()
        if not root:
            return 0
    out(f"Writing on file {a.o}... ")
    with open(a.o, "w") as fe:
        fe.write("".join(f"{int(v)}\t" for v in counts))
    out("done\n")
    out(f"Finished. It took  {(int(time.time()) - start) / 60.0:.2f} min\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
