"""`python -m midaspom_amd` -- the MIDASPOM command line over the GPU engine.

Single process: the same flags, defaults, stdout lines and posterior file as
bin_linux/MIDASPOM.out (sources/main_MIDASPOM.c:61-439); the compiled drop-in
is midaspom_amd/_build/midaspom.

Under torchrun (WORLD_SIZE > 1, one process per GPU): the drop-in for
`mpirun -np N MIDASPOM_MPI.out` -- e-row slabs per rank and one gather to
rank 0 over RCCL (sources/main_MIDASPOM_MPI.c:361-368, 482-506), including
that program's extra stdout lines (nextid per rank :301, per-process start /
end lines :356, :479, send / gather lines :489-507) and its raw-loglik output
when Ltot == 0 (:527).
"""
from __future__ import annotations

import argparse
import os
import sys
import time


def parse_args(argv):
    # getopt "m:p:d:i:o:s:l:u:" (:79); code defaults (:66-73), not the manual's
    ap = argparse.ArgumentParser(prog="midaspom", add_help=True)
    ap.add_argument("-m", type=float, default=400.0, help="mean dispersal distance")
    ap.add_argument("-p", type=float, default=0.5, help="prior occupancy of missing year-0 patches")
    ap.add_argument("-d", type=float, default=100.0, help="segment length")
    ap.add_argument("-i", default="input.txt", help="occupancy file")
    ap.add_argument("-o", default="posterior.txt", help="posterior output file")
    ap.add_argument("-s", type=int, default=101, help="grid steps")
    ap.add_argument("-l", type=float, default=0.0, help="lower bound")
    ap.add_argument("-u", type=float, default=1.0, help="upper bound")
    ap.add_argument("-g", type=int, default=None,
                    help="GPUs of this process (single process; default MIDASPOM_GPUS or the current device), "
                         "as the compiled midaspom's -g")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default nccl)")
    return ap.parse_args(argv)


def _print_problem(model, out, mpi=False):
    pb = model
    out(f"Number of habitat patches: {pb.n}\nNumber of sampled years: {pb.tmax}\n")
    out("Dispersal matrix:\n")
    M = pb.M
    for i in range(pb.n):
        out("".join(f"{M[i, j]:.3f} " for j in range(pb.n)) + "\n")
    if mpi:  # every rank, right after its state enumeration (main_MIDASPOM_MPI.c:301)
        out(f"nextid={pb.nextid}\n", all_ranks=True)
    out("Input occupancy data:\n")
    obs = pb.obs
    for t in range(pb.tmax):
        out(f"Year {t}: " + "".join(f"{v} " for v in obs[t]) + "\n")
    out("Number of possible states per year:\n")
    for t, k in enumerate(pb.npstates):
        out(f"Year {t}: {k}\n")
    out(f"Number of states to compute: {pb.nstates}\n")


def main(argv=None) -> int:
    import numpy as np

    import midaspom_amd as mdp
    from midaspom_amd import dist as mdist

    a = parse_args(sys.argv[1:] if argv is None else argv)
    rank, world, local = mdist.env_rank_world()
    mpi = world > 1 or mdist.under_launcher()
    root = rank == 0

    def out(text, all_ranks=False):
        if root or all_ranks:
            sys.stdout.write(text)
            sys.stdout.flush()

    if mpi:  # unguarded in the MPI build: every rank prints it (:78)
        out("------ MIDASPOM, beta MPI version ------\n-> N. Alcala, E. M. Cole, and N. A. Rosenberg <-\n",
            all_ranks=True)
    else:
        out("------ MIDASPOM, beta version ------\n-> N. Alcala, E. M. Cole, and N. A. Rosenberg <-\n")
    if a.s < 1:  # the reference indexes g[s - 1] (main_MIDASPOM.c:319): s = 0 is out of bounds there
        sys.stderr.write("midaspom: -s must be at least 1\n")
        return 1
    g, win = mdp.grid(a.s, a.l, a.u)
    out(f"Parameters for numerical approximation of the posterior density:\n\tWindow size={win:f}, "
        f"number of steps={a.s}\n")
    out(f"Reading observations from file {a.i}... ")
    try:
        model = mdp.Model.load(a.i, m=a.m, p=a.p, d=a.d)
    except mdp.MidaspomError as exc:
        sys.stderr.write(f"\nmidaspom: {exc}\n")
        return 2
    out("done\n")
    _print_problem(model, out, mpi=mpi)
    start = time.time()

    if not mpi:
        out("Starting parallel likelihood computation\n")
        ngpu = a.g if a.g is not None else int(os.environ.get("MIDASPOM_GPUS", "0"))
        with mdp.Engine(model, n_devices=max(0, ngpu)) as eng:  # 0: the current device
            lik = eng.loglik_grid(g, g, layout="ce")  # [c][e] slabs, read in place
        for ie in range(a.s):  # ((float)ie+1)*100.0/nstep, exact in double (:394)
            out(f"{(ie + 1) * 100.0 / a.s:.2f}% done\n")
        out("end likelihood computation\n")
    else:
        import torch
        import torch.distributed as dist

        backend = a.backend or "nccl"
        # one process per GPU; a rehearsal backend may run more ranks than
        # GPUs (ranks then share devices round-robin)
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        compute = mdist.gpu_slab_compute(model, dev)
        out(f"Starting parallel likelihood computation process {rank + 1}/{world}\n", all_ranks=True)
        # this rank's c columns for every e (dist.py: the per-c tables split
        # with the grid; built for the whole grid's |c| bound, so the same
        # bits as one rank); the progress lines keep the reference's e-row
        # slabs (main_MIDASPOM_MPI.c:361-368, :463)
        c0, c1 = mdist.row_slab(rank, world, a.s)
        local_lik = compute(g, g[c0:c1], cbound=float(abs(g).max()))
        r0, r1 = mdist.row_slab(rank, world, a.s)
        for ie in range(r0, r1):  # main_MIDASPOM_MPI.c:463
            out(f"{(ie + 1 - r0) * 100.0 / (r1 - r0):.2f}% done\n")
        out(f"end likelihood computation process {rank + 1}/{world}\n", all_ranks=True)
        if not root:
            out(f"Sending data (proc {rank})... ", all_ranks=True)
        else:
            out(f"Gathering data from {world - 1} proc... ")
        lik = mdist.gather_colslabs(local_lik, rank, world, a.s, a.s,
                                    device=None if backend == "nccl" else "cpu")
        out("done\n", all_ranks=True)
        compute.engine.close()
        dist.destroy_process_group()
        if not root:
            return 0

    finish(lik, win, a.o, mpi, out)
    elapsed = int(time.time()) - int(start)
    out(f"done\n Total running time: {elapsed / 60.0:.2f} min\n")
    return 0


def finish(lik, win, path, mpi, out):
    """Normalise and write (main_MIDASPOM.c:413-436); the MPI build writes
    raw log-likelihoods instead when Ltot == 0 (main_MIDASPOM_MPI.c:527)."""
    import midaspom_amd as mdp

    ltot = mdp.log_total(lik, win)
    out(f"Total log-likelihood={ltot:.5f}\n")
    out(f"Writing output in file {path}... ")
    mdp.write_posterior(path, lik, ltot, raw=bool(mpi) and ltot == 0)
    return ltot


if __name__ == "__main__":
    sys.exit(main())
