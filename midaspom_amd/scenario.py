"""`python -m midaspom_amd.scenario {dieoff|loss} ...` -- the scenario
programs over the GPU scenario engine.

Single process: the same flags, code defaults, stdout lines and output file
as the compiled drop-ins `midaspom_dieoff` / `midaspom_loss`
(midaspom_amd/csrc/midaspom_scenario_cli.c; reference
sources/main_MIDASPOM_dieoff.c:94-384, main_MIDASPOM_loss.c:115-421).

Under torchrun (WORLD_SIZE > 1, one process per GPU): the drop-in for
`mpirun -np N MIDASPOM_dieoff_MPI.out` / `MIDASPOM_loss_MPI.out` -- the K grid
split into contiguous row slabs (remainder to rank 0,
main_MIDASPOM_dieoff_MPI.c:323-330, main_MIDASPOM_loss_MPI.c:366-371), one
gather to rank 0, and that program's per-rank stdout lines (banner :108,
start / end :320, :397, send / gather :401-418).  Rank 0 writes the file.
"""
from __future__ import annotations

import argparse
import sys
import time

import numpy as np

BANNER = {
    ("dieoff", False): "------ MIDASPOM, in situ die-off hypothesis, beta version -------\n"
                       "-> N. Alcala, E. M. Cole, N. A. Rosenberg <-\n",
    ("dieoff", True): "------ MIDASPOM, in situ die-off hypothesis, beta MPI version -------\n"
                      "-> N. Alcala, E. M. Cole, N. A. Rosenberg <-\n",
    ("loss", False): "------ MIDASPOM, habitat loss hypothesis, beta version -------\n"
                     "-> N. Alcala, E. M. Cole, N. A. Rosenberg  <-\n",
    ("loss", True): "------ MIDASPOM, habitat loss hypothesis, beta MPI version -------\n"
                    "-> N. Alcala, E. M. Cole, N. A. Rosenberg  <-\n",
}


def parse_args(kind, argv):
    # getopt "b:a:e:c:m:p:d:i:o:s:l:u:" (dieoff) / "...s:v:l:u:L:U:" (loss);
    # code defaults (dieoff.c:96-105, loss.c:117-126); -a -e -c required (Q11)
    ap = argparse.ArgumentParser(prog=f"midaspom_{kind}")
    ap.add_argument("-b", type=int, default=20, help="years before the event")
    ap.add_argument("-a", type=int, required=True, help="years after the event")
    ap.add_argument("-e", type=float, required=True, help="extinction rate")
    ap.add_argument("-c", type=float, required=True, help="colonisation rate")
    ap.add_argument("-m", type=float, default=400.0, help="mean dispersal distance")
    ap.add_argument("-p", type=float, default=0.5, help="prior occupancy of missing patches")
    ap.add_argument("-d", type=float, default=200.0, help="segment length")
    ap.add_argument("-i", default="input.txt", help="occupancy file (first row used)")
    ap.add_argument("-o", default="lh_dieoff.txt" if kind == "dieoff" else "lh_loss.txt")
    ap.add_argument("-s", type=int, default=151, help="K grid steps")
    ap.add_argument("-l", type=float, default=0.1, help="K lower bound")
    ap.add_argument("-u", type=float, default=100.0, help="K upper bound")
    if kind == "loss":
        ap.add_argument("-v", type=int, default=20, help="source-distance grid steps")
        ap.add_argument("-L", type=float, default=200.0, help="source distance lower bound")
        ap.add_argument("-U", type=float, default=4000.0, help="source distance upper bound")
    ap.add_argument("-g", type=int, default=None,
                    help="GPUs (single process): K slabs, one thread per slab (default MIDASPOM_GPUS or 1)")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default nccl)")
    return ap.parse_args(argv)


def _states(row, p):
    """Observed first-row states and their float32 priors (dieoff.c:205-232)."""
    n = row.size
    miss = [j for j in range(n) if row[j] == -1]
    np_ = 1 << len(miss)
    ps = np.zeros(np_, dtype=np.int64)
    pr = np.ones(np_, dtype=np.float32)
    s1 = 0
    for j in range(n):
        if row[j] == -1:
            s1 += 1
        for k in range(np_):
            if row[j] > -1:
                ps[k] += int(row[j]) << (n - j - 1)
            else:
                b = k // (np_ >> s1) % 2
                ps[k] += b << (n - j - 1)
                pr[k] = np.float32(pr[k] * np.float32(np.float32(b) * np.float32(p) +
                                                       np.float32(1 - b) * np.float32(1 - np.float32(p))))
    return ps, pr


def _lik_slabs(mdp, mdist, row, kind, a, K, dv, nd):
    """Single-process -g N: the K grid in N contiguous slabs (the MPI
    partition), one thread and scenario engine per slab, the slabs dealt
    round-robin over the visible GPUs (midaspom_scenario_cli.c run_slab).
    The engine calls release the GIL (ctypes), so the slabs run together."""
    import os
    import threading

    ngpu = a.g if a.g is not None else int(os.environ.get("MIDASPOM_GPUS", "1"))
    ngpu = max(1, min(ngpu, a.s)) if a.s else 1
    ndev = max(1, mdp.device_count())
    lik = np.zeros((a.s, nd))
    errs = []

    def run(r):
        r0, r1 = mdist.row_slab(r, ngpu, a.s)
        try:
            if r1 > r0:
                with mdp.Scenario(row, kind, m=a.m, p=a.p, d=a.d, device=r % ndev) as sc:
                    lik[r0:r1] = sc.lik(a.e, a.c, K[r0:r1], dv if kind == "loss" else None,
                                        ts=a.b, tdis=a.a)[0, 0].reshape(r1 - r0, nd)
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
    return lik


def main(argv=None) -> int:
    import midaspom_amd as mdp
    from midaspom_amd import dist as mdist

    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in ("dieoff", "loss"):
        sys.stderr.write("usage: python -m midaspom_amd.scenario {dieoff|loss} [flags]\n")
        return 1
    kind = argv[0]
    rank, world, local = mdist.env_rank_world()
    root = rank == 0
    mpi = world > 1 or mdist.under_launcher()

    def out(text, all_ranks=False):
        if root or all_ranks:
            sys.stdout.write(text)
            sys.stdout.flush()

    out(BANNER[(kind, mpi)], all_ranks=True)  # unguarded in the MPI builds (:108)
    try:
        a = parse_args(kind, argv[1:])
    except SystemExit:
        sys.stderr.write("Options -a (years after the event), -e and -c are required.\n")
        return 1
    if kind == "dieoff":
        out(f"{a.b} years before increased die-off, {a.a} years after increased die-off\n")
    else:
        out(f"{a.b} years before habitat loss, {a.a} years after the loss\n")
    out(f"Reading observations from file {a.i}... ")
    try:
        row = mdp.first_row(a.i)
    except OSError:
        sys.stderr.write(f"cannot open {a.i}\n")
        return 1
    n = row.size
    if kind == "loss":
        out(f"{n} patches\nReading observations from file {a.i}... ")
    out("done\n")
    if kind == "dieoff":
        out(f"{n} patches\n")
    out("Migration matrix:\n")
    for i in range(n):
        out("".join(f"{0.0 if i == j else np.exp(-(1.0 / a.m) * abs(i - j) * a.d):.3f} " for j in range(n)) + "\n")
    ps, pr = _states(row, a.p)
    if kind == "loss":
        out("First occupancy survey:\n")
    for k in range(ps.size):
        bits = "".join(f"{(int(ps[k]) >> (n - 1 - j)) & 1} " for j in range(n))
        out(("\t" if kind == "loss" else "") + bits + f"; pr={float(pr[k]):.6f}\n")
    K = mdp.kgrid(a.s, a.l, a.u)
    dv = mdp.dgrid(a.v, a.L, a.U) if kind == "loss" else np.zeros(1)
    nd = dv.size
    start = int(time.time())
    if not mpi:
        out("Starting likelihood computation\n")
        lik = _lik_slabs(mdp, mdist, row, kind, a, K, dv, nd)
        out("end likelihood computation\n")
    else:
        import torch
        import torch.distributed as dist

        backend = a.backend or "nccl"
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        out(f"Starting parallel likelihood computation process {rank + 1}/{world}\n", all_ranks=True)
        r0, r1 = mdist.row_slab(rank, world, a.s)
        local_lik = np.zeros((r1 - r0, nd))
        if r1 > r0:
            with mdp.Scenario(row, kind, m=a.m, p=a.p, d=a.d, device=dev) as sc:
                local_lik = sc.lik(a.e, a.c, K[r0:r1], dv if kind == "loss" else None,
                                   ts=a.b, tdis=a.a)[0, 0].reshape(r1 - r0, nd)
        out(f"end likelihood computation process {rank + 1}/{world}\n", all_ranks=True)
        if not root:
            out(f"Sending data (proc {rank})... ", all_ranks=True)
        else:
            out(f"Gathering data from {world - 1} proc... ")
        t = torch.from_numpy(np.ascontiguousarray(local_lik))
        lik = mdist.gather_rows(t.to(f"cuda:{dev}") if backend == "nccl" else t, rank, world, a.s, nd,
                                device=None if backend == "nccl" else "cpu")
        out("done\n", all_ranks=True)
        dist.destroy_process_group()
        if not root:
            return 0
    out(f"Writing on file {a.o}... ")
    lik = np.asarray(lik).reshape(a.s, nd)
    with open(a.o, "w") as fe:
        for i in range(a.s):
            fe.write("".join(f"{v:.20f}\t" for v in lik[i]))
            if kind == "loss":
                fe.write("\n")
    out("done\n")
    out(f"Finished. It took  {(int(time.time()) - start) / 60.0:.2f} min\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
