"""Host-side pieces of `python -m midaspom_amd` (no GPU): the problem dump
and the finishing step, including the MPI build's raw branch when Ltot == 0
(main_MIDASPOM_MPI.c:527)."""
from __future__ import annotations

import io

import numpy as np

import midaspom_amd as mdp
from midaspom_amd import cli


def test_ltot_zero_raw_branch(tmp_path):
    # s = 2 on [0, 1]: win = 1 and trapezoid weights 1/4 each, so loglik = 0
    # everywhere gives Ltot = 2 log 1 + log(4 * 1/4) = 0 exactly
    lik = np.zeros((2, 2))
    g, win = mdp.grid(2, 0.0, 1.0)
    assert win == 1.0
    buf = io.StringIO()
    ltot = cli.finish(lik, win, tmp_path / "mpi.txt", True, lambda t, all_ranks=False: buf.write(t))
    assert ltot == 0.0
    assert buf.getvalue().startswith("Total log-likelihood=0.00000\n")
    assert (tmp_path / "mpi.txt").read_text() == "0.00000000000000000000\t" * 2 + "\n" + \
        "0.00000000000000000000\t" * 2 + "\n"
    # single process (MIDASPOM.out has no raw branch): exp(0 - 0) = 1
    cli.finish(lik + 0.0, win, tmp_path / "one.txt", False, lambda t, all_ranks=False: None)
    assert (tmp_path / "one.txt").read_text() == ("1.00000000000000000000\t" * 2 + "\n") * 2


def test_problem_dump_mpi_nextid_position():
    obs = np.array([[1, 0, -1, 1], [1, 1, 0, 1], [0, 1, -1, 1]])
    model = mdp.Model.from_obs(obs)
    lines = []
    cli._print_problem(model, lambda t, all_ranks=False: lines.append((t, all_ranks)), mpi=True)
    text = "".join(t for t, _ in lines)
    assert text.index("Dispersal matrix:") < text.index(f"nextid={model.nextid}\n") < \
        text.index("Input occupancy data:")
    assert [a for t, a in lines if t.startswith("nextid=")] == [True]
    lines.clear()
    cli._print_problem(model, lambda t, all_ranks=False: lines.append((t, all_ranks)), mpi=False)
    assert not any(t.startswith("nextid=") for t, _ in lines)


def test_future_completions_and_priors():
    """`python -m midaspom_amd.future` prints the last survey's completions
    the way the drop-in does (future.c:286-332): the first missing patch is
    the most significant bit, pr is float arithmetic times a double."""
    from midaspom_amd import future

    np_, comps = future._completions(np.array([1, -1, 0, -1]), 0.3)
    assert np_ == 4
    assert [v for v, _ in comps] == [[1, 0, 0, 0], [1, 0, 0, 1], [1, 1, 0, 0], [1, 1, 0, 1]]
    f07 = float(np.float32(0.7))  # (float)(1 - bit) * (1 - prioroc) with prioroc = 0.3f
    f03 = float(np.float32(0.3))
    assert [p for _, p in comps] == [f07 * f07, f07 * f03, f03 * f07, f03 * f03]
    assert future._completions(np.array([0, 1]), 0.5) == (1, [([0, 1], 1.0)])


def test_future_args_defaults():
    """The code defaults of main_MIDASPOM_future.c:123-133 (-D 1, not the
    manual's 0)."""
    from midaspom_amd import future

    a = future.parse_args([])
    assert (a.n, a.a, a.m, a.p, a.d, a.S, a.s, a.D) == (10000, 50, 400.0, 0.5, 200.0, 0.0, 200.0, 1.0)
    assert (a.q, a.i, a.o) == ("posterior.txt", "input.txt", "pext_future.txt")
