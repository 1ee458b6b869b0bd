"""Synthetic SPOM occupancy series.

Reproduces the survey's generator byte-for-byte (md5-checked in
tests/test_synth.py): a linear habitat of ``n`` segments whose last ``nvar``
columns are the only ones ever occupied (the "rightmost block", which also
avoids the serial reference's quirk Q1), simulated with the extinction-then-
colonisation SPOM of sources/main_MIDASPOM.c, with missing data (-1) in the
variable block at rate ``pmiss``.
"""
from __future__ import annotations

import numpy as np

# The BASELINE.json workloads as concrete inputs.
CONFIG2 = dict(n=64, T=50, nvar=8, e=0.3, c=0.1, m=400, d=100, pmiss=0.05, seed=1)
CONFIG3 = dict(n=256, T=200, nvar=8, e=0.1, c=0.05, m=400, d=100, pmiss=0.03, seed=2)
# SURVEY.md §8(c) "Q1 reproducer": the config-2 generator with the variable
# block in the middle (columns 28-35), so always-zero columns lie right of the
# last variable column -- the input on which the serial reference mis-numbers
# its states (quirk Q1, main_MIDASPOM.c:244) and the MPI build reports
# Ltot -153.68039 at -s 17 (main_MIDASPOM_MPI.c:262).
Q1_MID = dict(CONFIG2, v0=28)
# A 200-year survey with about four possible states per year (20 % of the
# variable patches unvisited): 3 086 forward uses per grid point, past the
# 2 048 of one specialised kernel -- the engine runs it as chunks of years.
LONG200 = dict(CONFIG2, T=200, pmiss=0.2, seed=11)
MD5 = {
    "config2": "6bd6f4bf7e69d794078d9c5718cda157",
    "config3": "5cf6ad09063e720a952fcd4c32b47030",
}


def generate(n: int, T: int, nvar: int, e: float, c: float, m: float, d: float,
             pmiss: float, seed: int, v0: int | None = None) -> str:
    """Return the occupancy file text (space-separated ints, '\\n' per year).
    ``v0`` moves the variable block to columns [v0, v0 + nvar) (default: the
    rightmost block of Appendix C)."""
    rng = np.random.default_rng(seed)
    v0 = n - nvar if v0 is None else v0
    var = np.arange(v0, v0 + nvar)
    idx = np.arange(n)
    disp = np.exp(-np.abs(idx[:, None] - idx[None, :]) * d / m)
    np.fill_diagonal(disp, 0)
    outside = np.ones(n, dtype=bool)
    outside[var] = False
    x = np.zeros(n, dtype=np.int64)
    x[var] = rng.integers(0, 2, nvar)
    x[var[0]] = 1
    rows = []
    for _ in range(T):
        obs = x.copy()
        mask = rng.random(nvar) < pmiss
        block = obs[var]
        block[mask] = -1
        obs[var] = block
        rows.append(" ".join(str(int(v)) for v in obs) + "\n")
        while True:  # redraw until the state stays in the block and is non-empty
            surv = x * (rng.random(n) > e)
            pc = np.minimum(1, c * (disp.T @ surv))
            new = (surv | ((rng.random(n) < pc) & (surv == 0))).astype(np.int64)
            if new[outside].sum() == 0 and new.sum() > 0:
                break
        x = new
    return "".join(rows)


def write(path, **cfg) -> str:
    text = generate(**cfg)
    with open(path, "w") as f:
        f.write(text)
    return str(path)


def random_obs(rng: np.random.Generator, n: int, T: int, nvar: int, pmiss: float,
               max_missing: int | None = None, p1: float = 0.5) -> np.ndarray:
    """Unstructured random observation matrix for parity fuzzing: ``nvar``
    random columns may be occupied (1 w.p. p1) or missing (-1 w.p. pmiss);
    at most ``max_missing`` missing cells per year."""
    obs = np.zeros((T, n), dtype=np.int32)
    cols = np.sort(rng.choice(n, size=nvar, replace=False))
    for t in range(T):
        vals = (rng.random(nvar) < p1).astype(np.int32)
        miss = rng.random(nvar) < pmiss
        if max_missing is not None and miss.sum() > max_missing:
            keep = rng.choice(np.flatnonzero(miss), size=max_missing, replace=False)
            miss[:] = False
            miss[keep] = True
        vals[miss] = -1
        obs[t, cols] = vals
    # make every chosen column variable at least once
    for q, col in enumerate(cols):
        if not obs[:, col].any():
            obs[rng.integers(T), col] = 1
    return obs


def alternating_obs(rng: np.random.Generator, n: int, T: int, nvar: int, dense: int, sparse: int,
                    nmiss: int = 0) -> np.ndarray:
    """Observation matrix for surveys with many variable patches: years
    alternate between ``dense`` occupied patches (of the ``nvar`` variable
    columns) and at most ``sparse`` occupied ones, so states carry many
    occupied patches while consecutive years overlap in at most ``sparse``
    (the Q groups stay small).  ``nmiss`` unvisited patches (-1) go into
    the sparse years."""
    obs = np.zeros((T, n), dtype=np.int32)
    cols = np.sort(rng.choice(n, size=nvar, replace=False))
    for t in range(T):
        k = dense if t % 2 == 0 else int(rng.integers(1, sparse + 1))
        on = rng.choice(cols, size=k, replace=False)
        obs[t, on] = 1
        if t % 2 == 1 and nmiss:
            free = np.setdiff1d(cols, on)
            obs[t, rng.choice(free, size=min(nmiss, free.size), replace=False)] = -1
    for col in cols:  # every chosen column variable at least once
        if not obs[:, col].any():
            obs[0, col] = 1
    return obs
