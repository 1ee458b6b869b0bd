"""GPU parity of the forward-simulation engine (mdp_future_*, the replicate
loop of main_MIDASPOM_future.c:343-386) against the CPU oracle driven by the
same addressed Philox stream: per-year all-extinct counts must agree EXACTLY
(integer work), including the carry-over of (e, c) when a posterior draw
falls past the last cell, missing-data initial states, source / K_D
scenarios, NaN posteriors, 8..64 patches and any replicate split."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle
from midaspom_amd import _lib

pytestmark = pytest.mark.gpu


def _post(golden, tmp_path, name, s=101, d=100):
    out = tmp_path / f"post_{s}_{d}.txt"
    oracle.run(golden / name, out, m=400, d=d, s=s)
    return oracle.read_posterior(out)


def _both(row, post, nrep, tfut, seed=0, rep0=0, **kw):
    with mdp.Future(row, post, **kw) as f:
        got = f.simulate(nrep, tfut, seed=seed, rep0=rep0)
    ref = oracle.future_counts(row, post, tfut=tfut, nrep=nrep, seed=seed, rep0=rep0, **kw)
    return got, ref


def test_manual_p6_example(golden):
    _, _, row = mdp.read_survey(golden / "manual_p3_obs.txt")
    post = np.loadtxt(golden / "manual_p3_posterior.txt")
    got, ref = _both(row, post, 20000, 10, seed=123, m=400, d=100, KS=1, dS=200)
    assert np.array_equal(got, ref), (got, ref)
    assert got[-1] > 0


def test_examples_input_default_flags(golden, tmp_path):
    """examples/input (n = 8 after the Q6 re-flow), its s = 101 posterior."""
    _, _, row = mdp.read_survey(golden / "occupancies.txt")
    post = _post(golden, tmp_path, "occupancies.txt")
    got, ref = _both(row, post, 30000, 50, seed=2024, m=400, d=100)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("KD,KS,dS", [(1.0, 0.0, 200.0), (0.3, 2.0, 50.0), (4.0, 0.7, 1000.0), (0.0, 1.0, 200.0)])
def test_scenarios_missing_data(golden, tmp_path, KD, KS, dS):
    row = np.array([1, -1, 0, 1, -1, -1, 0, 1, 0, -1, 1], dtype=np.int32)
    post = _post(golden, tmp_path, "manual_p3_obs.txt", s=41, d=200)
    got, ref = _both(row, post, 7000, 23, seed=99, m=300, d=150, KD=KD, KS=KS, dS=dS)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("n", [1, 2, 9, 16, 17, 33, 64])
def test_patch_counts(golden, tmp_path, n):
    rng = np.random.default_rng(n)
    row = rng.choice(np.array([-1, 0, 1], dtype=np.int32), size=n, p=[0.1, 0.4, 0.5]).astype(np.int32)
    if (row == -1).sum() > 12:
        row[row == -1] = 1
    post = _post(golden, tmp_path, "manual_p3_obs.txt", s=21, d=200)
    got, ref = _both(row, post, 3000, 17, seed=5 + n, m=400, d=100, KS=0.2)
    assert np.array_equal(got, ref)


def test_carry_over_and_split(golden, tmp_path):
    """Half the posterior mass: ~half the draws miss and keep the previous
    replicate's (e, c); any split of [0, N) gives the same totals."""
    _, _, row = mdp.read_survey(golden / "occupancies.txt")
    post = _post(golden, tmp_path, "occupancies.txt", s=21) * 0.5
    N, tfut = 9000, 30
    ref = oracle.future_counts(row, post, tfut=tfut, nrep=N, seed=77, m=400, d=100)
    with mdp.Future(row, post, m=400, d=100) as f:
        whole = f.simulate(N, tfut, seed=77)
        parts = sum(f.simulate(b - a, tfut, seed=77, rep0=a) for a, b in [(0, 1), (1, 4000), (4000, 8999), (8999, 9000)])
    assert np.array_equal(whole, ref) and np.array_equal(parts, ref)


def test_nan_and_degenerate_posteriors(golden, tmp_path):
    _, _, row = mdp.read_survey(golden / "manual_p3_obs.txt")
    post = _post(golden, tmp_path, "manual_p3_obs.txt", s=11, d=200)
    p1 = post.copy()
    p1[4, 7:] = np.nan  # the scan stops matching at the first NaN
    p0 = np.zeros_like(post)  # never found: (e, c) = (0, 0) for every replicate
    allnan = np.full((5, 5), np.nan)
    for p in (p1, p0, allnan, np.zeros((0, 0))):
        got, ref = _both(row, p, 4000, 12, seed=1, m=400, d=200, KS=0.5)
        assert np.array_equal(got, ref)


def test_device_variant_matches_host(golden, tmp_path):
    import torch
    _, _, row = mdp.read_survey(golden / "occupancies.txt")
    post = _post(golden, tmp_path, "occupancies.txt", s=21)
    with mdp.Future(row, post, m=400, d=100) as f:
        host = f.simulate(50000, 40, seed=3)
        out = torch.zeros(40, dtype=torch.int64, device="cuda:0")
        f.simulate_device(out.data_ptr(), 50000, 40, seed=3, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().astype(np.uint64), host)
        assert f.time_kernel(50000, 40, seed=3, reps=3) > 0


def test_lookback_overflow_flag_is_sticky(golden, tmp_path):
    """A posterior with almost no mass makes later replicates look back past
    the engine's limit: the device flag stays set across further launches
    until mdp_future_check reads it (and clears it); the host form reports
    its own launch."""
    import torch
    _, _, row = mdp.read_survey(golden / "occupancies.txt")
    post = _post(golden, tmp_path, "occupancies.txt", s=21)
    tiny = post * 1e-12
    st = torch.cuda.current_stream().cuda_stream
    out = torch.zeros(10, dtype=torch.int64, device="cuda:0")
    with mdp.Future(row, tiny, m=400, d=100) as bad, mdp.Future(row, post, m=400, d=100) as good:
        bad.simulate_device(out.data_ptr(), 200_000, 10, seed=1, stream=st)  # overflows
        bad.simulate_device(out.data_ptr(), 100, 10, seed=1, stream=st)      # does not
        with pytest.raises(_lib.MidaspomError):
            bad.check(st)
        bad.check(st)  # cleared by the previous check
        good.simulate_device(out.data_ptr(), 1000, 10, seed=1, stream=st)
        good.check(st)
        with pytest.raises(_lib.MidaspomError):
            bad.simulate(200_000, 10, seed=1)
        bad.check(st)  # the host form's overflow does not leak into the device flag


def test_large_ensemble_properties(golden, tmp_path):
    """Config-5 shape (10^6 replicates): counts are bounded, and the GPU total
    of a split run equals the whole run (size-independent properties)."""
    _, _, row = mdp.read_survey(golden / "occupancies.txt")
    post = _post(golden, tmp_path, "occupancies.txt")
    N, tfut = 1_000_000, 50
    with mdp.Future(row, post, m=400, d=100) as f:
        whole = f.simulate(N, tfut, seed=42)
        half = f.simulate(N // 2, tfut, seed=42) + f.simulate(N - N // 2, tfut, seed=42, rep0=N // 2)
    assert np.array_equal(whole, half)
    assert whole.max() <= N and whole[-1] > 0
    # the first 20k replicates of the same stream agree with the oracle exactly
    with mdp.Future(row, post, m=400, d=100) as f:
        got = f.simulate(20000, tfut, seed=42, rep0=123456)
    ref = oracle.future_counts(row, post, tfut=tfut, nrep=20000, seed=42, rep0=123456, m=400, d=100)
    assert np.array_equal(got, ref)


def test_future_cli_layout(golden, tmp_path):
    post = tmp_path / "posterior.txt"
    oracle.run(golden / "manual_p3_obs.txt", post, m=400, d=200, s=5)
    out = tmp_path / "pext.txt"
    r = subprocess.run([str(_lib.FUTURE_CLI_PATH), "-a", "10", "-m", "400", "-d", "100", "-i",
                        str(golden / "manual_p3_obs.txt"), "-q", str(post), "-o", str(out), "-S", "1", "-s", "200",
                        "-r", "123", "-n", "10000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "10 years in the future" in r.stdout and "5X5 posterior distribution" in r.stdout
    assert "npstates = 1" in r.stdout and "Starting likelihood computation" in r.stdout
    txt = out.read_text()
    assert txt.endswith("\t") and "\n" not in txt
    vals = [int(x) for x in txt.split("\t")[:-1]]
    _, _, row = mdp.read_survey(golden / "manual_p3_obs.txt")
    ref = oracle.future_counts(row, oracle.read_posterior(post), tfut=10, nrep=10000, seed=123, m=400, d=100,
                               KS=1, dS=200)
    assert vals == [int(x) for x in ref]


@pytest.mark.parametrize("seed", range(int(os.environ.get("MDP_FUZZ_FUT", "8"))))  # more: a longer fuzz
def test_random_futures(seed):
    """Random last surveys (1-64 patches, missing data), random posteriors
    (2-101 steps, sparse or flat, some exact zeros), rates K_D / K_S / d_S,
    horizons and replicate offsets: the GPU counts equal the oracle's under
    the same addressed Philox stream, count for count."""
    rng = np.random.default_rng(9000 + seed)
    n = int(rng.choice([1, 3, 8, 12, 20, 40, 64]))
    row = rng.choice([-1, 0, 1], size=n, p=[0.15, 0.45, 0.4]).astype(np.int32)
    if rng.random() < 0.3:
        row[rng.integers(0, n)] = 1  # never all empty at the start
    s = int(rng.choice([2, 5, 21, 101]))
    post = rng.random((s, s)) ** float(rng.choice([1.0, 8.0]))
    post[rng.random((s, s)) < 0.3] = 0.0
    kw = dict(m=float(rng.choice([100.0, 400.0])), d=float(rng.choice([50.0, 200.0])),
              KD=float(rng.choice([0.0, 0.5, 1.0, 3.0])), KS=float(rng.choice([0.0, 0.5, 2.0])),
              dS=float(rng.choice([50.0, 200.0, 1000.0])))
    nrep, tfut = int(rng.integers(1, 5000)), int(rng.integers(1, 60))
    got, ref = _both(row, post, nrep, tfut, seed=int(rng.integers(0, 2 ** 40)),
                     rep0=int(rng.integers(0, 10 ** 6)), **kw)
    assert np.array_equal(got, ref), (seed, got, ref)
