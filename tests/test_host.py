"""Host side of the product (parser, state enumeration, grid, normalisation,
writer) against the oracle restatement of main_MIDASPOM.c:137-287, 312-319,
413-436.  CPU only: integer/byte work must be bit-exact."""
from __future__ import annotations

import math

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle
from midaspom_amd import synth


def _same_model(pm: mdp.Model, om: oracle.OracleModel):
    assert (pm.n, pm.tmax, pm.nvar, pm.nextid) == (om.n, om.tmax, om.nvar, om.nextid)
    assert np.array_equal(pm.npstates, om.npstates)
    for a, b in zip(pm.year_ids, om.year_ids):
        assert np.array_equal(a, b)
    assert np.array_equal(pm.short_state, om.short_state)
    assert np.array_equal(pm.prior, om.prior)  # float32 widened, bit-exact


@pytest.mark.parametrize("fname", ["occupancies.txt", "manual_p3_obs.txt", "config2_64x50.txt",
                                   "config3_256x200.txt", "q1_64x50_mid.txt"])
@pytest.mark.parametrize("p", [0.5, 0.3])
def test_model_matches_oracle_files(golden, fname, p):
    pm = mdp.Model.load(golden / fname, m=400, p=p, d=100)
    om = oracle.OracleModel.load(golden / fname, 400, p, 100)
    _same_model(pm, om)


def test_example_reflow_q6(golden):
    """The shipped example has 8 tokens on line 1 and 9 on the others: n is
    taken from line 1 and the 56 tokens re-flow into 7 x 8 (quirk Q6)."""
    pm = mdp.Model.load(golden / "occupancies.txt")
    assert (pm.n, pm.tmax) == (8, 7)
    tokens = [int(t) for t in (golden / "occupancies.txt").read_text().split()]
    assert np.array_equal(pm.obs.ravel(), tokens[:56])


@pytest.mark.parametrize("seed", range(12))
def test_model_matches_oracle_random(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(3, 40))
    nvar = int(rng.integers(1, min(n, 10) + 1))
    T = int(rng.integers(1, 30))
    obs = synth.random_obs(rng, n, T, nvar, pmiss=0.15, max_missing=4)
    p = float(rng.choice([0.5, 0.25, 0.8]))
    pm = mdp.Model.from_obs(obs, m=400, p=p, d=float(rng.choice([50, 100, 200])))
    om = oracle.OracleModel.from_obs(obs, 400, p, 100)
    _same_model(pm, om)


def test_dispersal_matrix_bits(golden):
    pm = mdp.Model.load(golden / "config2_64x50.txt", m=400, d=100)
    M = pm.M
    a = 1.0 / 400
    # libm exp of ((-a)*|i-j|)*d, the reference's expression (:183-184)
    expect = np.array([[0.0 if i == j else math.exp(-a * abs(j - i) * 100.0) for j in range(pm.n)]
                       for i in range(pm.n)])
    assert np.array_equal(M, expect)


@pytest.mark.parametrize("s,lo,hi", [(101, 0, 1), (50, 0, 1), (17, 0.1, 0.9), (2, 0, 1), (1024, 0, 1)])
def test_grid_bitexact(s, lo, hi):
    g, win = mdp.grid(s, lo, hi)
    go, wo = oracle.grid(s, lo, hi)
    assert win == wo
    assert np.array_equal(g, go)


def test_log_total_and_writer_bitexact(tmp_path):
    rng = np.random.default_rng(3)
    s = 37
    lik = rng.normal(-20, 5, (s, s))
    lik[3, 4] = -np.inf
    g, win = mdp.grid(s)
    lt = mdp.log_total(lik, win)
    assert lt == oracle.ltot(lik, win)
    mdp.write_posterior(tmp_path / "a.txt", lik, lt)
    oracle.write_posterior(tmp_path / "b.txt", lik, lt)
    assert (tmp_path / "a.txt").read_bytes() == (tmp_path / "b.txt").read_bytes()


@pytest.mark.parametrize("threads", ["1", "3", "16"])
def test_threaded_normaliser_and_writer_bitexact(tmp_path, monkeypatch, threads):
    """Grids past 64 Ki cells take the threaded exps and row formatting:
    Ltot and every byte of the file equal the oracle's sequential forms,
    including -inf / NaN cells, huge values (a long %.20lf) and odd sizes."""
    monkeypatch.setenv("OMP_NUM_THREADS", threads)
    rng = np.random.default_rng(5)
    s = 263
    lik = rng.normal(-30, 8, (s, s))
    lik[0, :7] = -np.inf
    g, win = mdp.grid(s)
    lt = mdp.log_total(lik, win)
    assert lt == oracle.ltot(lik, win)
    mdp.write_posterior(tmp_path / "a.txt", lik, lt)
    oracle.write_posterior(tmp_path / "b.txt", lik, lt)
    assert (tmp_path / "a.txt").read_bytes() == (tmp_path / "b.txt").read_bytes()
    # the raw branch prints log-likelihoods as they are: NaN, -inf, a 1e300
    # (a 321-character cell)
    lik[100, 3], lik[7, 9] = np.nan, 1e300
    mdp.write_posterior(tmp_path / "r.txt", lik, 0.0, raw=True)
    ref = "".join("".join(f"{v:.20f}\t" for v in row) + "\n" for row in lik)
    assert (tmp_path / "r.txt").read_text() == ref


def test_writer_all_nan(tmp_path):
    s = 4
    lik = np.full((s, s), -np.inf)
    g, win = mdp.grid(s)
    lt = mdp.log_total(lik, win)
    assert np.isneginf(lt)
    mdp.write_posterior(tmp_path / "a.txt", lik, lt)
    text = (tmp_path / "a.txt").read_text()
    assert text == ("-nan\t" * s + "\n") * s


def test_writer_raw_branch(tmp_path):
    lik = np.array([[0.5, -1.25], [2.0, 0.0]])
    mdp.write_posterior(tmp_path / "r.txt", lik, 0.0, raw=True)
    assert (tmp_path / "r.txt").read_text().split() == [f"{v:.20f}" for v in lik.ravel()]


def test_bad_inputs(tmp_path):
    with pytest.raises(mdp.MidaspomError, match="EIO"):
        mdp.Model.load(tmp_path / "missing.txt")
    bad = tmp_path / "bad.txt"
    bad.write_text("0 2 1\n1 0 1\n")
    with pytest.raises(mdp.MidaspomError, match="EINVAL"):
        mdp.Model.load(bad)
    empty = tmp_path / "empty.txt"
    empty.write_text("")
    with pytest.raises(mdp.MidaspomError):
        mdp.Model.load(empty)


def test_missing_last_newline_drops_row(tmp_path):
    f = tmp_path / "x.txt"
    f.write_text("0 1 1\n1 0 1\n1 1 1")
    pm = mdp.Model.load(f)
    assert (pm.n, pm.tmax) == (3, 2)


@pytest.mark.parametrize("threads", ["1", "3"])
def test_batched_writer_and_ce_view_bitexact(tmp_path, monkeypatch, threads):
    """The writer formats parts of ~256 KB of text in bounded batches (a few
    parts per thread, written in order): at s = 700 (14 rows a part, 50
    parts, several batches with 3 threads) the file is byte-identical to the
    oracle's sequential writer.  The [c][e] device layout is read in place
    through the transposed view (mdp_*_view with se = 1, sc = s): the same
    Ltot bits and the same bytes."""
    monkeypatch.setenv("OMP_NUM_THREADS", threads)
    rng = np.random.default_rng(11)
    s = 700
    lik = rng.normal(-30, 8, (s, s))
    lik[3, :5] = -np.inf
    g, win = mdp.grid(s)
    lt = mdp.log_total(lik, win)
    assert lt == oracle.ltot(lik, win)
    ce = np.ascontiguousarray(lik.T)  # what MDP_LAYOUT_CE leaves in device memory
    assert mdp.log_total(ce.T, win) == lt
    mdp.write_posterior(tmp_path / "a.txt", lik, lt)
    mdp.write_posterior(tmp_path / "c.txt", ce.T, lt)
    oracle.write_posterior(tmp_path / "b.txt", lik, lt)
    ref = (tmp_path / "b.txt").read_bytes()
    assert (tmp_path / "a.txt").read_bytes() == ref
    assert (tmp_path / "c.txt").read_bytes() == ref
