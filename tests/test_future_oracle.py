"""Forward simulation (main_MIDASPOM_future.c) on the CPU: the generator's
known answers, the input readers of the product against the oracle's, the
oracle's replicate-split invariance (the carry-over of (e, c) across
replicates, future.c:361-377), and the statistical agreement of the
addressed Philox stream with the reference's own glibc rand() stream.

The reference program is not buildable here (it links CBLAS), so the only
reference output is the manual's one stochastic run (p.6), checked for
consistency, not pinned."""
from __future__ import annotations

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle

# Random123 known-answer vectors for philox4x32_10 (kat_vectors)
KAT = [
    (0x0, [0, 0, 0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    (0xffffffffffffffff, [0xffffffff] * 4, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    (0x299f31d0a4093822, [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize("key,ctr,want", KAT)
def test_philox_known_answers(key, ctr, want):
    assert oracle.philox(key, ctr) == want
    assert mdp.philox(key, ctr) == want


def test_readers_match_oracle(golden, tmp_path):
    for f in ("manual_p3_obs.txt", "occupancies.txt", "config2_64x50.txt"):
        n, t, row = mdp.read_survey(golden / f)
        on, ot, orow = oracle.last_row(golden / f)
        assert (n, t) == (on, ot) and np.array_equal(row, orow)
    # occupancies.txt re-flows (Q6): the last row is the last n tokens
    n, t, row = mdp.read_survey(golden / "occupancies.txt")
    toks = (golden / "occupancies.txt").read_text().split()
    assert n == 8 and t == 7 and list(row) == [int(x) for x in toks[(t - 1) * n: t * n]]
    post = tmp_path / "post.txt"
    oracle.run(golden / "manual_p3_obs.txt", post, m=400, d=200, s=11)
    a, b = mdp.read_posterior(post), oracle.read_posterior(post)
    assert a.shape == (11, 11) and np.array_equal(a, b)
    nanp = tmp_path / "nan.txt"
    nanp.write_text("-nan\t1.5\t\n0.25\t-nan\t\n")
    a = mdp.read_posterior(nanp)
    assert a.shape == (2, 2) and np.isnan(a[0, 0]) and a[0, 1] == 1.5 and np.isnan(a[1, 1])


def test_short_posterior_is_an_error(tmp_path):
    p = tmp_path / "short.txt"
    p.write_text("0.1\t0.2\t0.3\t\n0.4\t")
    with pytest.raises(mdp.MidaspomError):
        mdp.read_posterior(p)


def _manual(golden):
    _, _, row = oracle.last_row(golden / "manual_p3_obs.txt")
    post = np.loadtxt(golden / "manual_p3_posterior.txt")
    return row, post


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_oracle_split_invariance(golden, tmp_path, threads):
    """Counts over [0, N) equal the sum over any split, whatever the thread
    count: the carry-in of (e, c) reproduces the sequential loop."""
    _, _, row = oracle.last_row(golden / "occupancies.txt")
    post = oracle.read_posterior(_posterior(golden, tmp_path, "occupancies.txt", s=21))
    post = post * 0.5  # half the mass: many draws fall past the last cell (carry-over path)
    kw = dict(tfut=12, m=400, d=100, KS=0.5, dS=300, seed=7)
    full = oracle.future_counts(row, post, nrep=3000, threads=1, **kw)
    a = oracle.future_counts(row, post, nrep=1234, threads=threads, **kw)
    b = oracle.future_counts(row, post, nrep=3000 - 1234, rep0=1234, threads=threads, **kw)
    assert np.array_equal(full, a + b)
    assert full.sum() > 0


def _posterior(golden, tmp_path, name, s=101, d=100):
    out = tmp_path / f"post_{name}_{s}_{d}.txt"
    if not out.exists():
        oracle.run(golden / name, out, m=400, d=d, s=s)
    return out


def test_philox_stream_matches_glibc_stream_statistically(golden, tmp_path):
    """Same model, two random streams: the per-year extinct fractions agree
    within 5 binomial sigma (the reference's stream is glibc rand())."""
    _, _, row = oracle.last_row(golden / "manual_p3_obs.txt")
    post = oracle.read_posterior(_posterior(golden, tmp_path, "manual_p3_obs.txt", s=101, d=200))
    N = 40000
    kw = dict(tfut=15, m=400, d=100, KS=1.0, dS=200)
    a = oracle.future_counts(row, post, nrep=N, mode=oracle.RNG_PHILOX, seed=11, **kw).astype(float)
    b = oracle.future_counts(row, post, nrep=N, mode=oracle.RNG_GLIBC, seed=11, **kw).astype(float)
    pa, pb = a / N, b / N
    pm = (pa + pb) / 2
    sig = np.sqrt(np.maximum(pm * (1 - pm), 1e-12) * 2 / N)
    assert np.all(np.abs(pa - pb) <= 5 * sig + 1e-12), (pa, pb)


def test_manual_p6_example_is_consistent(golden, anchors):
    """Manual p.6: `-a 10 -m 400 -d 100 -S 1 -s 200`, 10 000 simulations ->
    0 0 0 0 4 8 12 12 32 52.  With the p.3 posterior the restated model's
    expectation lies within 4 sigma of every published count."""
    a = anchors["manual_future_p6"]
    row, post = _manual(golden)
    N = 200000
    c = oracle.future_counts(row, post, tfut=10, nrep=N, m=400, d=100, KS=1, dS=200, seed=3)
    exp10k = c.astype(float) / N * 10000
    want = np.array(a["counts"], dtype=float)
    sig = np.sqrt(np.maximum(exp10k * (1 - exp10k / 10000), 1.0))
    assert np.all(np.abs(want - exp10k) <= 4 * sig), (want, exp10k)
    assert abs(want[-1] - exp10k[-1]) <= 2 * sig[-1]


def test_future_errors(golden):
    row = np.zeros(65, dtype=np.int32)
    # the engine validates before touching a device
    with pytest.raises(mdp.MidaspomError, match="EUNSUPPORTED"):
        mdp.Future(row, np.ones((3, 3)))
    with pytest.raises(mdp.MidaspomError, match="EINVAL"):
        mdp.Future(np.array([0, 2, 1], dtype=np.int32), np.ones((3, 3)))
    with pytest.raises(mdp.MidaspomError, match="EINVAL"):
        mdp.Future(np.array([0, 1, 1], dtype=np.int32), np.ones((3, 3)), KD=-1.0)
