"""Downstream format checks: the files the engine
writes load and summarise as the reference's R scripts expect
(midaspom_amd/rpost.py restates their numerics).  CPU tests use the host
writer (mdp_write_posterior, no GPU) on oracle log-likelihoods and the
manual's tables; the GPU tests use the drop-in CLIs' own output files."""
from __future__ import annotations

import subprocess

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle
from midaspom_amd import _lib, rpost


def test_r_seq_matches_reference_grid():
    g, _ = mdp.grid(101)
    assert np.allclose(rpost.r_seq(0.0, 1.0, 101), g, rtol=0, atol=1e-15)


def test_which_max_is_column_major_first():
    a = np.array([[1.0, 5.0], [5.0, 0.0]])  # ties: (1,0) comes first column-major
    assert rpost._which_max_colmajor(a) == 2


def test_default_example_point_estimates(golden, tmp_path):
    """plot_posterior.R on the default example (s = 101): the mode is the
    SURVEY §8(c) anchor (e 0.71, c 0.52); the marginals (row / column
    means of a density scaled by 1/0.01^2) sum to 10^4/s."""
    g, win = mdp.grid(101)
    lik = oracle.OracleModel.load(golden / "occupancies.txt", 400, 0.5, 100).loglik_grid(g, g)
    ltot = mdp.log_total(lik, win)
    out = tmp_path / "posterior.txt"
    mdp.write_posterior(out, lik, ltot)
    s = rpost.posterior_summary(out, 0.0, 1.0, 101)
    assert s["jpost"].shape == (101, 101)
    assert s["eest"] == pytest.approx(0.71) and s["cest"] == pytest.approx(0.52)
    assert s["epost"].sum() == pytest.approx(1e4 / 101) and s["cpost"].sum() == pytest.approx(1e4 / 101)
    assert s["qel"].size > 0 and s["qcl"].size > 0
    assert np.all(np.diff(s["qel"]) == 1) and np.all(np.diff(s["qcl"]) == 1)  # one interval each


def test_manual_posterior_table(golden):
    s = rpost.posterior_summary(golden / "manual_p3_posterior.txt", 0.0, 1.0, 5)
    assert s["jpost"].shape == (5, 5)
    assert (s["eest"], s["cest"]) == (0.5, 0.5)  # the table's maximum, 2.757263


def _write_tab_line(path, values):
    path.write_text("".join(f"{v:.20f}\t" for v in values))


def _write_tab_rows(path, rows):
    path.write_text("".join("".join(f"{v:.20f}\t" for v in r) + "\n" for r in rows))


def test_hypothesis_test_on_manual_tables(anchors, tmp_path):
    """hypothesis_test.R on the manual's p.4 die-off and p.5 loss tables, in
    the drop-ins' output layouts (one tab-separated line; one row per K)."""
    d = tmp_path / "dieoff.txt"
    lo = tmp_path / "loss.txt"
    _write_tab_line(d, anchors["manual_dieoff_p4"]["values_6dp"])
    _write_tab_rows(lo, anchors["manual_loss_p5"]["values_6dp"])
    h = rpost.hypothesis_test(d, lo, n=5, kmin=0.1, kmax=100.0)
    # K = 1 is not on the 11-point log grid of [0.1, 100]: the null
    # likelihood interpolates between its neighbours (:33-35)
    kd = 10.0 ** rpost.r_seq(-1.0, 2.0, 11)
    i = int(np.flatnonzero(kd > 1.0)[0])
    v = anchors["manual_dieoff_p4"]["values_6dp"]
    assert h["postnull"] == pytest.approx((v[i] - v[i - 1]) / (kd[i] - kd[i - 1]) * (1 - kd[i - 1]) + v[i - 1])
    for k in ("AIC0", "AIC1", "AIC2", "lK01", "lK02", "lK12"):
        assert np.isfinite(h[k]), k
    ds = rpost.dieoff_summary(d, 0.1, 100.0, 11)
    assert 0.1 <= ds["Kdest"] <= 100.0
    ls = rpost.loss_summary(lo, 0.1, 100.0, 200.0, 4000.0, 11, 4)
    assert ls["jpostloss"].shape == (11, 4) and np.isfinite(ls["dlest"]) and np.isfinite(ls["Klest"])


def test_ragged_table_rejected(tmp_path):
    p = tmp_path / "bad.txt"
    p.write_text("1\t2\t\n3\t\n")
    with pytest.raises(ValueError, match="ragged"):
        rpost.read_table(p)


@pytest.mark.gpu
def test_cli_outputs_feed_the_r_pipeline(golden, tmp_path):
    """The drop-in CLIs' files (GPU engine) through the R scripts' numerics."""
    post = tmp_path / "posterior.txt"
    r = subprocess.run([str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-i", str(golden / "occupancies.txt"),
                        "-o", str(post)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    s = rpost.posterior_summary(post, 0.0, 1.0, 101)
    assert (s["eest"], s["cest"]) == (pytest.approx(0.71), pytest.approx(0.52))
    d, lo = tmp_path / "dieoff.txt", tmp_path / "loss.txt"
    common = ["-a", "10", "-e", "0.5", "-c", "0.5", "-m", "400", "-d", "200", "-s", "11",
              "-i", str(golden / "manual_p3_obs.txt")]
    for exe, out, extra in ((_lib.DIEOFF_CLI_PATH, d, []), (_lib.LOSS_CLI_PATH, lo, ["-v", "4"])):
        r = subprocess.run([str(exe)] + common + extra + ["-o", str(out)], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr
    h = rpost.hypothesis_test(d, lo, n=5, kmin=0.1, kmax=100.0)
    for k in ("AIC0", "AIC1", "AIC2", "lK01", "lK02", "lK12"):
        assert np.isfinite(h[k]), k
