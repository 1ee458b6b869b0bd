"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle on the
same inputs.

Tolerances (written here, per BASELINE north_star / SURVEY.md §8(c)):
  * log-likelihood: |dlogL| <= LOGLIK_ATOL (1e-9, i.e. 1e-9 relative on L)
    where L is a normal double; where it is subnormal or 0 (log L < -708.4)
    on either side, it must be so on both (assert_loglik_close);
    the factorised GPU form reorders an all-positive sum, so ~1e-13 is typical;
  * posterior: relative 1e-6 where posterior > 1e-14, absolute 1e-20 below;
  * "-nan" cells must sit at identical positions; -inf (L = 0: impossible
    transitions, underflow) only where the other side is -inf or subnormal.
"""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle
from midaspom_amd import _lib, synth

pytestmark = pytest.mark.gpu

LOGLIK_ATOL = 1e-9
POST_RTOL = 1e-6


# L below DBL_MIN is subnormal (or rounds to 0): its spacing is fixed
# (2^-1074), so its relative precision falls with it, and two summation
# orders -- the reference's BLAS builds among them -- round it differently;
# where one order underflows part-way through the years the other can end
# tens or hundreds of subnormal units away, or at 0.  Such cells (log L <
# -708.4, about 300 orders of magnitude below the posterior's %.20lf print
# floor, so the output file does not see them) must be subnormal or -inf on
# both sides; every cell with a normal L is held to `atol`.
LOG_DBL_MIN = float(np.log(np.finfo(np.float64).tiny))  # -708.396...


def assert_loglik_close(got, ref, atol=LOGLIK_ATOL):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "nan positions differ"
    ok = ~np.isnan(ref)
    sub = ok & ((ref < LOG_DBL_MIN) | (got < LOG_DBL_MIN))
    if sub.any():
        assert (got[sub] < LOG_DBL_MIN + 1e-9).all() and (ref[sub] < LOG_DBL_MIN + 1e-9).all(), \
            "a normal likelihood faces a subnormal / zero one"
    fin = ok & ~sub
    assert np.isfinite(got[fin]).all() and np.isfinite(ref[fin]).all()
    if fin.any():
        err = np.abs(got[fin] - ref[fin]).max()
        assert err <= atol, f"max |dlogL| = {err:.3e}"


def assert_posterior_close(got, ref):
    got, ref = np.asarray(got), np.asarray(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    big = ok & (ref > 1e-14)
    if big.any():
        rel = np.abs(got[big] - ref[big]) / ref[big]
        assert rel.max() <= POST_RTOL, f"max rel dposterior = {rel.max():.3e}"
    small = ok & ~big
    if small.any():
        assert np.abs(got[small] - ref[small]).max() <= 1e-20
    assert np.array_equal(got == 0, ref == 0) or np.abs(got - ref)[ok].max() <= 1e-20


def gpu_grid(model, e, c=None, **kw):
    c = e if c is None else c
    with mdp.Engine(model, **kw) as eng:
        return eng.loglik_grid(e, c)


# ---------------------------------------------------------------------------
# the SURVEY §8(c) anchor runs, end to end through the Python host
# ---------------------------------------------------------------------------
CASES = [
    ("manual_p3_obs.txt", dict(m=400, d=200, s=5)),
    ("occupancies.txt", dict(m=400, d=100, s=50)),
    ("occupancies.txt", dict(m=400, d=100, s=101)),
    ("occupancies.txt", dict(m=250, d=100, s=33, p=0.2)),
    ("config2_64x50.txt", dict(m=400, d=100, s=17)),
    ("config2_64x50.txt", dict(m=400, d=100, s=33, p=0.3)),
    ("config2_64x50.txt", dict(m=400, d=100, s=21, lo=0.05, hi=0.95)),
    ("config3_256x200.txt", dict(m=400, d=100, s=9)),
    ("config3_256x200.txt", dict(m=400, d=100, s=17)),
    ("config3_256x200.txt", dict(m=400, d=100, s=5)),  # Q4: all underflow -> -nan
    ("q1_64x50_mid.txt", dict(m=400, d=100, s=17)),    # Q1: variable block mid-row
    ("q1_64x50_mid.txt", dict(m=400, d=100, s=64)),
]


@pytest.mark.parametrize("fname,f", CASES, ids=[f"{a}-{b}" for a, b in CASES])
def test_file_runs_match_oracle(golden, fname, f):
    kw = dict(m=f["m"], p=f.get("p", 0.5), d=f["d"])
    s, lo, hi = f["s"], f.get("lo", 0.0), f.get("hi", 1.0)
    g, win = mdp.grid(s, lo, hi)
    model = mdp.Model.load(golden / fname, **kw)
    got = gpu_grid(model, g)
    om = oracle.OracleModel.load(golden / fname, kw["m"], kw["p"], kw["d"])
    ref = om.loglik_grid(g, g)
    assert_loglik_close(got, ref)
    lt_got, lt_ref = mdp.log_total(got, win), oracle.ltot(ref, win)
    if np.isfinite(lt_ref):
        assert lt_got == pytest.approx(lt_ref, rel=1e-12)
        assert f"{lt_got:.5f}" == f"{lt_ref:.5f}"
    else:
        assert np.isneginf(lt_got)
    assert_posterior_close(mdp.posterior(got, lt_got), mdp.posterior(ref, lt_ref))


def test_anchor_ltot_values(golden, anchors):
    """Total log-likelihood lines equal the reference's."""
    from conftest import run_by_name
    for name in ["manual_p3", "default_example_s101", "config1_s50", "config2_s17",
                 "config2_s17_p03", "config3_s9", "config3_s17", "config3_s32", "q1_mid_block_s17"]:
        r = run_by_name(anchors, name)
        f = r["flags"]
        lik, lt = mdp.run_file(golden / r["input"], m=f["m"], p=f.get("p", 0.5), d=f["d"], s=f["s"])
        assert f"{lt:.5f}" == r["ltot"], name


def test_manual_posterior_table(golden, tmp_path):
    lik, lt = mdp.run_file(golden / "manual_p3_obs.txt", tmp_path / "p.txt", m=400, d=200, s=5)
    assert np.array_equal(np.round(np.loadtxt(tmp_path / "p.txt"), 6),
                          np.loadtxt(golden / "manual_p3_posterior.txt"))


def test_q5_impossible_transition(tmp_path):
    obs = np.array([[0, 1, 1, 1], [0, 0, 0, 0], [0, 1, 0, 1]])
    lik, lt = None, None
    model = mdp.Model.from_obs(obs)
    g, win = mdp.grid(3)
    lik = gpu_grid(model, g)
    assert np.isneginf(lik).all()
    mdp.write_posterior(tmp_path / "q5.txt", lik, mdp.log_total(lik, win))
    assert set((tmp_path / "q5.txt").read_text().split()) == {"-nan"}


# ---------------------------------------------------------------------------
# fuzzing: random problems covering every forward-kernel variant
# ---------------------------------------------------------------------------
@pytest.fixture(params=["direct", "direct-qrows", "direct-plain", "generic", "wide", "wide-chunked", "wide-plain", "wide-hs",
                        "wide-hs-chunked"])
def engine_path(request, monkeypatch):
    """Every engine path: the direct one (the hipRTC-specialised forward
    kernel; on these small grids it computes its column's Q itself), the same
    with Q rows from k_qrows (MDP_FUSED=0), the direct path with the
    transition cache and XCD ordering off (MDP_JIT_SLOTS=0, MDP_JIT_XCD=0), and
    the generic kernels (MDP_JIT=0), and the wide path that years with more
    than 16 states need (MDP_WIDE=1: its forward on the matrix cores,
    k_fwd_mmt; chunked: one c value per item launch; plain: k_fwd_wide; hs:
    k_fwd_hs through the hidden states, whole and one c value per launch)."""
    for k in ("MDP_JIT", "MDP_JIT_SLOTS", "MDP_JIT_XCD", "MDP_FUSED", "MDP_WIDE", "MDP_WIDE_CB", "MDP_WIDE_MMA"):
        monkeypatch.delenv(k, raising=False)
    if request.param.startswith("wide"):
        monkeypatch.setenv("MDP_WIDE", "1")
        if request.param == "wide-chunked":
            monkeypatch.setenv("MDP_WIDE_CB", "1")
        if request.param == "wide-plain":
            monkeypatch.setenv("MDP_WIDE_MMA", "0")
        if request.param.startswith("wide-hs"):
            monkeypatch.setenv("MDP_WIDE_MMA", "3")
        if request.param == "wide-hs-chunked":
            monkeypatch.setenv("MDP_WIDE_CB", "1")
    elif request.param == "generic":
        monkeypatch.setenv("MDP_JIT", "0")
    elif request.param == "direct-qrows":
        monkeypatch.setenv("MDP_FUSED", "0")
    elif request.param == "direct-plain":
        monkeypatch.setenv("MDP_JIT_SLOTS", "0")
        monkeypatch.setenv("MDP_JIT_XCD", "0")
    return request.param


@pytest.mark.parametrize("seed", range(int(os.environ.get("MDP_FUZZ_LARGE", "24"))))  # more: a longer fuzz
def test_random_problems_large_grids(seed, monkeypatch):
    """Random problems on grids the small fuzz never reaches: several e
    blocks per column (ne > 512), odd and large nc (k_qrows with 1, 2 or 4 c
    values per workgroup), |c| > 1 for some.  The fused and Q-row variants
    must agree bit for bit on the whole grid, and both with the oracle at a
    sample of points."""
    rng = np.random.default_rng(5000 + seed)
    n = int(rng.integers(2, 40))
    nvar = int(rng.integers(1, min(n, 9) + 1))
    T = int(rng.integers(2, 30))
    obs = synth.random_obs(rng, n, T, nvar, pmiss=float(rng.choice([0.0, 0.1, 0.3])),
                           max_missing=int(rng.integers(0, 4)), p1=float(rng.uniform(0.2, 0.8)))
    m, d, p = float(rng.choice([100, 400])), float(rng.choice([50, 100, 200])), 0.5
    ne, nc = int(rng.integers(300, 1400)), int(rng.integers(1, 1300))
    e, _ = mdp.grid(ne, 0.0, float(rng.choice([1.0, 1.2])))
    c, _ = mdp.grid(nc, 0.0, float(rng.choice([1.0, 1.5])))
    model = mdp.Model.from_obs(obs, m=m, p=p, d=d)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MDP_FUSED", mode)
        out[mode] = gpu_grid(model, e, c)
    assert np.array_equal(out["1"], out["0"], equal_nan=True)
    ie = np.unique(np.r_[0, ne - 1, rng.integers(0, ne, 6)])
    ic = np.unique(np.r_[0, nc - 1, rng.integers(0, nc, 6)])
    ref = oracle.OracleModel.from_obs(obs, m, p, d).loglik_grid(e[ie], c[ic])
    assert_loglik_close(out["0"][np.ix_(ie, ic)], ref)


@pytest.mark.parametrize("seed", range(int(os.environ.get("MDP_FUZZ_SMALL", "24"))))  # more: a longer fuzz
def test_random_problems(seed, engine_path):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(2, 48))
    nvar = int(rng.integers(1, min(n, 10) + 1))
    T = int(rng.integers(1, 40))
    maxm = int(rng.integers(0, 5))  # up to 16 states per year
    obs = synth.random_obs(rng, n, T, nvar, pmiss=float(rng.choice([0.0, 0.1, 0.3])),
                           max_missing=maxm, p1=float(rng.uniform(0.2, 0.8)))
    p = float(rng.choice([0.5, 0.3, 0.7]))
    m, d = float(rng.choice([100, 400, 1000])), float(rng.choice([50, 100, 200]))
    s = int(rng.integers(2, 12))
    lo, hi = float(rng.choice([0.0, 0.1])), float(rng.choice([1.0, 0.9, 1.3]))
    e, _ = mdp.grid(s, lo, hi)
    c, _ = mdp.grid(s + 3, 0.0, float(rng.choice([1.0, 2.0])))
    model = mdp.Model.from_obs(obs, m=m, p=p, d=d)
    got = gpu_grid(model, e, c)
    ref = oracle.OracleModel.from_obs(obs, m, p, d).loglik_grid(e, c)
    assert_loglik_close(got, ref)


def test_structural_zeros_exact(golden, engine_path):
    """Structural zeros (L = 0 exactly: an impossible transition, quirk Q5;
    the e = 0 / e >= 1 / c = 0 borders of the shipped example, where some
    year's change has probability 0) are -inf on every path -- not a small
    subnormal, which assert_loglik_close would let through on the underflow
    side and which a broken zero slot or padded gather would produce."""
    obs = np.array([[0, 1, 1, 1], [0, 0, 0, 0], [0, 1, 0, 1]])
    g, _ = mdp.grid(5)
    assert np.isneginf(gpu_grid(mdp.Model.from_obs(obs), g)).all()
    g, _ = mdp.grid(9, 0.0, 1.25)
    model = mdp.Model.load(golden / "occupancies.txt")
    got = gpu_grid(model, g)
    ref = oracle.OracleModel.load(golden / "occupancies.txt", 400, 0.5, 100).loglik_grid(g, g)
    zero = np.isneginf(ref)
    assert zero.sum() >= 9 and (ref[~zero] > -700).all()  # borders only: no underflow here
    assert np.array_equal(np.isneginf(got), zero)
    assert_loglik_close(got, ref)


def test_negative_c_refused(golden):
    """c < 0 is refused with MDP_EINVAL (include/midaspom.h): the item factors
    |n - pC| equal the reference's (1 - piold)(1 - pC) + piold pC
    (main_MIDASPOM.c:40) only for pC = min(1, c S) >= 0."""
    model = mdp.Model.load(golden / "occupancies.txt")
    g, _ = mdp.grid(5)
    with mdp.Engine(model) as eng:
        with pytest.raises(_lib.MidaspomError, match=r"c\[1\] = -0.25 \(the engine takes finite c >= 0\)"):
            eng.loglik_grid(g, np.array([0.0, -0.25, 0.5]))
        with pytest.raises(_lib.MidaspomError):
            eng.set_grid(g, -g[1:])
        for bad in (np.nan, np.inf):
            with pytest.raises(_lib.MidaspomError):
                eng.loglik_grid(g, np.array([0.5, bad]))
        assert np.isfinite(eng.loglik_grid(g, g)[1:-1, 1:]).all()  # the engine stays usable (e = 0, 1: -inf)


def test_single_year_and_constant_series(engine_path):
    for obs in (np.array([[1, 0, -1, 1]]), np.array([[0, 1, 1]] * 6), np.array([[1], [1], [0], [1]])):
        model = mdp.Model.from_obs(obs)
        g, _ = mdp.grid(7)
        ref = oracle.OracleModel.from_obs(obs).loglik_grid(g, g)
        assert_loglik_close(gpu_grid(model, g), ref)


def _wide_obs(rng, n, T, missing):
    """n patches x T years, every year occupied; `missing` = {year: k} puts k
    unvisited (-1) patches into that year (2^k possible states)."""
    obs = (rng.random((T, n)) < 0.6).astype(np.int32)
    obs[:, 0] = 1
    for yr, k in missing.items():
        obs[yr, rng.choice(np.arange(1, n), size=k, replace=False)] = -1
    return obs


def _wide_engine_run(model, e, c, path, monkeypatch):
    """Run on the named path and check it ran: "default" (years of 17-64
    states: the specialised kernel with its states in LDS; more: the wide
    kernels), "wide" (MDP_WIDE=1: k_witems + k_wq + the matrix-core forward
    k_fwd_hs for years of more than 64 states and up to 10 variable patches,
    else k_fwd_mmt, years of up to 1 024 states), "wide-mmt" (k_fwd_mmt,
    MDP_WIDE_MMA=2), "wide-mma5" (round 5's
    k_fwd_mma, MDP_WIDE_MMA=1, up to 256 states), "wide-hs" (k_fwd_hs through
    the hidden states, MDP_WIDE_MMA=3, up to 10 variable patches) or
    "wide-plain" (k_fwd_wide, MDP_WIDE_MMA=0)."""
    monkeypatch.delenv("MDP_WIDE", raising=False)
    monkeypatch.delenv("MDP_WIDE_MMA", raising=False)
    if path.startswith("wide"):
        monkeypatch.setenv("MDP_WIDE", "1")
    if path == "wide-plain":
        monkeypatch.setenv("MDP_WIDE_MMA", "0")
    if path == "wide-mma5":
        monkeypatch.setenv("MDP_WIDE_MMA", "1")
    if path == "wide-hs":
        monkeypatch.setenv("MDP_WIDE_MMA", "3")
    if path == "wide-mmt":
        monkeypatch.setenv("MDP_WIDE_MMA", "2")
    with mdp.Engine(model) as eng:
        got = eng.loglik_grid(e, c)
        launched, info = eng.launched(), eng.info()
    if path.startswith("wide") or model.npstates.max() > 64:
        assert info["variant"] >= 20000, info
        assert launched_forward(model, path) in launched, launched
    else:
        assert 10000 <= info["variant"] < 20000, info
        assert any(k.startswith("mdp_fwd_jit<reading") for k in launched), launched
    return got


def launched_forward(model, path):
    """The wide forward kernel instantiation `path` runs for this model."""
    npm = int(model.npstates.max())
    nvar = len(model.var_cols)
    rt8 = 4 if os.environ.get("MDP_HS_WAVES") == "16" else 2  # (8 waves a block by default: 32 points)
    if path == "wide-hs" and nvar <= 10 and len(model.npstates) > 1:
        nb = max(8, nvar)
        return f"k_fwd_hs<{ {8: rt8, 9: 2, 10: 1}[nb]},{nb}>"
    if path == "wide-mma5" and npm <= 256:
        return f"k_fwd_mma<{64 if npm <= 64 else 128 if npm <= 128 else 256}>"
    if path in ("default", "wide") and npm > 64 and nvar <= 10 and len(model.npstates) > 1:
        nb = max(8, nvar)
        return f"k_fwd_hs<{ {8: rt8, 9: 2, 10: 1}[nb]},{nb}>"
    if path in ("default", "wide", "wide-hs", "wide-mmt") and npm <= 1024:
        return f"k_fwd_mmt<{'4,128,2buf' if npm <= 128 else '2,256,1buf' if npm <= 256 else '2,512,1buf' if npm <= 512 else '1,1024,1buf'}>"
    return "k_fwd_wide"


@pytest.mark.parametrize("path", ["default", "wide", "wide-mma5", "wide-hs", "wide-mmt", "wide-plain"])
@pytest.mark.parametrize("missing", [{0: 5}, {3: 5}, {2: 6}, {4: 6}, {0: 8}, {3: 8}, {1: 5, 2: 6}, {0: 6, 4: 7},
                                     {1: 8, 2: 7}, {2: 7, 3: 8}])
def test_wide_years_vs_oracle(missing, path, monkeypatch):
    """Years with more than 4 missing patches (> 16 states), in year 0, in
    later years, in consecutive years: the reference expands 2^k states for
    any k (main_MIDASPOM.c:225-251) and propagates them (:371-384); up to 64
    states the specialised kernel keeps them in LDS, beyond that (and forced)
    the wide kernels run -- k_fwd_mmt<4> on the matrix cores (64 points a
    block), round 5's k_fwd_mma<64|128|256> and k_fwd_wide when asked."""
    rng = np.random.default_rng(sum(100 * y + k for y, k in missing.items()))
    obs = _wide_obs(rng, 12, 5, missing)
    model = mdp.Model.from_obs(obs)
    assert model.npstates.max() == 2 ** max(missing.values())
    g, _ = mdp.grid(5)
    got = _wide_engine_run(model, g, g, path, monkeypatch)
    ref = oracle.OracleModel.from_obs(obs).loglik_grid(g, g, threads=16)
    assert np.isfinite(ref).sum() >= 9
    assert_loglik_close(got, ref)


@pytest.mark.parametrize("seed", range(int(os.environ.get("MDP_FUZZ_WIDE", "6"))))  # more: a longer fuzz
def test_random_wide_problems(seed, monkeypatch):
    """Random problems with 5-7 missing patches in random years (32-128
    states) and random dispersal / grid bounds, on the wide path (whole
    launches and one c value per launch) against the oracle."""
    rng = np.random.default_rng(7000 + seed)
    n, T = int(rng.integers(8, 16)), int(rng.integers(2, 7))
    years = rng.choice(T, size=int(rng.integers(1, 3)), replace=False)
    missing = {int(y): int(rng.integers(5, 8)) for y in years}
    obs = _wide_obs(rng, n, T, missing)
    m, d, p = float(rng.choice([100, 400])), float(rng.choice([50, 100, 200])), float(rng.choice([0.5, 0.3]))
    model = mdp.Model.from_obs(obs, m=m, p=p, d=d)
    e, _ = mdp.grid(int(rng.integers(2, 6)), 0.0, float(rng.choice([1.0, 1.2])))
    c, _ = mdp.grid(int(rng.integers(2, 6)), 0.0, float(rng.choice([1.0, 1.5])))
    ref = oracle.OracleModel.from_obs(obs, m, p, d).loglik_grid(e, c, threads=16)
    for path, cb in (("default", None), ("wide", None), ("wide-mma5", None), ("wide-hs", None), ("wide-mmt", None),
                     ("wide-plain", None), ("wide", "1"), ("wide-hs", "1")):
        if cb:
            monkeypatch.setenv("MDP_WIDE_CB", cb)
        got = _wide_engine_run(model, e, c, path, monkeypatch)
        assert_loglik_close(got, ref)


@pytest.mark.parametrize("seed", range(int(os.environ.get("MDP_FUZZ_HS", "6"))))  # more: a longer fuzz
def test_random_hidden_state_problems(seed, monkeypatch):
    """Random 10-patch problems with 5-9 unvisited patches in random years
    (32-512 states, consecutive big years included) and random dispersal /
    grid bounds, on k_fwd_hs (8-, 9- and 10-variable cubes; whole and one c
    value per launch) against the oracle."""
    rng = np.random.default_rng(9100 + seed)
    T = int(rng.integers(3, 7))
    years = rng.choice(T, size=int(rng.integers(1, min(T, 3) + 1)), replace=False)
    missing = {int(y): int(rng.integers(5, 10)) for y in years}
    obs = _wide_obs(rng, 10, T, missing)
    m, d, p = float(rng.choice([100, 400])), float(rng.choice([50, 100, 200])), float(rng.choice([0.5, 0.3]))
    model = mdp.Model.from_obs(obs, m=m, p=p, d=d)
    e, _ = mdp.grid(int(rng.integers(2, 5)), 0.0, float(rng.choice([1.0, 1.2])))
    c, _ = mdp.grid(int(rng.integers(2, 5)), 0.0, float(rng.choice([1.0, 1.5])))
    ref = oracle.OracleModel.from_obs(obs, m, p, d).loglik_grid(e, c, threads=16)
    for cb in (None, "1"):
        if cb:
            monkeypatch.setenv("MDP_WIDE_CB", cb)
        got = _wide_engine_run(model, e, c, "wide-hs", monkeypatch)
        assert_loglik_close(got, ref)


def _big_obs(rng, missing, full=()):
    """10 patches x 6 years (2^10 hidden states): `missing` = {year: k}
    unvisited patches among patches 1-9 (2^k states), and every patch
    unvisited in the years of `full` (1 024 states)."""
    obs = _wide_obs(rng, 10, 6, missing)
    for yr in full:
        obs[yr, :] = -1
    return obs


@pytest.mark.parametrize("path", ["default", "wide-mmt", "wide-plain"])
@pytest.mark.parametrize("missing,full", [({1: 9}, ()), ({0: 9}, ()), ({2: 9, 3: 9}, ()), ({4: 8}, (2,)),
                                          ({}, (0,)), ({1: 9}, (2, 3)), ({3: 7}, (5,))],
                         ids=["512@1", "512@0", "512@2+3", "1024@2", "1024@0", "512@1+1024@2+3", "1024@5"])
def test_big_years_vs_oracle(missing, full, path, monkeypatch):
    """Years of 512 and 1 024 states (9 and 10 unvisited patches; the
    reference expands any number, main_MIDASPOM.c:222-255, and propagates
    them by dgemm, :371-384): k_fwd_mmt<2> / <1> on the matrix cores by
    default (a wave takes 2 or 4 column tiles a year), k_fwd_wide when asked;
    one year, consecutive years, year 0 (Q3: ones over its states) and the
    last year, against the oracle on a whole 6 x 5 grid."""
    rng = np.random.default_rng(17 + sum(100 * y + k for y, k in missing.items()) + 7 * sum(full))
    obs = _big_obs(rng, missing, full)
    model = mdp.Model.from_obs(obs)
    assert model.npstates.max() == (1024 if full else 2 ** max(missing.values()))
    e, _ = mdp.grid(6, 0.0, 1.1)
    c, _ = mdp.grid(5)
    got = _wide_engine_run(model, e, c, path, monkeypatch)
    ref = oracle.OracleModel.from_obs(obs).loglik_grid(e, c, threads=16)
    assert np.isfinite(ref).sum() >= 9
    assert_loglik_close(got, ref)


@pytest.mark.parametrize("path", ["default", "wide-mmt", "wide-plain"])
def test_big_survey_series_sampled(tmp_path, path, monkeypatch):
    """The 10-variable-patch survey series of scripts/wide_timing.py (60 %
    unvisited: years of up to 1 024 states, two of 512; 643 328 uses per
    point): k_fwd_mmt<1> (16 points a block) and k_fwd_wide on a 37 x 23
    grid (the last point block partial), sampled against the oracle."""
    cfg = dict(synth.CONFIG2, nvar=10, pmiss=0.6, seed=5, T=30)
    f = synth.write(tmp_path / "big60.txt", **cfg)
    model = mdp.Model.load(f)
    assert model.npstates.max() == 1024
    e, _ = mdp.grid(37)
    c, _ = mdp.grid(23)
    got = _wide_engine_run(model, e, c, path, monkeypatch)
    rng = np.random.default_rng(8)
    ie, ic = rng.integers(0, 37, 16), rng.integers(0, 23, 16)
    ie[:4], ic[:4] = [0, 36, 0, 36], [0, 0, 22, 22]
    ref = oracle.OracleModel.load(f).loglik_points(e[ie], c[ic], threads=16)
    assert np.isfinite(ref).sum() >= 8
    assert_loglik_close(got[ie, ic], ref)


@pytest.mark.parametrize("path", ["default", "wide", "wide-hs"])
def test_wide_survey_series_sampled(tmp_path, path, monkeypatch):
    """A survey-like series (the Appendix C generator, config-2 shape, 45 %
    of the variable patches unvisited in each year: 2-64 states per year,
    wide years back to back, 7 264 uses: the specialised kernel in chunks
    with its states in LDS, and the wide kernels) on a 128 x 128 grid,
    sampled against the oracle."""
    cfg = dict(synth.CONFIG2, pmiss=0.45, seed=5, T=30)
    f = synth.write(tmp_path / "wide.txt", **cfg)
    model = mdp.Model.load(f)
    assert model.npstates.max() == 64
    g, _ = mdp.grid(128)
    got = _wide_engine_run(model, g, g, path, monkeypatch)
    rng = np.random.default_rng(3)
    ie, ic = rng.integers(0, 128, 64), rng.integers(0, 128, 64)
    ie[:4], ic[:4] = [0, 127, 0, 127], [0, 0, 127, 127]
    ref = oracle.OracleModel.load(f).loglik_points(g[ie], g[ic], threads=16)
    assert np.isfinite(ref).sum() >= 48
    assert_loglik_close(got[ie, ic], ref)


@pytest.mark.parametrize("path", ["default", "wide-mmt", "wide-plain"])
def test_wide_survey_series_128_states(tmp_path, path, monkeypatch):
    """The 60 %-unvisited survey series of scripts/wide_timing.py (up to 128
    states a year, 66 416 uses per point): k_fwd_mmt<4> by default, and
    k_fwd_wide, on a 130 x 70 grid (three 64-point blocks, the last partial),
    sampled against the oracle."""
    cfg = dict(synth.CONFIG2, pmiss=0.6, seed=5, T=50)
    f = synth.write(tmp_path / "wide60.txt", **cfg)
    model = mdp.Model.load(f)
    assert model.npstates.max() == 128
    e, _ = mdp.grid(130)
    c, _ = mdp.grid(70)
    got = _wide_engine_run(model, e, c, path, monkeypatch)
    rng = np.random.default_rng(4)
    ie, ic = rng.integers(0, 130, 24), rng.integers(0, 70, 24)
    ie[:4], ic[:4] = [0, 129, 0, 129], [0, 0, 69, 69]
    ref = oracle.OracleModel.load(f).loglik_points(e[ie], c[ic], threads=16)
    assert np.isfinite(ref).sum() >= 16
    assert_loglik_close(got[ie, ic], ref)


@pytest.mark.parametrize("path", ["default", "wide-mmt"])
def test_wide_survey_series_256_states(tmp_path, path, monkeypatch):
    """A 75 %-unvisited survey series (three years of 256 states, 257 024
    uses per point): k_fwd_mmt<4> (64 points a block)
    on a 70 x 40 grid (three 32-point blocks, the last partial), sampled
    against the oracle."""
    cfg = dict(synth.CONFIG2, pmiss=0.75, seed=5, T=30)
    f = synth.write(tmp_path / "wide75.txt", **cfg)
    model = mdp.Model.load(f)
    assert model.npstates.max() == 256
    e, _ = mdp.grid(70)
    c, _ = mdp.grid(40)
    got = _wide_engine_run(model, e, c, path, monkeypatch)
    rng = np.random.default_rng(6)
    ie, ic = rng.integers(0, 70, 16), rng.integers(0, 40, 16)
    ie[:4], ic[:4] = [0, 69, 0, 69], [0, 0, 39, 39]
    ref = oracle.OracleModel.load(f).loglik_points(e[ie], c[ic], threads=16)
    assert np.isfinite(ref).sum() >= 10
    assert_loglik_close(got[ie, ic], ref)


@pytest.mark.parametrize("fname,s", [("config2_64x50.txt", 64), ("occupancies.txt", 33)])
def test_wide_path_matches_direct_path(golden, monkeypatch, fname, s):
    """Forced onto the wide path, a problem the register kernels also run
    gives the same log-likelihoods (sums reordered: ~1e-13)."""
    model = mdp.Model.load(golden / fname)
    g, _ = mdp.grid(s)
    a = gpu_grid(model, g)
    monkeypatch.setenv("MDP_WIDE", "1")
    with mdp.Engine(model) as eng:
        assert eng.info()["variant"] >= 20000
        b = eng.loglik_grid(g, g)
        assert set(eng.kernel_ms()) <= {"k_zrows", "k_witems+k_wq", "k_witems", "k_fwd_wide", "k_fwd_mma", "k_fwd_mmt",
                                        "k_fwd_hs"}
    assert_loglik_close(b, a, atol=1e-11)


# ---------------------------------------------------------------------------
# BASELINE full sizes: nested sub-grid / sampled points against the oracle
# ---------------------------------------------------------------------------
def test_config2_full_grid_nested(golden):
    """s = 512: the nested -s 74 sub-grid (511 = 7*73) plus the border rows."""
    model = mdp.Model.load(golden / "config2_64x50.txt")
    g, win = mdp.grid(512)
    got = gpu_grid(model, g)
    # e = 0, e = 1 and c = 0 rows/cols are impossible (L = 0 -> -inf); the
    # oracle comparison below checks the -inf positions
    assert not np.isnan(got).any() and np.isfinite(got[1:-1, 1:]).all()
    idx = np.arange(0, 512, 7)
    om = oracle.OracleModel.load(golden / "config2_64x50.txt")
    ee, cc = np.meshgrid(g[idx], g[idx], indexing="ij")
    ref = om.loglik_points(ee.ravel(), cc.ravel(), threads=16).reshape(idx.size, idx.size)
    assert_loglik_close(got[np.ix_(idx, idx)], ref)


def test_config3_full_grid_sampled(golden):
    """Config 3's 1024^2 grid, sampled against the oracle: the reading kernel
    at 512 threads (a column of a tall grid in one block), after k_qrows."""
    model = mdp.Model.load(golden / "config3_256x200.txt")
    g, win = mdp.grid(1024)
    with mdp.Engine(model) as eng:
        got = eng.loglik_grid(g, g)
        launched = eng.launched()
    assert "mdp_fwd_jit<reading,kb512>" in launched, launched
    assert np.isfinite(got).any()
    rng = np.random.default_rng(7)
    ie, ic = rng.integers(0, 1024, 160), rng.integers(0, 1024, 160)
    ie[:4], ic[:4] = [0, 1023, 0, 1023], [0, 0, 1023, 1023]
    om = oracle.OracleModel.load(golden / "config3_256x200.txt")
    ref = om.loglik_points(g[ie], g[ic], threads=16)
    assert_loglik_close(got[ie, ic], ref)
    # posterior normalisation over the whole grid is finite and sums to ~1/win^2 trapezoid
    lt = mdp.log_total(got, win)
    assert np.isfinite(lt)


def test_grid_split_invariance(golden):
    """Row slabs computed separately equal the full grid (the multi-GPU and
    multi-rank partition relies on it)."""
    model = mdp.Model.load(golden / "config2_64x50.txt")
    g, _ = mdp.grid(129)
    with mdp.Engine(model) as eng:
        full = eng.loglik_grid(g, g)
        parts = [eng.loglik_grid(g[a:b], g) for a, b in [(0, 40), (40, 41), (41, 129)]]
    assert np.array_equal(np.vstack(parts), full)


def test_device_run_matches_host_path(golden):
    import torch
    model = mdp.Model.load(golden / "config2_64x50.txt")
    g, _ = mdp.grid(96)
    with mdp.Engine(model) as eng:
        host = eng.loglik_grid(g, g)
        eng.set_grid(g, g)
        out = torch.empty((96, 100), dtype=torch.float64, device="cuda")
        eng.set_profiling(True)
        eng.run(out.data_ptr(), 100, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ms = eng.kernel_ms()
    assert np.array_equal(out[:, :96].cpu().numpy(), host)
    assert set(ms) in ({"k_forward"}, {"k_qrows", "k_forward"}, {"k_zpv", "k_coefs", "k_forward"})
    assert all(v > 0 for v in ms.values())


def test_time_kernels_leaves_run_output(golden):
    import torch
    model = mdp.Model.load(golden / "config3_256x200.txt")
    g, _ = mdp.grid(600)
    with mdp.Engine(model) as eng:
        eng.set_grid(g, g)
        st = torch.cuda.current_stream().cuda_stream
        a = torch.empty((600, 600), dtype=torch.float64, device="cuda")
        b = torch.empty_like(a)
        eng.run(a.data_ptr(), 600, st)
        ms = eng.time_kernels(b.data_ptr(), 600, st, reps=3)
        torch.cuda.synchronize()
    assert "k_forward" in ms and all(v > 0 for v in ms.values())
    assert torch.equal(a, b)


@pytest.mark.parametrize("fname,s", [("config2_64x50.txt", 256), ("config3_256x200.txt", 128)])
def test_direct_and_generic_paths_agree(golden, monkeypatch, fname, s):
    model = mdp.Model.load(golden / fname)
    g, _ = mdp.grid(s, 0.0, 1.0)
    c, _ = mdp.grid(s + 1, 0.0, 1.5)
    monkeypatch.delenv("MDP_JIT", raising=False)
    with mdp.Engine(model) as eng:
        assert eng.info()["variant"] >= 10000  # the direct path is the default
        a = eng.loglik_grid(g, c)
        assert set(eng.kernel_ms()) <= {"k_zrows", "k_qrows", "k_forward"}
    monkeypatch.setenv("MDP_JIT", "0")
    with mdp.Engine(model) as eng:
        assert eng.info()["variant"] < 10000
        b = eng.loglik_grid(g, c)
    assert_loglik_close(a, b, atol=1e-11)


@pytest.mark.parametrize("fname,ne,nc", [("config2_64x50.txt", 200, 200), ("config3_256x200.txt", 64, 64),
                                          ("config2_64x50.txt", 1100, 37), ("config3_256x200.txt", 700, 33)])
def test_fused_and_qrows_identical(golden, monkeypatch, fname, ne, nc):
    """The fused forward kernel runs k_qrows' arithmetic for its column: the
    two direct variants agree bit for bit (also with several e blocks per
    column for the Q-row variant; config 3's tables do not fit the fused
    kernel's LDS, so there both runs take k_qrows)."""
    model = mdp.Model.load(golden / fname)
    e, _ = mdp.grid(ne)
    c, _ = mdp.grid(nc)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MDP_FUSED", mode)
        with mdp.Engine(model) as eng:
            out[mode] = eng.loglik_grid(e, c)
    assert np.array_equal(out["1"], out["0"])


def test_explicit_device_list(golden):
    model = mdp.Model.load(golden / "occupancies.txt")
    g, _ = mdp.grid(31)
    a = gpu_grid(model, g, devices=[0])
    b = gpu_grid(model, g)
    assert np.array_equal(a, b)


# ---------------------------------------------------------------------------
# the CLI drop-in
# ---------------------------------------------------------------------------
def test_cli_matches_oracle_file(golden, tmp_path):
    out = tmp_path / "post.txt"
    r = subprocess.run([str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", "101", "-i",
                        str(golden / "occupancies.txt"), "-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Total log-likelihood=-39.34251\n" in r.stdout
    lines = r.stdout.splitlines()
    assert lines[0] == "------ MIDASPOM, beta version ------"
    assert lines[3] == "\tWindow size=0.010000, number of steps=101"
    assert "Number of habitat patches: 8" in lines and "Number of sampled years: 7" in lines
    assert sum(1 for x in lines if x.endswith("% done")) == 101 and "100.00% done" in lines
    ref_out = tmp_path / "ref.txt"
    oracle.run(golden / "occupancies.txt", ref_out, s=101)
    got_txt, ref_txt = out.read_text(), ref_out.read_text()
    # identical bit layout: same cell count, tabs and newlines
    assert [len(l.split("\t")) for l in got_txt.split("\n")] == [len(l.split("\t")) for l in ref_txt.split("\n")]
    assert_posterior_close(np.loadtxt(out), np.loadtxt(ref_out))


@pytest.mark.parametrize("fname,flags", [
    ("occupancies.txt", ["-s", "1"]),            # one point (1, 1): -inf, Ltot -nan
    ("occupancies.txt", ["-s", "2"]),            # the grid corners only: all -inf
    ("occupancies.txt", ["-s", "37", "-p", "0.3", "-l", "0.1", "-u", "0.9", "-m", "200", "-d", "50"]),
    ("occupancies.txt", ["-s", "23", "-l", "0.2", "-u", "1.4"]),  # e, c past 1 (clamped)
    ("manual_p3_obs.txt", ["-s", "9", "-m", "400", "-d", "200", "-p", "0.7"]),
    ("config2_64x50.txt", ["-s", "19", "-l", "0.05", "-u", "0.95", "-p", "0.4"]),
])
def test_cli_flags_match_oracle_cli(golden, tmp_path, fname, flags):
    """Every flag of the drop-in (main_MIDASPOM.c:66-139) against the oracle's
    own CLI (oracle/orc_main.c) with the same command line, including the
    one- and two-point grids: same 'Total log-likelihood=' line, same file
    layout and '-nan' cells, posteriors within the parity bar."""
    out, ref_out = tmp_path / "post.txt", tmp_path / "ref.txt"
    r = subprocess.run([str(_lib.CLI_PATH), *flags, "-i", str(golden / fname), "-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    orc = subprocess.run([str(oracle.CLI), *flags, "-i", str(golden / fname),
                          "-o", str(ref_out)], capture_output=True, text=True, timeout=120)
    assert orc.returncode == 0, orc.stderr
    total = [ln for ln in r.stdout.splitlines() if ln.startswith("Total log-likelihood=")]
    assert total == [ln for ln in orc.stdout.splitlines() if ln.startswith("Total log-likelihood=")]
    got_txt, ref_txt = out.read_text(), ref_out.read_text()
    assert [ln.count("\t") for ln in got_txt.split("\n")] == [ln.count("\t") for ln in ref_txt.split("\n")]
    got_cells = [x for x in got_txt.split()]
    ref_cells = [x for x in ref_txt.split()]
    assert [x == "-nan" for x in got_cells] == [x == "-nan" for x in ref_cells]
    s = int(flags[1])
    got = np.array([float(x) for x in got_cells]).reshape(s, s)
    ref = np.array([float(x) for x in ref_cells]).reshape(s, s)
    assert_posterior_close(got, ref)


@pytest.mark.parametrize("pmiss,nvar,T,s", [(0.6, 8, 50, 9), (0.6, 10, 30, 5)], ids=["128states", "1024states"])
def test_cli_wide_series_match_oracle_cli(tmp_path, pmiss, nvar, T, s):
    """The drop-in CLI on survey series whose years reach 128 and 1 024
    states (the wide path, `k_fwd_hs` by default) against the oracle's CLI
    with the same command line: same 'Total log-likelihood=' line and file
    layout, posteriors within the parity bar."""
    f = synth.write(tmp_path / "wide.txt", **dict(synth.CONFIG2, pmiss=pmiss, seed=5, T=T, nvar=nvar))
    out, ref_out = tmp_path / "post.txt", tmp_path / "ref.txt"
    flags = ["-s", str(s), "-m", "400", "-d", "100"]
    r = subprocess.run([str(_lib.CLI_PATH), *flags, "-i", str(f), "-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    orc = subprocess.run([str(oracle.CLI), *flags, "-i", str(f), "-o", str(ref_out)],
                         capture_output=True, text=True, timeout=120)
    assert orc.returncode == 0, orc.stderr
    total = [ln for ln in r.stdout.splitlines() if ln.startswith("Total log-likelihood=")]
    assert total == [ln for ln in orc.stdout.splitlines() if ln.startswith("Total log-likelihood=")]
    got_txt, ref_txt = out.read_text(), ref_out.read_text()
    assert [ln.count("\t") for ln in got_txt.split("\n")] == [ln.count("\t") for ln in ref_txt.split("\n")]
    got_cells, ref_cells = got_txt.split(), ref_txt.split()
    assert [x == "-nan" for x in got_cells] == [x == "-nan" for x in ref_cells]
    got = np.array([float(x) for x in got_cells]).reshape(s, s)
    ref = np.array([float(x) for x in ref_cells]).reshape(s, s)
    assert_posterior_close(got, ref)


def test_cli_all_nan_file(tmp_path):
    inp = tmp_path / "q5.txt"
    inp.write_text("0 1 1 1\n0 0 0 0\n0 1 0 1\n")
    out = tmp_path / "o.txt"
    r = subprocess.run([str(_lib.CLI_PATH), "-s", "3", "-i", str(inp), "-o", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    assert "Total log-likelihood=-inf" in r.stdout
    assert out.read_text() == "-nan\t-nan\t-nan\t\n" * 3


@pytest.mark.gpu
def test_config1_after_other_kernels(golden):
    """Stale LDS / device memory from earlier kernels must not leak into the
    result: the scenario engine (154 KB of LDS per workgroup) runs first, then
    the config-1 grid (n = nvar = 8, no always-zero column) is checked.  This
    caught a staging race of a global_load_lds staging variant (since removed)."""
    row = mdp.first_row(golden / "occupancies.txt")
    with mdp.Scenario(row, "dieoff", m=400, d=100) as sc:
        sc.lik(np.linspace(0.0, 1.0, 64), np.array([0.3, 0.7]), mdp.kgrid(4), ts=5, tdis=3)
    g, _ = mdp.grid(50)
    model = mdp.Model.load(golden / "occupancies.txt", m=400, d=100)
    got = gpu_grid(model, g)
    ref = oracle.OracleModel.load(golden / "occupancies.txt", 400, 0.5, 100).loglik_grid(g, g)
    assert_loglik_close(got, ref)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_grid_dropping_columns_then_full_grid(monkeypatch, fused):
    """A c grid so small that every always-zero column's factor rounds to 1.0
    (all of them are dropped: kmax = 0, the fused image holds only zero Z
    rows), then a full grid on the same engine (the image is rebuilt with
    every column).  Both variants against the oracle."""
    monkeypatch.setenv("MDP_FUSED", fused)
    rng = np.random.default_rng(77)
    obs = synth.random_obs(rng, 24, 12, 4, pmiss=0.1, max_missing=3, p1=0.9)
    model = mdp.Model.from_obs(obs, m=400.0, p=0.5, d=100.0)
    ref_model = oracle.OracleModel.from_obs(obs, 400.0, 0.5, 100.0)
    e, _ = mdp.grid(9, 0.0, 1.0)
    tiny = np.array([0.0, 1e-30, 3e-25, 1e-21], dtype=np.float64)
    full, _ = mdp.grid(7, 0.0, 1.0)
    with mdp.Engine(model) as eng:
        for c in (tiny, full, tiny):
            ref = ref_model.loglik_grid(e, c)
            assert np.isfinite(ref).sum() >= 20  # not only impossible points
            assert_loglik_close(eng.loglik_grid(e, c), ref)


@pytest.mark.parametrize("fname", ["config2_64x50.txt", "config3_256x200.txt", "occupancies.txt"])
def test_work_fact_per_point_terms_from_the_model(golden, fname):
    """mdp_engine_work_fact's per-point terms restated from the enumerated
    model alone.  Ratio forms (the numerator, ABI 8): per
    point the set-up (1 - x, the division, the B and g power tables past
    their first powers), each distinct Q group (A & B, B) once (2 |A & B|),
    g^d once per distinct (group, d = |A| - |A & B| > 0) on s-form points,
    the state updates npc (2 npp - 1), one pre-scale per source above the
    year's minimum |A|, the deferred-exponent flushes (E >= 192: npc + the
    power by squaring), the end (np_last + 1 + the final power).  Legacy
    direct form: every use 2 |A&B| + 3, the weight table 2 maxA + one
    product per W[|A|][m] used, the prior sum 2 np_last - 1."""
    model = mdp.Model.load(golden / fname)
    ids, ss = model.year_ids, model.short_state
    use, use_min, mmax, seen = 0.0, 0.0, {}, set()
    groups, gd, yr, dp, dg = set(), set(), 0.0, 0, 0
    E, flushes = 0, []

    def powcost(x):
        return 0 if x <= 1 else x.bit_length() - 1 + bin(x).count("1") - 1

    for t in range(1, model.tmax):
        a_src = [bin(int(ss[a])).count("1") for a in ids[t - 1]]
        for b in ids[t]:
            for a in ids[t - 1]:
                A, B = int(ss[a]), int(ss[b])
                nX, nA = bin(A & B).count("1"), bin(A).count("1")
                use += 2 * nX + 3
                if (A & B, B, nA) not in seen:  # P depends on (A & B, B, |A|) only
                    seen.add((A & B, B, nA))
                    use_min += 2 * nX + 1
                mmax[nA] = max(mmax.get(nA, -1), nX)
                if (A & B, B) not in groups:
                    groups.add((A & B, B))
                    yr += 2 * nX
                if nA > nX:
                    dg = max(dg, nA - nX)
                    if (A & B, B, nA - nX) not in gd:
                        gd.add((A & B, B, nA - nX))
        use_min += len(ids[t]) * (2 * len(ids[t - 1]) - 1)  # the state updates of year t
        amin = min(a_src)
        dp = max(dp, max(a_src) - amin)
        yr += len(ids[t]) * (2 * len(ids[t - 1]) - 1) + sum(1 for a in a_src if a > amin)
        E += amin
        if E >= 192:
            yr += len(ids[t]) + powcost(E)
            E = 0
    maxA = max(mmax) if mmax else 0
    weight = 2 * maxA + sum(m + 1 for m in mmax.values())
    final = 2 * len(ids[-1]) - 1
    setup_t = 2 + max(dp - 1, 0)
    setup_s = setup_t + max(dg - 1, 0)
    use_s, use_t = yr + len(gd), yr
    final_r = len(ids[-1]) + 1 + (powcost(E) + 1 if E else 0)
    g, _ = mdp.grid(8)  # e = i/7: rows 0-3 s-form (x < 1/2), 4-7 t-form
    with mdp.Engine(model) as eng:
        eng.set_grid(g, g)
        w = eng.work_fact(8, 8)
    assert (w["use_pt"], w["use_pt_min"], w["weight_pt"], w["final_pt"]) == (use, use_min, weight, final)
    per_c = w["z_c"] + w["pc_c"] + w["item_c"] + w["q_c"]
    assert w["flop"] == 8 * per_c + 64 * (use + weight + final)
    assert w["flop_min_direct"] == 8 * per_c + 64 * (use_min + weight + final)
    assert w["setup_pt"] == pytest.approx(0.5 * (setup_s + setup_t))
    assert w["use_pt_ratio"] == pytest.approx(0.5 * (use_s + use_t))
    assert w["final_pt_ratio"] == final_r
    assert w["flop_min"] == pytest.approx(8 * per_c + 64 * (0.5 * (setup_s + use_s + setup_t + use_t) + final_r))


def test_wide_single_year():
    """One year with 6 unvisited patches (64 states), no transition: the wide
    path's L = prior0 * 64 (Q3 semantics, main_MIDASPOM.c:368-392)."""
    obs = np.array([[1, -1, -1, 1, -1, -1, -1, -1, 0, 1]])
    model = mdp.Model.from_obs(obs, p=0.3)
    g, _ = mdp.grid(4)
    with mdp.Engine(model) as eng:
        assert eng.info()["variant"] >= 20000
        got = eng.loglik_grid(g, g)
    ref = oracle.OracleModel.from_obs(obs, 400.0, 0.3, 100.0).loglik_grid(g, g)
    assert_loglik_close(got, ref)
    assert np.allclose(got, np.log(float(model.prior[0]) * 64))


def test_engine_log_accuracy():
    """The forward kernels' FP64 log (mdp_log, hipRTC prelude) against the
    host libm on values across the whole double range: subnormals, powers of
    two, values near 1 and sqrt(2), the special cases.  Bound: 2 ulp of the
    result (or 2^-1074 absolute near log 1 = 0)."""
    rng = np.random.default_rng(17)
    x = np.concatenate([
        np.exp(rng.uniform(-745.0, 709.0, 200_000)),
        rng.uniform(0.5, 2.0, 100_000),
        1.0 + rng.uniform(-1e-6, 1e-6, 20_000),
        np.sqrt(2.0) * (1.0 + rng.uniform(-1e-12, 1e-12, 1_000)),
        2.0 ** np.arange(-1074, 1024, dtype=np.float64),
        np.array([5e-324, 1e-310, 2.2250738585072014e-308, 1.0, np.nextafter(1.0, 2.0), np.nextafter(1.0, 0.0),
                  np.finfo(np.float64).max]),
    ])
    y = np.empty_like(x)
    _lib.check(_lib.lib().mdp_log_check(x.ctypes.data_as(_lib.c_dbl_p), y.ctypes.data_as(_lib.c_dbl_p), x.size))
    import math
    ref = np.array([math.log(v) for v in x])  # glibc: correctly rounded to < 1 ulp
    ulp = np.spacing(np.abs(ref))
    err = np.abs(y - ref)
    assert (err <= 2 * ulp + 5e-324).all(), float((err / ulp).max())
    sp = np.array([0.0, -0.0, -1.0, np.inf, np.nan, -np.inf])
    ys = np.empty_like(sp)
    _lib.check(_lib.lib().mdp_log_check(sp.ctypes.data_as(_lib.c_dbl_p), ys.ctypes.data_as(_lib.c_dbl_p), sp.size))
    assert ys[0] == -np.inf and ys[1] == -np.inf and np.isnan(ys[2]) and ys[3] == np.inf
    assert np.isnan(ys[4]) and np.isnan(ys[5])
