"""GPU parity for surveys with many variable patches (nvar 11-24): the
reference takes any nvar (main_MIDASPOM.c:172-175, 198-211) and the engine
accepts up to 24, with kernel templates sized for 16 and 24 variable columns
(k_qrows<16|24,...>, k_witems<16|24>, k_coefs<...,16|24>) and forward
kernels of degree 16 and 24 (states with 9-16 and 17-24 occupied patches).
Every such template is run here against the oracle at sampled grid points,
and the test asserts from the engine's own launch record
(mdp_engine_launched) that the intended instantiation ran.

The problems alternate dense years (11, 15 or 19 occupied patches) with
sparse ones (at most 3-4 occupied, some unvisited), so every state carries
many occupied patches while consecutive years overlap little -- the shape
that keeps the direct plan's Q groups within the LDS (synth.alternating_obs).
Tolerance: |dlogL| <= 1e-9 (tests/test_gpu_parity.py)."""
from __future__ import annotations

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle
from midaspom_amd import synth

from test_gpu_parity import assert_loglik_close

pytestmark = pytest.mark.gpu

# nvar -> (n, T, nvar, dense, sparse, nmiss, seed); maxA = dense
PROBLEMS = {12: (16, 8, 12, 11, 4, 2, 1), 16: (20, 8, 16, 15, 4, 2, 2), 20: (22, 7, 20, 19, 3, 2, 3)}
NV = {12: 16, 16: 16, 20: 24}    # k_qrows / k_witems / k_coefs template width
DEG = {12: 16, 16: 16, 20: 24}   # forward degree bucket (maxA 11 / 15 / 19)

E_BIG, _ = mdp.grid(65)           # e grid of every path
C_BIG, _ = mdp.grid(601)          # >= 512 c values: k_qrows takes 2 per workgroup (nvar <= 16)
E_SMALL, C_SMALL = E_BIG[::4], C_BIG[::40]   # 17 x 16 sub-grid (generic path: its Z/PV block is 2^nvar per c)

_REF = {}


def _problem(nvar):
    n, T, nv, dense, sparse, nmiss, seed = PROBLEMS[nvar]
    obs = synth.alternating_obs(np.random.default_rng(seed), n, T, nv, dense, sparse, nmiss)
    return obs, mdp.Model.from_obs(obs, m=400.0, p=0.5, d=100.0)


def _reference(nvar):
    """Oracle log-likelihoods at sampled points of the small grid (shared by
    every path of one problem; the dense oracle costs ~5 s a point at nvar 20)."""
    if nvar not in _REF:
        obs, _ = _problem(nvar)
        rng = np.random.default_rng(100 + nvar)
        npts = 12 if nvar == 20 else 24
        ie = np.r_[1, E_SMALL.size - 1, rng.integers(1, E_SMALL.size, npts - 2)]
        ic = np.r_[1, C_SMALL.size - 1, rng.integers(1, C_SMALL.size, npts - 2)]
        ref = oracle.OracleModel.from_obs(obs, 400.0, 0.5, 100.0).loglik_points(E_SMALL[ie], C_SMALL[ic],
                                                                                  threads=16)
        assert np.isfinite(ref).sum() >= npts // 2
        _REF[nvar] = (ie, ic, ref)
    return _REF[nvar]


def _run(model, e, c, env, monkeypatch):
    for k in ("MDP_JIT", "MDP_FUSED", "MDP_WIDE", "MDP_WIDE_CB", "MDP_WIDE_MMA"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with mdp.Engine(model) as eng:
        out = eng.loglik_grid(e, c)
        return out, eng.launched(), eng.info()


@pytest.mark.parametrize("nvar", sorted(PROBLEMS))
def test_model_shape(nvar):
    _, model = _problem(nvar)
    ss = model.short_state
    occ = max(bin(int(s)).count("1") for s in ss)
    assert model.nvar == nvar and occ == PROBLEMS[nvar][3]
    assert (9 <= occ <= 16) if DEG[nvar] == 16 else (17 <= occ <= 24)


@pytest.mark.parametrize("nvar", sorted(PROBLEMS))
def test_direct_fused(nvar, monkeypatch):
    """Small grid, default: the hipRTC forward kernel computes its column's Q itself."""
    _, model = _problem(nvar)
    ie, ic, ref = _reference(nvar)
    got, launched, info = _run(model, E_SMALL, C_SMALL, {}, monkeypatch)
    assert info["variant"] >= 10000
    assert f"mdp_fwd_jit<fused,maxA{PROBLEMS[nvar][3]}>" in launched, launched
    assert_loglik_close(got[ie, ic], ref)


@pytest.mark.parametrize("nvar", sorted(PROBLEMS))
@pytest.mark.parametrize("grid", ["narrow", "wide601"])
def test_direct_qrows(nvar, grid, monkeypatch):
    """k_qrows<NV, 0, CB> + the reading forward kernel: CB = 1 on a narrow c
    grid, CB = 2 on 601 c values (nvar <= 16; nvar > 16 always takes 1)."""
    _, model = _problem(nvar)
    ie, ic, ref = _reference(nvar)
    c = C_SMALL if grid == "narrow" else C_BIG
    got, launched, _ = _run(model, E_BIG, c, {"MDP_FUSED": "0"}, monkeypatch)
    cb = 2 if (grid == "wide601" and nvar <= 16) else 1
    assert f"k_qrows<{NV[nvar]},0,{cb}>" in launched, launched
    assert f"mdp_fwd_jit<reading,maxA{PROBLEMS[nvar][3]}>" in launched, launched
    ce = 1 if grid == "narrow" else 40
    assert_loglik_close(got[ie * 4, ic * ce], ref)


@pytest.mark.parametrize("nvar", sorted(PROBLEMS))
def test_direct_paths_agree_bitwise(nvar, monkeypatch):
    """The fused and Q-row variants do identical arithmetic."""
    _, model = _problem(nvar)
    a, _, _ = _run(model, E_SMALL, C_SMALL, {"MDP_FUSED": "1"}, monkeypatch)
    b, _, _ = _run(model, E_SMALL, C_SMALL, {"MDP_FUSED": "0"}, monkeypatch)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("nvar", sorted(PROBLEMS))
def test_generic_path(nvar, monkeypatch):
    """MDP_JIT=0: k_zpv + k_coefs<., ., NV> + the degree-16/24 forward kernel."""
    _, model = _problem(nvar)
    ie, ic, ref = _reference(nvar)
    got, launched, info = _run(model, E_SMALL, C_SMALL, {"MDP_JIT": "0"}, monkeypatch)
    assert info["variant"] < 10000
    assert any(k.startswith("k_coefs<") and k.endswith(f",{NV[nvar]}>") for k in launched), launched
    assert any(k.startswith("k_forward") and f",{DEG[nvar]}," in k for k in launched), launched
    assert_loglik_close(got[ie, ic], ref)


@pytest.mark.parametrize("nvar", sorted(PROBLEMS))
@pytest.mark.parametrize("chunked", [False, True])
@pytest.mark.parametrize("mma", [True, False])
def test_wide_path(nvar, chunked, mma, monkeypatch):
    """MDP_WIDE=1: k_zrows + k_witems<NV> + k_wq + the forward on the matrix
    cores, k_fwd_mmt (or k_fwd_wide, MDP_WIDE_MMA=0), whole and one c value
    per item launch."""
    _, model = _problem(nvar)
    ie, ic, ref = _reference(nvar)
    env = {"MDP_WIDE": "1", **({"MDP_WIDE_CB": "1"} if chunked else {}), **({} if mma else {"MDP_WIDE_MMA": "0"})}
    got, launched, info = _run(model, E_SMALL, C_SMALL, env, monkeypatch)
    assert info["variant"] >= 20000
    fwd = "k_fwd_mmt<4,128,2buf>" if mma else "k_fwd_wide"
    assert {f"k_witems<{NV[nvar]}>", "k_wq", fwd, "k_zrows"} <= launched, launched
    assert_loglik_close(got[ie, ic], ref)
