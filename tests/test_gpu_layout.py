"""Output layout of the device-resident run (mdp_engine_set_layout, ABI 6):
MDP_LAYOUT_CE writes log L of point (ie, ic) at d_out[ic*ld + ie] instead of
the reference's lik[i][j] order d_out[ie*ld + ic] (main_MIDASPOM.c:390).  The
kernels are the same code objects with the strides as arguments, so every
path must give the EC result transposed, bit for bit, and leave the padding
past the extent untouched."""
from __future__ import annotations

import numpy as np
import pytest

import midaspom_amd as mdp
from pathlib import Path

GOLDEN = Path(__file__).parent / "golden"

pytestmark = pytest.mark.gpu

KNOBS = ("MDP_JIT", "MDP_FUSED", "MDP_WIDE", "MDP_JIT_CHUNK", "MDP_JIT_GATHER", "MDP_QGLOBAL", "MDP_VSPLIT", "MDP_WIDE_MMA")


def _run_both(model, e, c, env, monkeypatch):
    import torch

    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ne, nc = e.size, c.size
    with mdp.Engine(model, devices=[0]) as eng:
        eng.set_grid(e, c)
        ec = torch.full((ne, nc + 3), 7.0, dtype=torch.float64, device="cuda")
        eng.run(ec.data_ptr(), nc + 3)
        eng.set_layout("ce")
        ce = torch.full((nc, ne + 5), 7.0, dtype=torch.float64, device="cuda")
        eng.run(ce.data_ptr(), ne + 5)
        torch.cuda.synchronize()
        launched = eng.launched()
    ec, ce = ec.cpu().numpy(), ce.cpu().numpy()
    assert (ec[:, nc:] == 7.0).all() and (ce[:, ne:] == 7.0).all()
    return ec[:, :nc], ce[:, :ne], launched


def _wide_obs(rng, n, T, missing):
    obs = rng.integers(0, 2, size=(T, n))
    for y, k in missing.items():
        obs[y, rng.choice(n, size=k, replace=False)] = -1
    return obs


CASES = {
    "fused": (lambda: mdp.Model.load(str(GOLDEN / "config2_64x50.txt")), 96, 80, {}, "mdp_fwd_jit<fused"),
    "reading": (lambda: mdp.Model.load(str(GOLDEN / "config2_64x50.txt")), 96, 80, {"MDP_FUSED": "0"},
                "mdp_fwd_jit<reading"),
    "chunked": (lambda: mdp.Model.load(str(GOLDEN / "config2_64x50.txt")), 300, 33, {"MDP_JIT_CHUNK": "40"},
                "chunks"),
    "generic": (lambda: mdp.Model.load(str(GOLDEN / "config2_64x50.txt")), 70, 50, {"MDP_JIT": "0"}, "k_forward"),
    "lds_states": (lambda: mdp.Model.from_obs(_wide_obs(np.random.default_rng(3), 12, 5, {1: 6})), 130, 37, {},
                   "mdp_fwd_jit<reading"),
    "wide": (lambda: mdp.Model.from_obs(_wide_obs(np.random.default_rng(3), 12, 5, {1: 6})), 130, 37,
             {"MDP_WIDE": "1"}, "k_fwd_mmt"),
    "wide_mma5": (lambda: mdp.Model.from_obs(_wide_obs(np.random.default_rng(3), 12, 5, {1: 6})), 130, 37,
                  {"MDP_WIDE": "1", "MDP_WIDE_MMA": "1"}, "k_fwd_mma"),
    "wide_big": (lambda: mdp.Model.from_obs(_wide_obs(np.random.default_rng(3), 10, 4, {1: 9})), 70, 37,
                 {}, "k_fwd_hs<1,10>"),
    "wide_big_mmt": (lambda: mdp.Model.from_obs(_wide_obs(np.random.default_rng(3), 10, 4, {1: 9})), 70, 37,
                     {"MDP_WIDE_MMA": "2"}, "k_fwd_mmt<2,512,1buf>"),
    "wide_hs": (lambda: mdp.Model.from_obs(_wide_obs(np.random.default_rng(3), 12, 5, {1: 6})), 130, 37,
                {"MDP_WIDE": "1", "MDP_WIDE_MMA": "3"}, "k_fwd_mmt"),  # 12 variable patches: > 10, k_fwd_mmt
    "wide_plain": (lambda: mdp.Model.from_obs(_wide_obs(np.random.default_rng(3), 12, 5, {1: 6})), 130, 37,
                   {"MDP_WIDE": "1", "MDP_WIDE_MMA": "0"}, "k_fwd_wide"),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_ce_layout_is_ec_transposed(name, monkeypatch):
    make, ne, nc, env, kernel = CASES[name]
    model = make()
    e = np.sort(np.random.default_rng(ne).uniform(0.05, 0.9, ne))
    c = np.sort(np.random.default_rng(nc).uniform(0.01, 0.6, nc))
    ec, ce, launched = _run_both(model, e, c, env, monkeypatch)
    assert any(kernel in k for k in launched), launched
    assert np.array_equal(ec.T, ce, equal_nan=True)
    assert np.isfinite(ec).mean() > 0.5


def test_layout_rejects_short_ld():
    model = mdp.Model.load(str(GOLDEN / "config2_64x50.txt"))
    with mdp.Engine(model, devices=[0]) as eng:
        eng.set_grid(np.linspace(0.1, 0.9, 40), np.linspace(0.1, 0.5, 20))
        eng.set_layout("ce")
        with pytest.raises(mdp.MidaspomError):
            eng.run(1 << 20, 39)  # ld < ne: refused before any launch
        with pytest.raises(KeyError):
            eng.set_layout("xy")


@pytest.mark.parametrize("name", ["fused", "reading", "wide"])
def test_loglik_grid_ignores_engine_layout(name, monkeypatch):
    """mdp_loglik_grid's host result is [e][c] whatever mdp_engine_set_layout
    chose for mdp_engine_run: after set_layout('ce') on a grid with nc > ne
    (where a CE write through loglik_grid's [e][c] slab would also overrun
    it), the result equals a fresh engine's, bit for bit."""
    import torch

    make, _, _, env, _ = CASES[name]
    model = make()
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    e = np.sort(np.random.default_rng(1).uniform(0.05, 0.9, 23))
    c = np.sort(np.random.default_rng(2).uniform(0.01, 0.6, 90))
    with mdp.Engine(model, devices=[0]) as fresh:
        ref = fresh.loglik_grid(e, c)
    with mdp.Engine(model, devices=[0]) as eng:
        eng.set_grid(e, c)
        eng.set_layout("ce")
        out = torch.empty((c.size, e.size), dtype=torch.float64, device="cuda")
        eng.run(out.data_ptr(), e.size)
        got = eng.loglik_grid(e, c)
        torch.cuda.synchronize()
        ce = out.cpu().numpy()
    assert np.array_equal(got, ref, equal_nan=True)
    assert np.array_equal(ce.T, ref, equal_nan=True)
