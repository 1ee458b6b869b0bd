"""Long series: the reference's forward loop has no length limit
(main_MIDASPOM.c:371-384).  A series with more forward uses than one
specialised kernel holds (2 048) runs as chunks of years, the state vector
handed between chunks through an HBM scratch; a Q row past the LDS is staged
per chunk by gathering only the groups the chunk reads; k_qrows tables past
its LDS are built in HBM by k_zrows + k_witems + k_wq.  Every such variant
does the same arithmetic as the single-kernel path, so the outputs must be
identical bit for bit; the long survey itself is checked against the oracle.
Tolerance against the oracle: |dlogL| <= 1e-9 (tests/test_gpu_parity.py)."""
from __future__ import annotations

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle
from midaspom_amd import synth

from test_gpu_parity import assert_loglik_close

pytestmark = pytest.mark.gpu

KNOBS = ("MDP_JIT", "MDP_FUSED", "MDP_WIDE", "MDP_JIT_CHUNK", "MDP_JIT_GATHER", "MDP_QGLOBAL")


def _run(model, e, c, env, monkeypatch):
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with mdp.Engine(model) as eng:
        out = eng.loglik_grid(e, c)
        return out, eng.launched()


# (file, ne, nc, uses per chunk giving 2-4 chunks: each chunk is one hipRTC
# compile of ~1 s, and hipRTC compiles one program at a time)
FILES = [("config2_64x50.txt", 300, 77, 40), ("config3_256x200.txt", 700, 40, 110),
         ("occupancies.txt", 31, 29, 5), ("q1_64x50_mid.txt", 64, 64, 60)]


@pytest.mark.parametrize("fname,ne,nc,chunk", FILES, ids=[f[0] for f in FILES])
@pytest.mark.parametrize("env", [{"MDP_JIT_CHUNK": ""}, {"MDP_JIT_CHUNK": "", "MDP_JIT_GATHER": "1"},
                                 {"MDP_JIT_GATHER": "1"}, {"MDP_QGLOBAL": "1"},
                                 {"MDP_QGLOBAL": "1", "MDP_JIT_CHUNK": ""}],
                         ids=["chunks", "chunks-gather", "gather", "qglobal", "qglobal-chunks"])
def test_chunked_and_global_variants_bitwise(golden, monkeypatch, fname, ne, nc, chunk, env):
    env = {k: (v or str(chunk)) for k, v in env.items()}
    model = mdp.Model.load(golden / fname)
    e, _ = mdp.grid(ne)
    c, _ = mdp.grid(nc, 0.0, 1.2)
    ref, _ = _run(model, e, c, {"MDP_FUSED": "0"}, monkeypatch)
    got, launched = _run(model, e, c, env, monkeypatch)
    if "MDP_JIT_CHUNK" in env:
        assert any("chunks" in k for k in launched), launched
    if "MDP_JIT_GATHER" in env:
        assert any("gather" in k for k in launched), launched
    if "MDP_QGLOBAL" in env:
        assert {"k_zrows", "k_wq"} <= launched and not any(k.startswith("k_qrows") for k in launched), launched
    assert np.array_equal(got, ref, equal_nan=True)


def test_random_problems_chunked(monkeypatch):
    """Random problems with missing data (multi-state years at chunk
    boundaries), two chunkings each, against the one-kernel run."""
    rng = np.random.default_rng(42)
    for trial in range(4):
        n, T, nvar = int(rng.integers(6, 30)), int(rng.integers(5, 12)), int(rng.integers(2, 7))
        obs = synth.random_obs(rng, n, T, nvar, pmiss=0.3, max_missing=3)
        model = mdp.Model.from_obs(obs, m=400.0, p=0.4, d=100.0)
        e, _ = mdp.grid(int(rng.integers(20, 600)))
        c, _ = mdp.grid(int(rng.integers(3, 40)))
        ref, _ = _run(model, e, c, {"MDP_FUSED": "0"}, monkeypatch)
        uses = int((model.npstates[1:] * model.npstates[:-1]).sum())
        for chunk in sorted({max(1, uses // 3), max(1, uses // 2)}):
            chunk = str(chunk)
            got, launched = _run(model, e, c, {"MDP_JIT_CHUNK": chunk, "MDP_JIT_GATHER": str(trial % 2)},
                                 monkeypatch)
            assert np.array_equal(got, ref, equal_nan=True), (trial, chunk)


def test_long_survey_runs_chunked_vs_oracle(tmp_path, monkeypatch):
    """synth.LONG200: 200 years, ~4 states a year, 3 086 uses -- the direct
    path in chunks (not the generic kernels), sampled against the oracle on a
    256 x 256 grid, and equal to the generic path to rounding."""
    f = synth.write(tmp_path / "long.txt", **synth.LONG200)
    model = mdp.Model.load(f)
    nps = model.npstates
    assert int((nps[1:] * nps[:-1]).sum()) > 2048 and nps.max() <= 16
    # the likely region (the series was simulated at e = 0.3, c = 0.1): over
    # most of [0, 1]^2 a 200-year likelihood underflows (quirk Q4)
    ge, _ = mdp.grid(256, 0.1, 0.6)
    gc, _ = mdp.grid(256, 0.01, 0.4)
    got, launched = _run(model, ge, gc, {}, monkeypatch)
    assert any(k.startswith("mdp_fwd_jit<reading") and "chunks" in k for k in launched), launched
    rng = np.random.default_rng(9)
    ie, ic = rng.integers(0, 256, 40), rng.integers(0, 256, 40)
    ie[:4], ic[:4] = [0, 255, 0, 255], [0, 0, 255, 255]
    ref = oracle.OracleModel.load(f).loglik_points(ge[ie], gc[ic], threads=16)
    assert np.isfinite(ref).sum() >= 30
    assert_loglik_close(got[ie, ic], ref)
    gen, launched = _run(model, ge, gc, {"MDP_JIT": "0"}, monkeypatch)
    assert any(k.startswith("k_forward") for k in launched)
    assert_loglik_close(got, gen, atol=1e-10)
