"""Every kernel-variant engine option the default library accepts
(mdp_engine_create_opts, include/midaspom.h) run against the
oracle on the GPU.

Options select among kernel variants that must give the reference's results
(main_MIDASPOM.c:341-395); a variant no test runs is not shipped.
tests/test_engine_options.py checks on the CPU that every name the library
accepts appears in this file's VARIANTS (or, for the tooling options that
select no kernel, in TOOLING) -- so adding an option without a parity case
fails the CPU suite.
"""
from __future__ import annotations

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle
from midaspom_amd import synth

from test_gpu_parity import assert_loglik_close

pytestmark = pytest.mark.gpu

# (option string, problem): "cfg1" = the shipped example (8 variable patches,
# fused kernel), "cfg2" = the config-2 input on a 40 x 37 grid, "wide45" =
# the 45 %-unvisited series (years of up to 64 states: the LDS-state kernel),
# "tall" = config 2 on a 700 x 33 grid (several e blocks a column: k_qrows +
# the reading kernel)
VARIANTS = [
    ("MDP_FUSED=1", "cfg2"),
    ("MDP_FUSED=0", "cfg2"),
    ("MDP_FUSED_COLS=1", "cfg2"),
    ("MDP_FUSED_COLS=3", "cfg1"),
    ("MDP_FUSED_COLS=4", "cfg2"),
    ("MDP_EPL=1", "tall"),
    ("MDP_EPL=4", "tall"),
    ("MDP_EPL=1;MDP_JIT_KBLOCK=512", "cfg2"),
    ("MDP_JIT_KBLOCK=512", "tall"),
    ("MDP_JIT_SLOTS=0", "cfg2"),
    ("MDP_JIT_SLOTS=16", "tall"),
    ("MDP_JIT_WINDOW=4", "cfg2"),
    ("MDP_JIT_WINDOW=16", "tall"),
    ("MDP_JIT_XCD=0", "tall"),
    ("MDP_JIT_EFAST=0", "tall"),
    ("MDP_QROWS_XCD=0", "tall"),
    ("MDP_JIT_SPLIT=0", "cfg2"),
    ("MDP_JIT_ROT=0", "cfg2"),
    ("MDP_FAST_LOG=0", "cfg1"),
    ("MDP_JIT=0", "cfg2"),
    ("MDP_JIT=0;MDP_FWD=scalar", "cfg1"),
    ("MDP_JIT_CHUNK=64", "cfg2"),
    ("MDP_JIT_GATHER=1", "cfg2"),
    ("MDP_QGLOBAL=1", "tall"),
    ("MDP_WIDE=1", "cfg1"),
    ("MDP_WIDE=1;MDP_WIDE_CB=3", "cfg1"),
    ("MDP_WIDE=1;MDP_WIDE_MMA=0", "cfg2"),
    ("MDP_VSPLIT=1", "wide45"),
    ("MDP_VSPLIT=2", "wide45"),
    ("MDP_VLDS_EPL=2", "wide45"),
    ("MDP_VLDS_MAXUSES=100", "wide45"),  # past it: the wide kernels take the problem
    ("MDP_WIDE=1;MDP_WIDE_MMA=3;MDP_HS_RADIX=1", "wide45"),
    ("MDP_WIDE=1;MDP_WIDE_MMA=3;MDP_HS_RADIX=2", "wide45"),
    ("MDP_WIDE=1;MDP_WIDE_MMA=3;MDP_HS_RADIX=4", "wide45"),
    ("MDP_WIDE=1;MDP_WIDE_MMA=3;MDP_HS_WAVES=8", "wide45"),
    ("MDP_WIDE=1;MDP_WIDE_MMA=3;MDP_HS_WAVES=16", "wide45"),
]
# options that select no kernel: compile-time diagnostics and host threads
TOOLING = ["MDP_JIT_CHECK", "MDP_JIT_DUMP", "MDP_JIT_THREADS", "MDP_JIT_VERBOSE"]


def _problem(name, golden, tmp_path):
    if name == "cfg1":
        f, e, c = golden / "occupancies.txt", mdp.grid(17)[0], mdp.grid(19)[0]
    elif name == "cfg2":
        f, e, c = golden / "config2_64x50.txt", mdp.grid(40)[0], mdp.grid(37, 0.0, 1.3)[0]
    elif name == "tall":
        f, e, c = golden / "config2_64x50.txt", mdp.grid(700)[0], mdp.grid(33)[0]
    else:
        f = synth.write(tmp_path / "wide45.txt", **dict(synth.CONFIG2, pmiss=0.45, seed=5, T=12))
        e, c = mdp.grid(70)[0], mdp.grid(9)[0]
    return f, e, c


@pytest.mark.parametrize("opts,prob", VARIANTS, ids=[f"{o}-{p}" for o, p in VARIANTS])
def test_option_variant_matches_oracle(golden, tmp_path, opts, prob):
    f, e, c = _problem(prob, golden, tmp_path)
    model = mdp.Model.load(f)
    with mdp.Engine(model, options=opts) as eng:
        got = eng.loglik_grid(e, c)
    om = oracle.OracleModel.load(f)
    if e.size * c.size <= 2000:
        ref = om.loglik_grid(e, c, threads=16)
        assert_loglik_close(got, ref)
    else:  # sampled points (corners included)
        rng = np.random.default_rng(11)
        ie, ic = rng.integers(0, e.size, 48), rng.integers(0, c.size, 48)
        ie[:4], ic[:4] = [0, e.size - 1, 0, e.size - 1], [0, 0, c.size - 1, c.size - 1]
        assert_loglik_close(got[ie, ic], om.loglik_points(e[ie], c[ic], threads=16))


def test_tooling_options_change_no_result(golden, tmp_path):
    f = golden / "config2_64x50.txt"
    e, c = mdp.grid(24)[0], mdp.grid(21)[0]
    model = mdp.Model.load(f)
    with mdp.Engine(model) as eng:
        a = eng.loglik_grid(e, c)
    dump = tmp_path / "src"
    with mdp.Engine(model, options=f"MDP_JIT_DUMP={dump};MDP_JIT_THREADS=1;MDP_JIT_VERBOSE=1") as eng:
        b = eng.loglik_grid(e, c)
    assert np.array_equal(a, b)
    assert list(tmp_path.glob("src*.hip")), "MDP_JIT_DUMP wrote no source"
