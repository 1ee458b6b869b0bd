"""Pin the scenario oracle (oracle/spom_dieoff_oracle.c, a CPU restatement of
main_MIDASPOM_dieoff.c / main_MIDASPOM_loss.c) to the manual's worked
examples (Manual_linux.pdf p.4 and p.5, tests/golden/anchors.json), and check
the product's host-side grids against the reference formulas."""
from __future__ import annotations

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle


def test_first_row_matches_reference_reader(golden):
    row = oracle.first_row(golden / "manual_p3_obs.txt")
    assert row.tolist() == [0, 1, 1, 1, 1]
    assert np.array_equal(mdp.first_row(golden / "manual_p3_obs.txt"), row)
    # examples/input: 8 tokens on line 1 (Q6 re-flow does not matter here)
    assert mdp.first_row(golden / "occupancies.txt").size == 8


def test_grids_match_oracle():
    assert np.array_equal(mdp.kgrid(151), oracle.kgrid(151))
    assert np.array_equal(mdp.kgrid(11, 0.5, 20.0), oracle.kgrid(11, 0.5, 20.0))
    d = mdp.dgrid(20)
    assert d[0] == 200.0 and d[-1] == 4000.0 and np.allclose(np.diff(d), 200.0)


def test_oracle_dieoff_manual_p4(golden, anchors):
    a = anchors["manual_dieoff_p4"]
    f = a["flags"]
    row = oracle.first_row(golden / a["input"])
    L = oracle.dieoff_lik(row, oracle.kgrid(f["s"]), f["e"], f["c"], ts=20, tdis=f["a"], m=f["m"], d=f["d"])
    assert np.array_equal(np.round(L, 6), np.array(a["values_6dp"]))


def test_oracle_loss_manual_p5(golden, anchors):
    a = anchors["manual_loss_p5"]
    f = a["flags"]
    row = oracle.first_row(golden / a["input"])
    L = oracle.loss_lik(row, oracle.kgrid(f["s"]), mdp.dgrid(f["v"]), f["e"], f["c"], ts=20, tdis=f["a"],
                        m=f["m"], d=f["d"])
    assert np.array_equal(np.round(L, 6), np.array(a["values_6dp"]))


def test_vector_oracle_matches_dense_oracle():
    """orc_scenario_vec (vector propagation, the checker for n > 12 where the
    dense products are out of reach) against the dense restatement on random
    rows, both scenarios, ts / tdis including 0."""
    rng = np.random.default_rng(11)
    for trial in range(10):
        n = int(rng.integers(1, 9))
        row = rng.choice(np.array([-1, 0, 1], dtype=np.int32), size=n, p=[0.2, 0.3, 0.5]).astype(np.int32)
        ts, tdis = int(rng.integers(0, 6)), int(rng.integers(0, 4))
        e, c = float(rng.uniform(0, 1.2)), float(rng.uniform(0, 1.5))
        K = float(rng.choice([0.3, 1.0, 7.0]))
        m, d, p = float(rng.choice([100, 400])), float(rng.choice([50, 200])), float(rng.choice([0.5, 0.3]))
        dense = oracle.dieoff_lik(row, np.array([K]), e, c, ts=ts, tdis=tdis, m=m, p=p, d=d)[0]
        vec = oracle.scenario_vec(row, "dieoff", K, e, c, ts=ts, tdis=tdis, m=m, p=p, d=d)
        assert vec == pytest.approx(dense, rel=1e-12, abs=1e-300), (trial, n)
        ds = float(rng.choice([100.0, 800.0]))
        dense = oracle.loss_lik(row, np.array([K]), np.array([ds]), e, c, ts=ts, tdis=tdis, m=m, p=p, d=d)[0, 0]
        vec = oracle.scenario_vec(row, "loss", K, e, c, ts=ts, tdis=tdis, m=m, p=p, d=d, dsrc=ds)
        assert vec == pytest.approx(dense, rel=1e-12, abs=1e-300), (trial, n)
