"""Pin the scenario oracle (oracle/spom_dieoff_oracle.c, a CPU restatement of
main_MIDASPOM_dieoff.c / main_MIDASPOM_loss.c) to the manual's worked
examples (Manual_linux.pdf p.4 and p.5, tests/golden/anchors.json), and check
the product's host-side grids against the reference formulas."""
from __future__ import annotations

import numpy as np

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
