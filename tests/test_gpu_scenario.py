"""GPU parity of the scenario engine (die-off / habitat loss, mdp_scenario_*)
against the CPU oracle and the manual's worked examples.

Tolerance: the engine propagates vectors instead of forming matrix powers
(DESIGN.md §11), so it reorders all-positive sums: relative 1e-9 where
L > 1e-14, absolute 1e-20 below (the %.20lf print floor of the reference's
output is ~1e-20)."""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import midaspom_amd as mdp
import oracle
from midaspom_amd import _lib

pytestmark = pytest.mark.gpu


def close(got, ref, rtol=1e-9):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape
    big = ref > 1e-14
    if big.any():
        rel = np.abs(got[big] - ref[big]) / ref[big]
        assert rel.max() <= rtol, f"max rel {rel.max():.3e}"
    assert np.abs(got[~big] - ref[~big]).max(initial=0.0) <= 1e-20


def test_dieoff_manual_p4(golden, anchors):
    a = anchors["manual_dieoff_p4"]
    f = a["flags"]
    row = mdp.first_row(golden / a["input"])
    with mdp.Scenario(row, "dieoff", m=f["m"], d=f["d"]) as sc:
        L = sc.lik(f["e"], f["c"], mdp.kgrid(f["s"]), ts=20, tdis=f["a"])[0, 0]
    assert np.array_equal(np.round(L, 6), np.array(a["values_6dp"]))


def test_loss_manual_p5(golden, anchors):
    a = anchors["manual_loss_p5"]
    f = a["flags"]
    row = mdp.first_row(golden / a["input"])
    with mdp.Scenario(row, "loss", m=f["m"], d=f["d"]) as sc:
        L = sc.lik(f["e"], f["c"], mdp.kgrid(f["s"]), mdp.dgrid(f["v"]), ts=20, tdis=f["a"])[0, 0]
    assert np.array_equal(np.round(L, 6), np.array(a["values_6dp"]))


@pytest.mark.parametrize("kind", ["dieoff", "loss"])
def test_examples_input_grid_vs_oracle(golden, kind):
    """n = 8 (256 states): a small (e, c, K[, d]) grid against the oracle."""
    row = mdp.first_row(golden / "occupancies.txt")
    e, c = np.array([0.05, 0.3, 0.9, 1.4]), np.array([0.1, 0.6, 2.0])
    K = mdp.kgrid(5)
    d = mdp.dgrid(3)
    with mdp.Scenario(row, kind, m=400, d=100) as sc:
        got = sc.lik(e, c, K, d, ts=7, tdis=4)
    for ie, ev in enumerate(e):
        for ic, cv in enumerate(c):
            if kind == "dieoff":
                ref = oracle.dieoff_lik(row, K, ev, cv, ts=7, tdis=4, m=400, d=100)
            else:
                ref = oracle.loss_lik(row, K, d, ev, cv, ts=7, tdis=4, m=400, d=100)
            close(got[ie, ic], ref)


@pytest.mark.parametrize("kernel", ["lds", "big", "row"])
@pytest.mark.parametrize("seed", range(int(os.environ.get("MDP_FUZZ_SCN", "8"))))  # more: a longer fuzz
def test_random_rows(seed, kernel, monkeypatch):
    """Random first rows (n <= 8, missing patches), rates, K / source grids,
    ts and tdis (0 included) and e counts across the 32-value e chunks, on
    the LDS kernel, k_scn_big (MDP_SCN_BIG=1) and k_scn_row (MDP_SCN_ROW=1),
    against the oracle."""
    monkeypatch.setenv("MDP_SCN_BIG", "1" if kernel == "big" else "0")
    monkeypatch.setenv("MDP_SCN_ROW", "1" if kernel == "row" else "0")
    rng = np.random.default_rng(500 + seed)
    n = int(rng.integers(1, 9))
    row = rng.choice([-1, 0, 1], size=n, p=[0.2, 0.4, 0.4]).astype(np.int32)
    kind = "loss" if seed % 2 else "dieoff"
    e = rng.uniform(0.0, 1.2, int(rng.choice([1, 3, 33, 70])))
    c = rng.uniform(0.0, 1.5, 2)
    K = mdp.kgrid(4, 0.2, 30.0)
    d = np.array([150.0, 900.0])
    ts, tdis = int(rng.integers(0, 6)), int(rng.integers(0, 6))
    m, dd, p = float(rng.choice([100, 400])), float(rng.choice([50, 200])), float(rng.choice([0.5, 0.3]))
    with mdp.Scenario(row, kind, m=m, p=p, d=dd) as sc:
        got = sc.lik(e, c, K, d, ts=ts, tdis=tdis)
    for ie in sorted({0, e.size - 1, int(rng.integers(0, e.size))}):
        for ic in range(c.size):
            if kind == "dieoff":
                ref = oracle.dieoff_lik(row, K, e[ie], c[ic], ts=ts, tdis=tdis, m=m, p=p, d=dd)
            else:
                ref = oracle.loss_lik(row, K, d, e[ie], c[ic], ts=ts, tdis=tdis, m=m, p=p, d=dd)
            close(got[ie, ic], ref)


def test_too_many_patches_fails_loudly():
    # 2^17 states per grid point: past the engine's n <= 16
    with pytest.raises(mdp.MidaspomError, match="UNSUPPORTED"):
        mdp.Scenario(np.zeros(17, dtype=np.int32), "dieoff")


def test_dieoff_cli_output_layout(golden, anchors, tmp_path):
    a = anchors["manual_dieoff_p4"]
    out = tmp_path / "lh.txt"
    r = subprocess.run([str(_lib.DIEOFF_CLI_PATH), "-a", "10", "-e", "0.5", "-c", "0.5", "-m", "400", "-d", "200",
                        "-s", "11", "-i", str(golden / a["input"]), "-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "------ MIDASPOM, in situ die-off hypothesis, beta version -------"
    assert "20 years before increased die-off, 10 years after increased die-off" in lines
    assert "5 patches" in lines and "Starting likelihood computation" in lines
    txt = out.read_text()
    assert "\n" not in txt and txt.endswith("\t")
    vals = [float(x) for x in txt.split("\t") if x]
    assert np.array_equal(np.round(vals, 6), np.array(a["values_6dp"]))


def test_loss_cli_output_layout(golden, anchors, tmp_path):
    a = anchors["manual_loss_p5"]
    out = tmp_path / "lh.txt"
    r = subprocess.run([str(_lib.LOSS_CLI_PATH), "-a", "10", "-e", "0.5", "-c", "0.5", "-m", "400", "-d", "200",
                        "-s", "11", "-v", "4", "-i", str(golden / a["input"]), "-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "First occupancy survey:" in r.stdout
    rows = [[float(x) for x in ln.split("\t") if x] for ln in out.read_text().splitlines()]
    assert np.array_equal(np.round(rows, 6), np.array(a["values_6dp"]))


def test_cli_requires_event_flags(golden, tmp_path):
    r = subprocess.run([str(_lib.DIEOFF_CLI_PATH), "-i", str(golden / "manual_p3_obs.txt")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "required" in r.stderr


@pytest.mark.parametrize("kind", ["dieoff", "loss"])
def test_device_resident_run_matches_host(golden, kind):
    import torch
    row = mdp.first_row(golden / "occupancies.txt")
    e, c = np.linspace(0.05, 0.95, 19), np.array([0.1, 0.6, 2.0])
    K, d = mdp.kgrid(6), mdp.dgrid(3)
    with mdp.Scenario(row, kind, m=400, d=100) as sc:
        host = sc.lik(e, c, K, d, ts=5, tdis=3)
        shape = sc.set_grid(e, c, K, d, ts=5, tdis=3)
        out = torch.empty(shape, dtype=torch.float64, device="cuda:0")
        sc.run(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), host)
        ms = sc.time_kernels(out.data_ptr(), torch.cuda.current_stream().cuda_stream, reps=2)
        assert ms["k_scn_v"] > 0 and ms["k_scn_lik"] > 0
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), host)


def test_config4_full_workload(golden):
    """BASELINE config 4 at its workload: examples/input row 1 (n = 8), e and c
    = grid(256) on [0, 1], K = kgrid(256, 0.1, 100), ts = 20, tdis = 10 --
    the call bench.py --config 4 times (main_MIDASPOM_dieoff.c:307-351 for
    every (e, c, K)).  All 256^3 values finite and >= 0; the 8 (e, c, K)
    corners and 64 random (e, c) pairs x 8 K each against the oracle (one
    oracle call per (e, c), so its P^tdis is shared by the K values; the
    calls run on a thread pool -- the C oracle releases the GIL)."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    import torch
    s, ts, tdis = 256, 20, 10
    row = mdp.first_row(golden / "occupancies.txt")
    g, _ = mdp.grid(s, 0.0, 1.0)
    K = mdp.kgrid(s, 0.1, 100.0)
    with mdp.Scenario(row, "dieoff", m=400.0, d=100.0) as sc:
        shape = sc.set_grid(g, g, K, ts=ts, tdis=tdis)
        assert shape == (s, s, s)
        out = torch.empty(shape, dtype=torch.float64, device="cuda:0")
        sc.run(out.data_ptr())
        lik = out.cpu().numpy()  # ordered after the kernel: both on the null stream
    assert np.isfinite(lik).all() and (lik >= 0).all()
    rng = np.random.default_rng(4)
    jobs = [(ie, ic, np.array([0, s - 1])) for ie in (0, s - 1) for ic in (0, s - 1)]
    for ie, ic in zip(rng.integers(0, s, 64), rng.integers(0, s, 64)):
        jobs.append((int(ie), int(ic), np.sort(rng.choice(s, size=8, replace=False))))

    def ref(job):
        ie, ic, iK = job
        return oracle.dieoff_lik(row, K[iK], g[ie], g[ic], ts=ts, tdis=tdis, m=400.0, d=100.0)

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        refs = list(ex.map(ref, jobs))
    got = np.concatenate([lik[ie, ic, iK] for ie, ic, iK in jobs])
    close(got, np.concatenate(refs))


# ---------------------------------------------------------------------------
# n > 8 patches: k_scn_big (state vectors in HBM); dieoff.c:238 and loss.c:222
# build 2^n states for whatever the first survey row holds
# ---------------------------------------------------------------------------
ROW12 = np.array([1, 0, 1, -1, 0, 1, 1, 0, -1, 1, 0, 1], dtype=np.int32)


@pytest.mark.parametrize("kind", ["dieoff", "loss"])
@pytest.mark.parametrize("row", [ROW12[:3], ROW12[:6], mdp.first_row(Path(__file__).parent / "golden" / "occupancies.txt")],
                         ids=["n3", "n6", "n8"])
def test_big_kernel_matches_lds_kernel(monkeypatch, kind, row):
    """The general kernels forced onto n <= 8 (k_scn_big: MDP_SCN_BIG=1;
    k_scn_row: MDP_SCN_ROW=1) agree with the LDS kernel."""
    e, c = np.array([0.05, 0.4, 0.9, 1.3]), np.array([0.1, 0.7, 2.0])
    K, d = mdp.kgrid(4), mdp.dgrid(2)
    out = []
    for big, rowk in (("0", "0"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("MDP_SCN_BIG", big)
        monkeypatch.setenv("MDP_SCN_ROW", rowk)
        with mdp.Scenario(row, kind, m=400, d=100) as sc:
            out.append(sc.lik(e, c, K, d, ts=6, tdis=4))
    close(out[1], out[0], rtol=1e-12)
    close(out[2], out[0], rtol=1e-12)


@pytest.mark.parametrize("kind", ["dieoff", "loss"])
@pytest.mark.parametrize("n", [9, 10, 12])
def test_row_kernel_matches_big_kernel(monkeypatch, kind, n):
    """For 8 < n <= 12 the default is k_scn_row (one workgroup per point,
    threads over rows, states in LDS); it runs k_scn_big's contraction and
    operator order, so the two agree to rounding of the final sum, on a grid
    with 1 to 33 e values (ts = 0 and tdis = 0 included)."""
    rng = np.random.default_rng(n)
    row = rng.choice([-1, 0, 1], size=n, p=[0.2, 0.4, 0.4]).astype(np.int32)
    for ne, ts, tdis in ((1, 3, 2), (33, 0, 2), (5, 4, 0)):
        e, c = rng.uniform(0.0, 1.2, ne), np.array([0.15, 0.8])
        K, d = mdp.kgrid(3, 0.2, 30.0), mdp.dgrid(2)
        out = []
        for big in ("0", "1"):
            monkeypatch.setenv("MDP_SCN_BIG", big)
            with mdp.Scenario(row, kind, m=400, d=100) as sc:
                out.append(sc.lik(e, c, K, d, ts=ts, tdis=tdis))
        close(out[0], out[1], rtol=1e-12)


@pytest.mark.parametrize("kind", ["dieoff", "loss"])
@pytest.mark.parametrize("n", [9, 10])
def test_scenario_more_than_8_patches_vs_oracle(kind, n):
    import os
    from concurrent.futures import ThreadPoolExecutor
    row = ROW12[:n]
    e, c = np.array([0.1, 0.45, 0.8]), np.array([0.15, 0.6])
    K, d = np.array([0.3, 1.0, 7.5]), np.array([250.0, 900.0])
    with mdp.Scenario(row, kind, m=400, d=100) as sc:
        got = sc.lik(e, c, K, d, ts=20, tdis=10)
    assert np.isfinite(got).all() and (got >= 0).all()
    jobs = [(ie, ic) for ie in range(e.size) for ic in range(c.size)]

    def ref(job):
        ie, ic = job
        if kind == "dieoff":
            return oracle.dieoff_lik(row, K, e[ie], c[ic], ts=20, tdis=10, m=400.0, d=100.0)
        return oracle.loss_lik(row, K, d, e[ie], c[ic], ts=20, tdis=10, m=400.0, d=100.0)

    with ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        refs = list(ex.map(ref, jobs))
    for (ie, ic), r in zip(jobs, refs):
        close(got[ie, ic], r)


def test_scenario_12_patches_vs_oracle():
    """n = 12 (4096 states) against the oracle's dense 4096^2 form, one K, a
    one-year event (the oracle's dgemms dominate the test)."""
    row = ROW12
    with mdp.Scenario(row, "dieoff", m=400, d=100) as sc:
        got = sc.lik(np.array([0.3]), np.array([0.4]), np.array([0.5, 3.0]), ts=1, tdis=1)[0, 0]
        full = sc.lik(np.array([0.3, 0.6]), np.array([0.4]), mdp.kgrid(5), ts=20, tdis=10)
    ref = oracle.dieoff_lik(row, np.array([0.5]), 0.3, 0.4, ts=1, tdis=1, m=400.0, d=100.0)
    close(got[:1], ref)
    assert np.isfinite(full).all() and (full >= 0).all()


def test_scenario_13_patches_split_invariance():
    """n = 13 (8192 states, beyond any oracle run here): at K_D = 1 the
    die-off operator before the event equals the one after it, so
    L(ts = a, tdis = b) = L(ts = a + b, tdis = 0) for every split -- a
    property of the reference's formulation (dieoff.c:304-351) that holds
    at any n."""
    row = np.array([1, 0, 1, -1, 0, 1, 1, 0, -1, 1, 0, 1, 1], dtype=np.int32)
    e, c, K = np.array([0.2, 0.55]), np.array([0.35]), np.array([1.0])
    with mdp.Scenario(row, "dieoff", m=400, d=100) as sc:
        a = sc.lik(e, c, K, ts=4, tdis=2)
        b = sc.lik(e, c, K, ts=6, tdis=0)
        d = sc.lik(e, c, K, ts=1, tdis=5)
    assert np.isfinite(a).all() and (a > 0).all()
    close(a, b, rtol=1e-12)
    close(d, b, rtol=1e-12)


@pytest.mark.parametrize("kind,n,npts", [("dieoff", 13, 8), ("loss", 13, 8), ("dieoff", 14, 4), ("loss", 14, 4),
                                          ("dieoff", 16, 2)])
def test_scenario_13_to_16_patches_vs_vector_oracle(kind, n, npts):
    """n = 13..16 (k_scn_big, the default past 12 patches) against the
    oracle's vector-propagation form (orc_scenario_vec: the reference's
    matrix entries, products associated right to left) at sampled
    (e, c, K[, d]) points with a multi-year event."""
    from concurrent.futures import ThreadPoolExecutor
    rng = np.random.default_rng(n)
    row = rng.choice(np.array([-1, 0, 1], dtype=np.int32), size=n, p=[0.1, 0.35, 0.55]).astype(np.int32)
    row[0] = 1
    e, c, K = np.array([0.15, 0.5]), np.array([0.3, 0.8]), np.array([0.5, 4.0])
    ts, tdis = 3, 2
    ds = mdp.dgrid(2)
    with mdp.Scenario(row, kind, m=400, d=100) as sc:
        got = sc.lik(e, c, K, ts=ts, tdis=tdis, **({"dsrc": ds} if kind == "loss" else {}))
    pts = [(ie, ic, iK, idd) for ie in range(2) for ic in range(2) for iK in range(2)
           for idd in range(2 if kind == "loss" else 1)]
    pts = [pts[i] for i in rng.choice(len(pts), size=npts, replace=False)]

    def ref(pt):
        ie, ic, iK, idd = pt
        return oracle.scenario_vec(row, kind, K[iK], e[ie], c[ic], ts=ts, tdis=tdis, m=400.0, d=100.0,
                                   dsrc=float(ds[idd]))
    with ThreadPoolExecutor(max_workers=8) as ex:
        refs = list(ex.map(ref, pts))
    for pt, r in zip(pts, refs):
        g = got[pt] if kind == "loss" else got[pt[:3]]
        close(np.array([g]), np.array([r]))
