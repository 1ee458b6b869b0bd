"""Downstream consumers of the output files.

The reference post-processes its outputs with R scripts (R is not installed
here).  This module restates their numerical parts -- no plotting -- so the
files this engine writes can be checked to load and summarise exactly as the
reference's pipeline expects:

    posterior_summary   Rscript/plot_posterior.R:14-37
    dieoff_summary      Rscript/plot_posterior_dieoff.R:14-26
    loss_summary        Rscript/plot_posterior_loss.R:14-29
    hypothesis_test     Rscript/hypothesis_test.R:13-46
    extinction_curve    Rscript/plot_extinction.R:13-22

R semantics kept: read.table / scan split on any whitespace (the trailing
tab of every row is harmless), which.max returns the first maximum in
column-major order, seq(l, u, length.out = n) is l + i (u - l) / (n - 1).
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np

__all__ = ["read_table", "scan", "r_seq", "posterior_summary", "dieoff_summary", "loss_summary",
           "hypothesis_test", "extinction_curve"]


def read_table(path) -> np.ndarray:
    """as.matrix(read.table(path)): one row per line, fields split on whitespace."""
    rows = [ln.split() for ln in Path(path).read_text().splitlines() if ln.strip()]
    if not rows:
        raise ValueError(f"{path}: empty table")
    widths = {len(r) for r in rows}
    if len(widths) != 1:
        raise ValueError(f"{path}: ragged rows {sorted(widths)}")
    return np.array([[float(x) for x in r] for r in rows], dtype=np.float64)


def scan(path) -> np.ndarray:
    """scan(path): every whitespace-separated number, in file order."""
    return np.array([float(x) for x in Path(path).read_text().split()], dtype=np.float64)


def r_seq(lo: float, hi: float, n: int) -> np.ndarray:
    """seq(lo, hi, length.out = n)."""
    if n == 1:
        return np.array([lo], dtype=np.float64)
    return lo + np.arange(n, dtype=np.float64) * ((hi - lo) / (n - 1))


def _which_max_colmajor(a: np.ndarray) -> int:
    """R's which.max on a matrix: 1-based index of the first maximum in
    column-major order (NaN entries are skipped, as R does)."""
    flat = a.flatten(order="F")
    ok = ~np.isnan(flat)
    if not ok.any():
        raise ValueError("which.max of an all-NaN matrix")
    idx = np.flatnonzero(ok)
    return int(idx[np.argmax(flat[ok])]) + 1


def posterior_summary(postfile, lo: float = 0.0, hi: float = 1.0, step: int | None = None) -> dict:
    """plot_posterior.R: normalised joint density, point estimates (the grid
    mode), marginal densities and the 95 % central interval indices."""
    jpost = read_table(postfile)
    if step is None:
        step = jpost.shape[0]
    if jpost.shape != (step, step):
        raise ValueError(f"posterior is {jpost.shape}, expected {step}x{step}")
    el = r_seq(lo, hi, step)
    cl = r_seq(lo, hi, step)
    jpost = jpost / jpost.sum() / 0.01 / 0.01
    ml = _which_max_colmajor(jpost)
    eest = el[(ml - 1) % step]
    cest = cl[(ml - 1) // step]
    epost = jpost.mean(axis=1)  # rowMeans
    cpost = jpost.mean(axis=0)  # colMeans
    ce, cc = np.cumsum(epost), np.cumsum(cpost)
    qel = np.flatnonzero((ce >= 0.025 / 0.01) & (ce < 0.975 / 0.01)) + 1  # R 1-based indices
    qcl = np.flatnonzero((cc >= 0.025 / 0.01) & (cc < 0.975 / 0.01)) + 1
    return {"jpost": jpost, "eest": float(eest), "cest": float(cest), "epost": epost, "cpost": cpost,
            "qel": qel, "qcl": qcl, "el": el, "cl": cl}


def dieoff_summary(postfile, kmin: float, kmax: float, step_k: int) -> dict:
    """plot_posterior_dieoff.R: posterior density over log10 K_D and the
    first K_D whose density reaches 95 % of the maximum."""
    post = scan(postfile)
    if post.size != step_k:
        raise ValueError(f"{post.size} values, expected {step_k}")
    kl = 10.0 ** r_seq(math.log10(kmin), math.log10(kmax), step_k)
    post_k = post / post.sum() / (math.log10(kmax) - math.log10(kmin)) * (step_k - 1)
    kd = kl[post_k >= 0.95 * post_k.max()]
    return {"postK": post_k, "Kl": kl, "Kdest": float(kd[0]) if kd.size else float("nan")}


def loss_summary(postfile, kmin: float, kmax: float, dmin: float, dmax: float, step_k: int,
                 step_d: int) -> dict:
    """plot_posterior_loss.R: matrix(scan(file), stepK, stepd, byrow = T)
    and the 95 %-of-maximum point estimates of d_L and K_L."""
    v = scan(postfile)
    if v.size != step_k * step_d:
        raise ValueError(f"{v.size} values, expected {step_k}x{step_d}")
    j = v.reshape(step_k, step_d)
    kl = 10.0 ** r_seq(math.log10(kmin), math.log10(kmax), step_k)
    dl = r_seq(dmin, dmax, step_d)
    cs, rs = j.sum(axis=0), j.sum(axis=1)
    dlest = dl[cs >= 0.95 * cs.max()]
    klest = kl[rs >= 0.95 * rs.max()]
    return {"jpostloss": j, "dlest": float(dlest[0]) if dlest.size else float("nan"),
            "Klest": float(klest[0]) if klest.size else float("nan")}


def hypothesis_test(dieoff_file, loss_file, n: int, kmin: float, kmax: float) -> dict:
    """hypothesis_test.R: AIC of H0 (no event), H1 (die-off), H2 (habitat
    loss) and the log10 Bayes factors, with the script's own normalisations
    (lK01 divides by the loss table's row count, :43)."""
    postdieoff = scan(dieoff_file)
    jpostloss = read_table(loss_file)
    step_kl, step_d = jpostloss.shape
    step_kd = postdieoff.size
    kdl = 10.0 ** r_seq(math.log10(kmin), math.log10(kmax), step_kd)
    if np.any(kdl == 1.0):
        postnull = float(postdieoff[np.flatnonzero(kdl == 1.0)[0]])
    else:
        idn = int(np.flatnonzero(kdl > 1.0)[0])
        postnull = float((postdieoff[idn] - postdieoff[idn - 1]) / (kdl[idn] - kdl[idn - 1]) * (1 - kdl[idn - 1])
                         + postdieoff[idn - 1])
    two_n = 2.0 ** n
    return {
        "postnull": postnull,
        "AIC0": 2 * 1 - 2 * math.log(postnull / two_n),
        "AIC1": 2 * 2 - 2 * math.log(float(postdieoff.max()) / two_n),
        "AIC2": 2 * 3 - 2 * math.log(float(jpostloss.max()) / two_n),
        "lK01": math.log10(postnull / (float(postdieoff.sum()) / step_kl)),
        "lK02": math.log10(postnull / (float(jpostloss.sum()) / step_kl / step_d)),
        "lK12": math.log10(float(postdieoff.sum()) / (float(jpostloss.sum()) / step_d)),
    }


def extinction_curve(prext_file, tmax: int, nrep: int) -> np.ndarray:
    """plot_extinction.R: per-year extinction probability pext / nrep."""
    pext = scan(prext_file)
    if pext.size != tmax:
        raise ValueError(f"{pext.size} years, expected {tmax}")
    return pext / nrep
