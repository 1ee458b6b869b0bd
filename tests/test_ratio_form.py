"""The forward kernels' ratio forms (csrc/spom_jit.cpp), restated
in Python and checked on the CPU against the direct evaluation
P = sum_m Q[m] x^(|A|-m) y^m of the reference's transition
(main_MIDASPOM.c:18-50, :363-384): per-lane t-form (x >= y) / s-form,
Horner chains over stored or reversed coefficients, g^(|A|-nX) per
transition, the source factor B^|A| deferred as a pending exponent with
per-year source pre-scaling and flushes.  This pins the algebra (including
flushes, e = 0, e >= 1 and e < 0) independently of the generated kernels,
which the GPU parity tests check against the oracle."""
from __future__ import annotations

import numpy as np
import pytest

import midaspom_amd as mdp

FLUSH = 192  # spom_jit.cpp kFlushExp


def _problem(model):
    v = model._view
    n, nvar = model.n, model.nvar
    off = model.year_off
    yid = np.ctypeslib.as_array(v.year_ids, shape=(int(off[-1]),))
    M = np.ctypeslib.as_array(v.M, shape=(n, n))
    varc = np.ctypeslib.as_array(v.var_cols, shape=(nvar,))
    return n, nvar, off, yid, model.short_state, M, varc, float(model.prior[0])


def _pc_fn(model, c):
    """Pc[j][B](c) of the reference (main_MIDASPOM.c:18-50), memoised per j."""
    n, nvar, off, yid, ss, M, varc, _ = _problem(model)
    isvar = np.zeros(n, bool)
    isvar[varc] = True
    col_bit = {int(varc[b]): nvar - 1 - b for b in range(nvar)}
    S = {}
    Q = {}

    def pc(j, B):
        if j not in S:
            s = np.zeros(n)
            for b in range(nvar):
                if (j >> (nvar - 1 - b)) & 1:
                    t = M[varc[b]].copy()
                    t[varc[b]] = 0.0
                    s += t
            S[j] = s
        p = np.minimum(1.0, c * S[j])
        f = 1.0
        for k in range(n):
            if isvar[k]:
                bit = col_bit[k]
                if (j >> bit) & 1:
                    continue
                f *= p[k] if (B >> bit) & 1 else 1.0 - p[k]
            else:
                f *= 1.0 - p[k]
        return f

    return pc


def _q_table(model, c):
    """Q_ab[m](c) of every consecutive-year pair: Pc[j][B] summed over j <= A&B, |j| = m."""
    n, nvar, off, yid, ss, M, varc, _ = _problem(model)
    pc = _pc_fn(model, c)
    Q = {}
    for t in range(1, len(off) - 1):
        for a_ in yid[off[t - 1]:off[t]]:
            for b_ in yid[off[t]:off[t + 1]]:
                A, B = int(ss[a_]), int(ss[b_])
                X = A & B
                if (X, B) in Q:
                    continue
                q = np.zeros(bin(X).count("1") + 1)
                sub = X
                while True:
                    q[bin(sub).count("1")] += pc(sub, B)
                    if sub == 0:
                        break
                    sub = (sub - 1) & X
                Q[(X, B)] = q
    return Q


def _forward(model, Q, e, ratio):
    n, nvar, off, yid, ss, M, varc, prior = _problem(model)
    pcnt = lambda v: bin(v).count("1")
    x = min(e, 1.0)
    y = 1.0 - x
    tf = x >= y
    z = (y / x if tf else x / y) if ratio else None
    Bb = x if tf else y
    g = 1.0 if tf else z
    v = np.ones(int(off[1]))
    E = 0
    for t in range(1, len(off) - 1):
        prev, cur = yid[off[t - 1]:off[t]], yid[off[t]:off[t + 1]]
        a = [pcnt(int(ss[k])) for k in prev]
        am = min(a)
        if ratio:
            v = v * np.array([Bb ** (ak - am) for ak in a])
        nv = np.zeros(len(cur))
        for l, bl in enumerate(cur):
            for k, ak in enumerate(prev):
                A, B = int(ss[ak]), int(ss[bl])
                q = Q[(A & B, B)]
                nX, aa = len(q) - 1, pcnt(A)
                if ratio:
                    qq = q[::-1] if tf else q
                    h = qq[0]
                    for m in range(1, nX + 1):
                        h = h * z + qq[m]
                    if aa > nX:
                        h *= g ** (aa - nX)
                    nv[l] += v[k] * h
                else:
                    nv[l] += v[k] * sum(q[m] * x ** (aa - m) * y ** m for m in range(nX + 1))
        v = nv
        if ratio:
            E += am
            if E >= FLUSH:
                v = v * Bb ** E
                E = 0
    L = v.sum() * prior
    if ratio:
        L *= Bb ** E
    return np.log(L) if L > 0 else -np.inf


@pytest.mark.parametrize("fname,points", [
    ("manual_p3_obs.txt", [(0.0, 0.3), (0.2, 0.5), (0.5, 0.5), (0.8, 0.1), (1.0, 0.7), (1.3, 0.2), (-0.25, 0.4)]),
    ("occupancies.txt", [(0.05, 0.1), (0.45, 0.6), (0.71, 0.52), (0.99, 0.9)]),
    ("config2_64x50.txt", [(0.3, 0.1), (0.62, 0.2)]),
])
def test_ratio_forms_match_direct(golden, fname, points):
    model = mdp.Model.load(golden / fname, m=400, d=100)
    for e, c in points:
        Q = _q_table(model, c)
        ref, got = _forward(model, Q, e, False), _forward(model, Q, e, True)
        if np.isfinite(ref):
            assert abs(got - ref) <= 1e-11 * max(1.0, abs(ref)), (e, c, got, ref)
        else:
            assert not np.isfinite(got) or got < -700, (e, c, got, ref)


def test_ratio_forms_flush(golden):
    """A 200-year series (config 3's file) crosses the flush threshold."""
    model = mdp.Model.load(golden / "config3_256x200.txt", m=400, d=100)
    for e, c in [(0.1, 0.05), (0.3, 0.06)]:
        Q = _q_table(model, c)
        ref, got = _forward(model, Q, e, False), _forward(model, Q, e, True)
        assert abs(got - ref) <= 1e-11 * abs(ref), (e, c, got, ref)


def _forward_gemm(model, Q, es):
    """The matrix-core wide kernel's formulation (k_fwd_mma):
    per year one product n = W C over K = every source's (k, m <= |A_k|), with
    W[p][(k, m)] = v[p][k] x_p^(|A_k| - m) y_p^m and C[(k, m)][l] = Q_kl[m]
    (zero past the transition's nX), for a batch of points at once."""
    n, nvar, off, yid, ss, M, varc, prior = _problem(model)
    pcnt = lambda v: bin(v).count("1")
    x = np.minimum(np.asarray(es, float), 1.0)
    y = 1.0 - x
    V = np.ones((len(es), int(off[1])))
    for t in range(1, len(off) - 1):
        prev, cur = yid[off[t - 1]:off[t]], yid[off[t]:off[t + 1]]
        Ks = [(k, pcnt(int(ss[ak])), m) for k, ak in enumerate(prev) for m in range(pcnt(int(ss[ak])) + 1)]
        W = np.stack([V[:, k] * x ** (a - m) * y ** m for k, a, m in Ks], axis=1)
        C = np.zeros((len(Ks), len(cur)))
        for i, (k, a, m) in enumerate(Ks):
            A = int(ss[prev[k]])
            for l, bl in enumerate(cur):
                q = Q[(A & int(ss[bl]), int(ss[bl]))]
                if m < len(q):
                    C[i, l] = q[m]
        V = W @ C
    L = V.sum(axis=1) * prior
    with np.errstate(divide="ignore"):
        return np.log(L)


@pytest.mark.parametrize("fname", ["manual_p3_obs.txt", "occupancies.txt", "config2_64x50.txt"])
def test_gemm_form_matches_direct(golden, fname):
    model = mdp.Model.load(golden / fname, m=400, d=100)
    es = [0.0, 0.2, 0.5, 0.8, 1.0, 1.3]
    for c in (0.1, 0.52):
        Q = _q_table(model, c)
        got = _forward_gemm(model, Q, es)
        for e, g in zip(es, got):
            ref = _forward(model, Q, e, False)
            if np.isfinite(ref):
                assert abs(g - ref) <= 1e-11 * max(1.0, abs(ref)), (e, c, g, ref)
            else:
                assert not np.isfinite(g), (e, c, g, ref)


def _forward_hs(model, c, e):
    """The hidden-state form of k_fwd_hs (csrc/spom_engine.hip, DESIGN.md
    §4.5): per year U[j] = y^|j| sum_{A >= j} v[A] x^(|A| - |j|) by one
    butterfly pass per patch of W (V[j] += x V[j | b], y^|j| applied once at
    the end), then n[l] = sum_{j <= B_l, j in D} Pc[j][B_l] U[j]."""
    n, nvar, off, yid, ss, M, varc, prior = _problem(model)
    pc = _pc_fn(model, c)
    x = min(e, 1.0)
    y = 1.0 - x
    v = {int(ss[k]): 1.0 for k in yid[off[0]:off[1]]}
    for t in range(1, len(off) - 1):
        W = 0
        for A in v:
            W |= A
        U = dict(v)
        for b in range(nvar):
            bit = 1 << b
            if not W & bit:
                continue
            for a1 in [a for a in U if a & bit]:
                U[a1 ^ bit] = U.get(a1 ^ bit, 0.0) + x * U[a1]
        U = {j: u * y ** bin(j).count("1") for j, u in U.items()}
        nv = {}
        for bl in yid[off[t]:off[t + 1]]:
            B = int(ss[bl])
            key, acc, j = B & W, 0.0, B & W
            while True:
                if j in U:
                    acc += pc(j, B) * U[j]
                if j == 0:
                    break
                j = (j - 1) & key
            nv[B] = acc
        v = nv
    L = sum(v.values()) * prior
    return np.log(L) if L > 0 else -np.inf


@pytest.mark.parametrize("fname", ["manual_p3_obs.txt", "occupancies.txt", "config2_64x50.txt", "wide45"])
def test_hidden_state_form_matches_direct(golden, tmp_path, fname):
    """k_fwd_hs's factorisation (v Pe by butterflies over the hidden states,
    then U Pc) against the direct per-transition sum, on the shipped inputs
    and on a survey-like series with years of up to 64 states."""
    from midaspom_amd import synth
    if fname == "wide45":
        f = synth.write(tmp_path / "w.txt", **dict(synth.CONFIG2, pmiss=0.45, seed=5, T=6))
    else:
        f = golden / fname
    model = mdp.Model.load(f, m=400, d=100)
    for c in (0.1, 0.52):
        Q = _q_table(model, c)
        for e in (0.0, 0.2, 0.5, 0.8, 1.0, 1.3):
            ref = _forward(model, Q, e, False)
            got = _forward_hs(model, c, e)
            if np.isfinite(ref):
                assert abs(got - ref) <= 1e-11 * max(1.0, abs(ref)), (e, c, got, ref)
            else:
                assert not np.isfinite(got), (e, c, got, ref)
