"""oracle -- TEST INFRASTRUCTURE ONLY.

ctypes binding of the CPU restatement of the reference likelihood
(oracle/spom_oracle.c).  Importable only by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, as the checker / CPU baseline.  The product
package (midaspom_amd) never imports this module.

Pinning: tests/test_oracle_golden.py checks this oracle against the manual's
worked example (Manual_linux.pdf p.3) and the reference outputs recorded in
SURVEY.md §8(c)/Appendix C (posterior md5s, Total log-likelihood values).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
BUILD = ORACLE_DIR / "_build"
LIB = BUILD / "liboracle.so"
CLI = BUILD / "orc_main"

_dp = ctypes.POINTER(ctypes.c_double)
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        h = ctypes.CDLL(str(LIB))
        vp = ctypes.c_void_p
        h.orc_model_load.argtypes = [ctypes.c_char_p, ctypes.c_double, ctypes.c_float, ctypes.c_double,
                                     ctypes.POINTER(vp)]
        h.orc_model_build.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_uint, ctypes.c_uint,
                                      ctypes.c_double, ctypes.c_float, ctypes.c_double, ctypes.POINTER(vp)]
        h.orc_model_free.argtypes = [vp]
        for name in ("orc_model_n", "orc_model_tmax", "orc_model_nvar", "orc_model_nstates",
                     "orc_model_nextid"):
            getattr(h, name).argtypes = [vp]
            getattr(h, name).restype = ctypes.c_uint
        h.orc_model_np.argtypes = [vp, ctypes.c_uint]
        h.orc_model_np.restype = ctypes.c_uint
        h.orc_model_simp.argtypes = [vp, ctypes.c_uint, ctypes.c_uint]
        h.orc_model_simp.restype = ctypes.c_uint
        h.orc_model_short2all.argtypes = [vp, ctypes.c_uint]
        h.orc_model_short2all.restype = ctypes.c_uint
        h.orc_model_prior.argtypes = [vp, ctypes.c_uint]
        h.orc_model_prior.restype = ctypes.c_double
        h.orc_grid.argtypes = [ctypes.c_uint, ctypes.c_double, ctypes.c_double, _dp]
        h.orc_grid.restype = ctypes.c_double
        h.orc_loglik_grid_mt.argtypes = [vp, _dp, _dp, ctypes.c_uint, ctypes.c_uint, _dp]
        h.orc_loglik_points.argtypes = [vp, _dp, _dp, ctypes.c_size_t, _dp]
        h.orc_ltot.argtypes = [_dp, ctypes.c_uint, ctypes.c_double]
        h.orc_ltot.restype = ctypes.c_double
        h.orc_write_posterior.argtypes = [ctypes.c_char_p, _dp, ctypes.c_uint, ctypes.c_double]
        ip = ctypes.POINTER(ctypes.c_int32)
        common = [ip, ctypes.c_uint32, ctypes.c_double, ctypes.c_float, ctypes.c_double, ctypes.c_int,
                  ctypes.c_int, ctypes.c_double, ctypes.c_double, _dp, ctypes.c_uint32]
        h.orc_dieoff_lik.argtypes = common + [_dp]
        h.orc_loss_lik.argtypes = common + [_dp, ctypes.c_uint32, _dp]
        h.orc_scenario_vec.argtypes = [ip, ctypes.c_uint32, ctypes.c_double, ctypes.c_float, ctypes.c_double,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_int, _dp]
        h.orc_kgrid.argtypes = [ctypes.c_uint32, ctypes.c_double, ctypes.c_double, _dp]
        h.orc_philox.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.POINTER(ctypes.c_uint32)]
        h.orc_future_sim.argtypes = [ip, ctypes.c_uint, _dp, ctypes.c_uint, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                     ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                                     ctypes.c_uint, ctypes.POINTER(ctypes.c_uint64)]
        _lib = h
    return _lib


def _p(a):
    return a.ctypes.data_as(_dp)


class OracleModel:
    def __init__(self, handle):
        self.h = handle

    @classmethod
    def load(cls, path, m=400.0, p=0.5, d=100.0):
        h = ctypes.c_void_p()
        rc = lib().orc_model_load(os.fsencode(str(path)), m, p, d, ctypes.byref(h))
        if rc:
            raise RuntimeError(f"oracle load failed ({rc})")
        return cls(h)

    @classmethod
    def from_obs(cls, obs, m=400.0, p=0.5, d=100.0):
        a = np.ascontiguousarray(obs, dtype=np.int32)
        h = ctypes.c_void_p()
        rc = lib().orc_model_build(a.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), a.shape[1], a.shape[0],
                                   m, p, d, ctypes.byref(h))
        if rc:
            raise RuntimeError(f"oracle build failed ({rc})")
        return cls(h)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_model_free(self.h)
            self.h = None

    def _u(self, name, *a):
        return getattr(lib(), name)(self.h, *a)

    n = property(lambda s: s._u("orc_model_n"))
    tmax = property(lambda s: s._u("orc_model_tmax"))
    nvar = property(lambda s: s._u("orc_model_nvar"))
    nstates = property(lambda s: s._u("orc_model_nstates"))
    nextid = property(lambda s: s._u("orc_model_nextid"))

    @property
    def npstates(self):
        return np.array([self._u("orc_model_np", t) for t in range(self.tmax)])

    @property
    def year_ids(self):
        nps = self.npstates
        return [np.array([self._u("orc_model_simp", t, q) for q in range(nps[t])]) for t in range(self.tmax)]

    @property
    def short_state(self):
        return np.array([self._u("orc_model_short2all", a) for a in range(self.nextid)])

    @property
    def prior(self):
        return np.array([self._u("orc_model_prior", q) for q in range(self.npstates[0])])

    def loglik_grid(self, e, c=None, threads=None):
        e = np.ascontiguousarray(e, dtype=np.float64)
        c = e if c is None else np.ascontiguousarray(c, dtype=np.float64)
        if e.size != c.size:
            ee, cc = np.meshgrid(e, c, indexing="ij")
            return self.loglik_points(ee.ravel(), cc.ravel(), threads).reshape(e.size, c.size)
        out = np.empty((e.size, c.size))
        threads = threads or min(8, os.cpu_count() or 1)
        if np.array_equal(e, c):
            lib().orc_loglik_grid_mt(self.h, _p(e), _p(c), e.size, threads, _p(out))
            return out
        ee, cc = np.meshgrid(e, c, indexing="ij")
        return self.loglik_points(ee.ravel(), cc.ravel(), threads).reshape(e.size, c.size)

    def loglik_points(self, e, c, threads=None):
        """loglik at paired points (e[q], c[q]); threads split the list."""
        e = np.ascontiguousarray(e, dtype=np.float64)
        c = np.ascontiguousarray(c, dtype=np.float64)
        out = np.empty(e.size)
        threads = max(1, min(threads or 1, e.size))
        if threads == 1:
            lib().orc_loglik_points(self.h, _p(e), _p(c), e.size, _p(out))
            return out
        import concurrent.futures as cf
        bounds = np.linspace(0, e.size, threads + 1).astype(int)

        def work(i):
            a, b = bounds[i], bounds[i + 1]
            if b > a:
                lib().orc_loglik_points(self.h, _p(e[a:b]), _p(c[a:b]), b - a, _p(out[a:b]))
        # ctypes releases the GIL during the call, so threads run in parallel
        with cf.ThreadPoolExecutor(threads) as ex:
            list(ex.map(work, range(threads)))
        return out


def grid(s, lo=0.0, hi=1.0):
    g = np.empty(s)
    win = lib().orc_grid(s, lo, hi, _p(g))
    return g, win


def ltot(lik, win):
    a = np.ascontiguousarray(lik, dtype=np.float64)
    return lib().orc_ltot(_p(a), a.shape[0], win)


def write_posterior(path, lik, lt):
    a = np.ascontiguousarray(lik, dtype=np.float64)
    rc = lib().orc_write_posterior(os.fsencode(str(path)), _p(a), a.shape[0], lt)
    if rc:
        raise RuntimeError("oracle write failed")


def run(path, out=None, m=400.0, p=0.5, d=100.0, s=101, lo=0.0, hi=1.0, threads=None):
    """Full reference pipeline on the CPU: returns (loglik, ltot)."""
    model = OracleModel.load(path, m, p, d)
    g, win = grid(s, lo, hi)
    lik = model.loglik_grid(g, g, threads)
    lt = ltot(lik, win)
    if out is not None:
        write_posterior(out, lik, lt)
    return lik, lt


# ---------------------------------------------------------------------------
# scenario likelihoods (oracle/spom_dieoff_oracle.c): dieoff.c / loss.c
# ---------------------------------------------------------------------------
def first_row(path):
    """The first survey row as the reference reads it (dieoff.c:185-201)."""
    data = Path(path).read_bytes()
    n = 1 + sum(1 for ch in data.split(b"\n", 1)[0] if ch in (32, 9))
    toks = data.split()
    return np.array([int(t) for t in toks[:n]], dtype=np.int32)


def kgrid(s, lo=0.1, hi=100.0):
    K = np.empty(s)
    lib().orc_kgrid(s, lo, hi, _p(K))
    return K


def dieoff_lik(row, K, e, c, ts=20, tdis=10, m=400.0, p=0.5, d=200.0):
    row = np.ascontiguousarray(row, dtype=np.int32)
    K = np.ascontiguousarray(K, dtype=np.float64)
    out = np.empty(K.size)
    rc = lib().orc_dieoff_lik(row.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), row.size, m, p, d, ts, tdis,
                              e, c, _p(K), K.size, _p(out))
    if rc:
        raise RuntimeError("orc_dieoff_lik failed")
    return out


def loss_lik(row, K, dsrc, e, c, ts=20, tdis=10, m=400.0, p=0.5, d=200.0):
    row = np.ascontiguousarray(row, dtype=np.int32)
    K = np.ascontiguousarray(K, dtype=np.float64)
    dsrc = np.ascontiguousarray(dsrc, dtype=np.float64)
    out = np.empty((K.size, dsrc.size))
    rc = lib().orc_loss_lik(row.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), row.size, m, p, d, ts, tdis,
                            e, c, _p(K), K.size, _p(dsrc), dsrc.size, _p(out))
    if rc:
        raise RuntimeError("orc_loss_lik failed")
    return out


def scenario_vec(row, kind, K, e, c, ts=20, tdis=10, m=400.0, p=0.5, d=200.0, dsrc=0.0):
    """One (e, c, K[, d]) point of the die-off / loss likelihood by vector
    propagation (orc_scenario_vec): the reference's matrix entries, products
    associated right to left, for n up to 20 patches."""
    row = np.ascontiguousarray(row, dtype=np.int32)
    out = ctypes.c_double()
    rc = lib().orc_scenario_vec(row.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), row.size, m, p, d, ts, tdis,
                                e, c, K, dsrc, 1 if kind == "loss" else 0, ctypes.byref(out))
    if rc:
        raise RuntimeError("orc_scenario_vec failed")
    return out.value


# ---------------------------------------------------------------------------
# forward simulation (oracle/spom_future_oracle.c): future.c
# ---------------------------------------------------------------------------
RNG_PHILOX, RNG_GLIBC = 0, 1


def philox(key: int, ctr):
    """Philox4x32-10(key, ctr[4]) -> 4 uint32 words."""
    h = lib()
    c = (ctypes.c_uint32 * 4)(*[int(x) & 0xffffffff for x in ctr])
    o = (ctypes.c_uint32 * 4)()
    h.orc_philox(ctypes.c_uint32(key & 0xffffffff), ctypes.c_uint32((key >> 32) & 0xffffffff), c, o)
    return list(o)


def last_row(path):
    """(n, tmax, last survey row) as future.c:193-225 reads them."""
    data = Path(path).read_bytes()
    n = 1 + sum(1 for ch in data.split(b"\n", 1)[0] if ch in (32, 9))
    tmax = data.count(b"\n")
    row = [0] * n
    for q, tok in enumerate(data.split()[: tmax * n]):
        row[q % n] = int(tok)
    return n, tmax, np.array(row, dtype=np.int32)


def read_posterior(path):
    """necstep x necstep posterior as future.c:237-262 reads it."""
    data = Path(path).read_bytes()
    s = sum(1 for ch in data.split(b"\n", 1)[0] if ch in (32, 9))
    vals = np.array([float(t) for t in data.split()[: s * s]], dtype=np.float64)
    return vals.reshape(s, s)


def future_counts(row, post, tfut=50, nrep=10000, m=400.0, d=200.0, KD=1.0, KS=0.0, dS=200.0,
                  mode=RNG_PHILOX, seed=0, rep0=0, threads=None):
    """Per-year all-extinct counts over replicates [rep0, rep0 + nrep)."""
    h = lib()
    row = np.ascontiguousarray(row, dtype=np.int32)
    post = np.ascontiguousarray(post, dtype=np.float64)
    counts = np.zeros(tfut, dtype=np.uint64)
    threads = threads or min(16, os.cpu_count() or 1)
    rc = h.orc_future_sim(row.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), row.size, _p(post),
                          post.shape[0] if post.size else 0, m, d, KD, KS, dS, mode,
                          ctypes.c_uint64(seed), ctypes.c_uint64(rep0), ctypes.c_uint64(nrep), tfut, threads,
                          counts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if rc:
        raise RuntimeError("orc_future_sim failed")
    return counts
