"""midaspom_amd -- MI355X-native MIDASPOM posterior-grid likelihood engine.

Host-side mirror of the reference pipeline (sources/main_MIDASPOM.c) over the
C ABI of include/midaspom.h:

    model = Model.load("occupancies.txt", m=400, p=0.5, d=100)   # :137-287
    g, win = grid(101, 0.0, 1.0)                                 # :312-319
    with Engine(model) as eng:
        lik = eng.loglik_grid(g, g)                              # :341-395 on the GPU
    ltot = log_total(lik, win)                                   # :413-425
    write_posterior("posterior.txt", lik, ltot)                  # :427-436

Every compute call goes through libmidaspom.so (HIP, gfx950); there is no
CPU fallback in this package.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

from . import _lib
from ._lib import MidaspomError, check, lib

__all__ = [
    "Model", "Engine", "grid", "log_total", "write_posterior", "posterior",
    "run_file", "MidaspomError", "Scenario", "kgrid", "dgrid", "first_row",
    "Future", "read_survey", "read_posterior", "device_count",
]


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class Model:
    """Parsed + enumerated occupancy model (``mdp_model``)."""

    def __init__(self, handle: ctypes.c_void_p):
        self._h = handle
        self._view = _lib.Problem()
        check(lib().mdp_model_problem(self._h, ctypes.byref(self._view)))

    @classmethod
    def load(cls, path, m: float = 400.0, p: float = 0.5, d: float = 100.0) -> "Model":
        h = ctypes.c_void_p()
        check(lib().mdp_model_load(os.fsencode(str(path)), float(m), float(p), float(d),
                                   ctypes.byref(h)))
        return cls(h)

    @classmethod
    def from_obs(cls, obs, m: float = 400.0, p: float = 0.5, d: float = 100.0) -> "Model":
        a = np.ascontiguousarray(obs, dtype=np.int32)
        if a.ndim != 2:
            raise ValueError("obs must be a 2-D [years][patches] matrix")
        h = ctypes.c_void_p()
        check(lib().mdp_model_from_obs(a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       a.shape[1], a.shape[0], float(m), float(p), float(d),
                                       ctypes.byref(h)))
        return cls(h)

    def close(self):
        if self._h:
            lib().mdp_model_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- read-only views -------------------------------------------------
    @property
    def problem(self) -> _lib.Problem:
        return self._view

    n = property(lambda s: s._view.n)
    tmax = property(lambda s: s._view.tmax)
    nvar = property(lambda s: s._view.nvar)
    nextid = property(lambda s: s._view.nextid)
    nstates = property(lambda s: 1 << s._view.nvar)

    @property
    def obs(self) -> np.ndarray:
        v = self._view
        return np.ctypeslib.as_array(v.obs, shape=(v.tmax, v.n)).copy()

    @property
    def M(self) -> np.ndarray:
        v = self._view
        return np.ctypeslib.as_array(v.M, shape=(v.n, v.n)).copy()

    @property
    def var_cols(self) -> np.ndarray:
        v = self._view
        if v.nvar == 0:
            return np.zeros(0, dtype=np.uint32)
        return np.ctypeslib.as_array(v.var_cols, shape=(v.nvar,)).copy()

    @property
    def year_off(self) -> np.ndarray:
        v = self._view
        return np.ctypeslib.as_array(v.year_off, shape=(v.tmax + 1,)).copy()

    @property
    def npstates(self) -> np.ndarray:
        return np.diff(self.year_off)

    @property
    def year_ids(self) -> list:
        off = self.year_off
        flat = np.ctypeslib.as_array(self._view.year_ids, shape=(int(off[-1]),)).copy()
        return [flat[off[t]:off[t + 1]] for t in range(self.tmax)]

    @property
    def short_state(self) -> np.ndarray:
        v = self._view
        return np.ctypeslib.as_array(v.short_state, shape=(v.nextid,)).copy()

    @property
    def prior(self) -> np.ndarray:
        off = self.year_off
        return np.ctypeslib.as_array(self._view.prior, shape=(int(off[1]),)).copy()


class Engine:
    """GPU likelihood engine (``mdp_engine``) over one or more devices."""

    def __init__(self, model: Model, devices=None, n_devices: int | None = None, options=None):
        """options: engine options (dict or "K=V;..." string,
        ``mdp_engine_create_opts``); None forwards the MDP_* variables set in
        the environment (``_lib.options_string``)."""
        self.model = model  # keep the host tables alive
        h = ctypes.c_void_p()
        opts = _lib.options_string(options)
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = lib().mdp_engine_create_opts(ctypes.byref(model.problem), arr, len(devices), opts, ctypes.byref(h))
        else:
            rc = lib().mdp_engine_create_opts(ctypes.byref(model.problem), None, int(n_devices or 0), opts,
                                              ctypes.byref(h))
        check(rc)
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().mdp_engine_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def loglik_grid(self, e, c, layout: str = "ec") -> np.ndarray:
        """log L on the e x c grid (host arrays in, host [ne][nc] out).
        layout="ce" computes the devices' native [c][e] and returns its
        transposed view (still indexed [ie][ic]; log_total / write_posterior
        read it in place)."""
        e = np.ascontiguousarray(e, dtype=np.float64)
        c = np.ascontiguousarray(c, dtype=np.float64)
        if layout == "ce":
            out = np.empty((c.size, e.size), dtype=np.float64)
            check(lib().mdp_loglik_grid_layout(self._h, _dptr(e), e.size, _dptr(c), c.size, 1, _dptr(out)))
            return out.T
        out = np.empty((e.size, c.size), dtype=np.float64)
        check(lib().mdp_loglik_grid(self._h, _dptr(e), e.size, _dptr(c), c.size, _dptr(out)))
        return out

    def set_grid(self, e, c) -> None:
        e = np.ascontiguousarray(e, dtype=np.float64)
        c = np.ascontiguousarray(c, dtype=np.float64)
        check(lib().mdp_engine_set_grid(self._h, _dptr(e), e.size, _dptr(c), c.size))
        self.ne, self.nc = e.size, c.size

    def set_cbound(self, cbound: float) -> None:
        """Build the per-c tables of the following grids for |c| <= max(the
        grid's, cbound) (ABI 9): ranks computing column slabs of one grid pass
        its max |c|, so every slab has the bits of a one-rank run."""
        check(lib().mdp_engine_set_cbound(self._h, float(cbound)))

    def set_layout(self, layout: str) -> None:
        """Layout ``run`` writes: "ec" (default) out[ie*ld + ic], the
        reference's lik[i][j]; "ce" out[ic*ld + ie] (ld >= ne), whose stores
        coalesce (``mdp_engine_set_layout``)."""
        check(lib().mdp_engine_set_layout(self._h, {"ec": 0, "ce": 1}[layout]))

    def run(self, d_out: int, ld_out: int, stream: int = 0) -> None:
        """Compute into device memory at address ``d_out`` (e.g. a torch
        tensor's data_ptr()) on hipStream ``stream``, used as given: 0 is
        HIP's null stream, which is torch's default stream."""
        check(lib().mdp_engine_run(self._h, ctypes.c_void_p(d_out), ld_out, ctypes.c_void_p(stream)))

    def set_profiling(self, on: bool = True) -> None:
        check(lib().mdp_engine_set_profiling(self._h, int(bool(on))))

    def kernel_ms(self) -> dict:
        buf = (ctypes.c_double * 8)()
        k = check(lib().mdp_engine_kernel_ms(self._h, buf, 8))
        names = [lib().mdp_engine_kernel_name(self._h, i).decode() for i in range(k)]
        return {nm: buf[i] for i, nm in enumerate(names) if nm}

    def time_kernels(self, d_out: int, ld_out: int, stream: int = 0, reps: int = 50) -> dict:
        """Mean duration (ms) of each kernel of the path, each launched `reps`
        times back to back (no per-launch events); d_out ends as run() leaves it."""
        buf = (ctypes.c_double * 3)()
        k = check(lib().mdp_engine_time_kernels(self._h, ctypes.c_void_p(d_out), ld_out,
                                                ctypes.c_void_p(stream), reps, buf, 3))
        names = [lib().mdp_engine_kernel_name(self._h, i).decode() for i in range(k)]
        return {nm: buf[i] for i, nm in enumerate(names) if nm}

    def diag_report(self) -> str:
        """Phase-stamp report of the last run (diag library, engine option MDP_DIAG=1)."""
        buf = ctypes.create_string_buffer(8192)
        check(lib().mdp_engine_diag_report(self._h, buf, len(buf)))
        return buf.value.decode()

    def info(self) -> dict:
        inf = _lib.EngineInfo()
        check(lib().mdp_engine_get_info(self._h, ctypes.byref(inf)))
        return {f: getattr(inf, f) for f, _ in inf._fields_}

    def launched(self) -> set:
        """The kernel instantiations this engine has launched (e.g.
        {"k_qrows<16,0,2>", "mdp_fwd_jit<reading,maxA12>"})."""
        buf = ctypes.create_string_buffer(4096)
        check(lib().mdp_engine_launched(self._h, buf, len(buf)))
        return set(buf.value.decode().split())

    def work(self, ne: int, nc: int) -> dict:
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(lib().mdp_engine_work(self._h, ne, nc, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return {"flop_impl": a.value, "flop_survey": b.value, "bytes_min": c.value}


    def work_fact(self, ne: int, nc: int) -> dict:
        """Closed-form FP64 work of the factorised algorithm on an ne x nc
        grid (``mdp_engine_work_fact``): per-c and per-point
        terms and the total ``flop``."""
        w = _lib.Work()
        check(lib().mdp_engine_work_fact(self._h, ne, nc, ctypes.byref(w)))
        return {f: getattr(w, f) for f, _ in w._fields_}


def device_count() -> int:
    """Visible HIP devices, from the library (mdp_device_count)."""
    return int(lib().mdp_device_count())


def grid(s: int, lo: float = 0.0, hi: float = 1.0):
    """(g, win): the reference's parameter grid (:120, :312-319)."""
    g = np.empty(int(s), dtype=np.float64)
    win = lib().mdp_grid(int(s), float(lo), float(hi), _dptr(g))
    return g, win


def _view(lik: np.ndarray):
    """(base array, se, sc) of an s x s float64 [e][c] matrix given as is or
    as the transpose of a C-contiguous [c][e] array (lik = ce.T): the host
    functions read either in place through mdp_*_view, no copy."""
    a = np.asarray(lik)
    if a.ndim != 2 or a.shape[0] != a.shape[1]:
        raise ValueError("needs a square s x s grid")
    if a.dtype == np.float64 and a.T.flags.c_contiguous and not a.flags.c_contiguous:
        return a.T, 1, a.shape[0]
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.shape[0], 1


def log_total(lik: np.ndarray, win: float) -> float:
    """Trapezoid log normaliser (:413-425); lik may be an [e][c] array or the
    transposed view of a [c][e] one."""
    a, se, sc = _view(lik)
    return float(lib().mdp_log_total_view(_dptr(a), a.shape[0], se, sc, float(win)))


def write_posterior(path, lik: np.ndarray, ltot: float, raw: bool = False) -> None:
    """Posterior text file, reference bit layout (:427-436); lik as for log_total."""
    a, se, sc = _view(lik)
    check(lib().mdp_write_posterior_view(os.fsencode(str(path)), _dptr(a), a.shape[0], se, sc, float(ltot),
                                         int(raw)))


def posterior(lik: np.ndarray, ltot: float) -> np.ndarray:
    with np.errstate(invalid="ignore", over="ignore"):
        return np.exp(lik - ltot)


def run_file(input_path, output_path=None, m=400.0, p=0.5, d=100.0, s=101, lo=0.0, hi=1.0,
             devices=None):
    """Whole MIDASPOM.out pipeline on the GPU; returns (loglik, ltot)."""
    model = Model.load(input_path, m=m, p=p, d=d)
    g, win = grid(s, lo, hi)
    with Engine(model, devices=devices) as eng:
        lik = eng.loglik_grid(g, g, layout="ce")  # the devices' native layout, read in place
    ltot = log_total(lik, win)
    if output_path is not None:
        write_posterior(output_path, lik, ltot)
    return lik, ltot


# ---------------------------------------------------------------------------
# scenario likelihoods: in-situ die-off and habitat loss
# ---------------------------------------------------------------------------
def kgrid(s: int, lo: float = 0.1, hi: float = 100.0) -> np.ndarray:
    """log10-spaced K grid of main_MIDASPOM_dieoff.c:284-286."""
    K = np.empty(s)
    lib().mdp_kgrid(s, lo, hi, _dptr(K))
    return K


def dgrid(s: int, lo: float = 200.0, hi: float = 4000.0) -> np.ndarray:
    """Linear source-distance grid of main_MIDASPOM_loss.c:319-322."""
    d = np.empty(s)
    lib().mdp_dgrid(s, lo, hi, _dptr(d))
    return d


def first_row(path) -> np.ndarray:
    """The first survey row as the scenario programs read it
    (main_MIDASPOM_dieoff.c:185-201: n from line 1, then n integers)."""
    data = Path(path).read_bytes()
    n = 1 + sum(1 for ch in data.split(b"\n", 1)[0] if ch in (32, 9))
    return np.array([int(t) for t in data.split()[:n]], dtype=np.int32)


class Scenario:
    """GPU likelihood of the first survey row under the die-off (kind
    'dieoff', main_MIDASPOM_dieoff.c) or habitat-loss (kind 'loss',
    main_MIDASPOM_loss.c) scenario."""

    def __init__(self, row, kind: str = "dieoff", m: float = 400.0, p: float = 0.5, d: float = 200.0,
                 device: int = 0, options=None):
        if kind not in ("dieoff", "loss"):
            raise ValueError("kind must be 'dieoff' or 'loss'")
        self.kind = kind
        row = np.ascontiguousarray(row, dtype=np.int32)
        h = ctypes.c_void_p()
        opts = _lib.options_string(options, _lib.SCENARIO_OPTION_NAMES)
        check(lib().mdp_scenario_create_opts(row.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), row.size, m, p, d,
                                             1 if kind == "loss" else 0, device, opts, ctypes.byref(h)))
        self._h = h

    def close(self):
        if self._h:
            lib().mdp_scenario_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def lik(self, e, c, K, dsrc=None, ts: int = 20, tdis: int = 10) -> np.ndarray:
        """L[ie][ic][iK] (die-off) or L[ie][ic][iK][id] (loss), raw likelihoods."""
        e = np.ascontiguousarray(np.atleast_1d(e), dtype=np.float64)
        c = np.ascontiguousarray(np.atleast_1d(c), dtype=np.float64)
        K = np.ascontiguousarray(np.atleast_1d(K), dtype=np.float64)
        if self.kind == "loss":
            dsrc = np.ascontiguousarray(np.atleast_1d(dsrc), dtype=np.float64)
            nd = dsrc.size
            shape = (e.size, c.size, K.size, nd)
        else:
            dsrc = np.zeros(1)
            nd = 1
            shape = (e.size, c.size, K.size)
        out = np.empty(int(np.prod(shape)))
        check(lib().mdp_scenario_lik(self._h, ts, tdis, _dptr(e), e.size, _dptr(c), c.size, _dptr(K), K.size, _dptr(dsrc),
                                     nd, _dptr(out)))
        return out.reshape(shape)

    def set_grid(self, e, c, K, dsrc=None, ts: int = 20, tdis: int = 10) -> tuple:
        """Upload an (e, c, K[, d]) grid once for run(); returns the output shape."""
        e = np.ascontiguousarray(np.atleast_1d(e), dtype=np.float64)
        c = np.ascontiguousarray(np.atleast_1d(c), dtype=np.float64)
        K = np.ascontiguousarray(np.atleast_1d(K), dtype=np.float64)
        if self.kind == "loss":
            dsrc = np.ascontiguousarray(np.atleast_1d(dsrc), dtype=np.float64)
            shape = (e.size, c.size, K.size, dsrc.size)
        else:
            dsrc = np.zeros(1)
            shape = (e.size, c.size, K.size)
        check(lib().mdp_scenario_set_grid(self._h, ts, tdis, _dptr(e), e.size, _dptr(c), c.size, _dptr(K), K.size,
                                          _dptr(dsrc), dsrc.size))
        self.shape = shape
        return shape

    def run(self, d_out: int, stream: int = 0) -> None:
        """Compute the set grid into device memory at ``d_out`` (float64, the
        set_grid shape), asynchronously on hipStream ``stream`` (0 = HIP's
        null stream, torch's default)."""
        check(lib().mdp_scenario_run(self._h, ctypes.c_void_p(d_out), ctypes.c_void_p(stream)))

    def time_kernels(self, d_out: int, stream: int = 0, reps: int = 10) -> dict:
        ms = (ctypes.c_double * 2)()
        check(lib().mdp_scenario_time_kernels(self._h, ctypes.c_void_p(d_out), ctypes.c_void_p(stream), reps, ms))
        return {"k_scn_v": ms[0], "k_scn_lik": ms[1]}


# ---------------------------------------------------------------------------
# forward simulation of extinction (main_MIDASPOM_future.c)
# ---------------------------------------------------------------------------
def read_survey(path):
    """(n, tmax, last survey row) as future.c:193-225 reads them."""
    n, t = ctypes.c_uint32(), ctypes.c_uint32()
    p = ctypes.POINTER(ctypes.c_int32)()
    check(lib().mdp_future_read_survey(os.fsencode(str(path)), ctypes.byref(n), ctypes.byref(t), ctypes.byref(p)))
    try:
        row = np.ctypeslib.as_array(p, shape=(n.value,)).copy()
    finally:
        lib().mdp_free(p)
    return n.value, t.value, row


def read_posterior(path) -> np.ndarray:
    """necstep x necstep posterior as future.c:237-262 reads it."""
    s = ctypes.c_uint32()
    p = ctypes.POINTER(ctypes.c_double)()
    check(lib().mdp_future_read_posterior(os.fsencode(str(path)), ctypes.byref(s), ctypes.byref(p)))
    try:
        post = np.ctypeslib.as_array(p, shape=(s.value * s.value,)).copy() if s.value else np.zeros(0)
    finally:
        lib().mdp_free(p)
    return post.reshape(s.value, s.value)


class Future:
    """GPU replicate loop of MIDASPOM_future (``mdp_future``): per-year counts
    of replicates with every patch extinct."""

    def __init__(self, row, post, m: float = 400.0, d: float = 200.0, KD: float = 1.0, KS: float = 0.0,
                 dS: float = 200.0, device: int = 0):
        row = np.ascontiguousarray(row, dtype=np.int32)
        post = np.ascontiguousarray(post, dtype=np.float64)
        self._post = post
        h = ctypes.c_void_p()
        check(lib().mdp_future_create(row.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), row.size, _dptr(post),
                                      post.shape[0] if post.size else 0, m, d, KD, KS, dS, device,
                                      ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().mdp_future_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def simulate(self, nrep: int, tfut: int = 50, seed: int = 0, rep0: int = 0) -> np.ndarray:
        """counts[t] over replicates [rep0, rep0 + nrep) (host uint64 array)."""
        counts = np.zeros(tfut, dtype=np.uint64)
        check(lib().mdp_future_simulate(self._h, seed, rep0, nrep, tfut,
                                        counts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
        return counts

    def simulate_device(self, d_counts: int, nrep: int, tfut: int, seed: int = 0, rep0: int = 0,
                        stream: int = 0) -> None:
        """Into device memory at ``d_counts`` (uint64[tfut]), asynchronously
        on hipStream ``stream`` (0 = HIP's null stream, torch's default).
        Call check() before trusting the counts."""
        check(lib().mdp_future_simulate_device(self._h, seed, rep0, nrep, tfut, ctypes.c_void_p(d_counts),
                                               ctypes.c_void_p(stream)))

    def check(self, stream: int = 0) -> None:
        """Wait for ``stream``; raise if any device launch since the previous
        check overflowed the posterior look-back (the flag is cleared here)."""
        check(lib().mdp_future_check(self._h, ctypes.c_void_p(stream)))

    def time_kernel(self, nrep: int, tfut: int, seed: int = 0, reps: int = 10) -> float:
        ms = ctypes.c_double()
        check(lib().mdp_future_time_kernel(self._h, seed, nrep, tfut, reps, ctypes.byref(ms)))
        return ms.value


def philox(key: int, ctr) -> list:
    """The engine's generator, Philox4x32-10(key, ctr[4]) (host restatement)."""
    c = (ctypes.c_uint32 * 4)(*[int(x) & 0xffffffff for x in ctr])
    o = (ctypes.c_uint32 * 4)()
    check(lib().mdp_future_philox(key & 0xffffffffffffffff, c, o))
    return list(o)
