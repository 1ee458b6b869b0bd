"""ctypes binding of the in-tree C ABI (include/midaspom.h).

The shared library is midaspom_amd/_build/libmidaspom.so, built by
``__graft_entry__.build()`` (``make -C midaspom_amd/csrc``).  There is no
fallback: importing a compute entry point without the library raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
BUILD_DIR = PKG_DIR / "_build"
LIB_PATH = BUILD_DIR / "libmidaspom.so"
# the measurement build (`make -C midaspom_amd/csrc diag`: phase stamps,
# MDP_JIT_HACK); loaded instead of LIB_PATH only when MIDASPOM_DIAG_LIB=1,
# which only scripts/ set -- the CLIs, tests and bench.py use LIB_PATH
DIAG_LIB_PATH = BUILD_DIR / "libmidaspom_diag.so"
CLI_PATH = BUILD_DIR / "midaspom"
DIEOFF_CLI_PATH = BUILD_DIR / "midaspom_dieoff"
LOSS_CLI_PATH = BUILD_DIR / "midaspom_loss"
FUTURE_CLI_PATH = BUILD_DIR / "midaspom_future"

MDP_OK = 0
ERRORS = {
    -1: "MDP_EINVAL",
    -2: "MDP_EIO",
    -3: "MDP_ENOMEM",
    -4: "MDP_EHIP",
    -5: "MDP_ENODEV",
    -6: "MDP_EUNSUPPORTED",
}


class MidaspomError(RuntimeError):
    """A negative return code from the C ABI, with mdp_last_error()."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


c_u32 = ctypes.c_uint32
c_dbl_p = ctypes.POINTER(ctypes.c_double)
c_u32_p = ctypes.POINTER(ctypes.c_uint32)
c_i32_p = ctypes.POINTER(ctypes.c_int32)


class Problem(ctypes.Structure):
    """Mirror of ``mdp_problem``."""

    _fields_ = [
        ("n", c_u32),
        ("tmax", c_u32),
        ("nvar", c_u32),
        ("nextid", c_u32),
        ("obs", c_i32_p),
        ("var_cols", c_u32_p),
        ("M", c_dbl_p),
        ("short_state", c_u32_p),
        ("year_off", c_u32_p),
        ("year_ids", c_u32_p),
        ("prior", ctypes.POINTER(ctypes.c_float)),
    ]


class Work(ctypes.Structure):
    """Mirror of ``mdp_work`` (closed-form factorised FP64 work)."""

    _fields_ = [(f, ctypes.c_double) for f in
                ("z_c", "pc_c", "item_c", "q_c", "weight_pt", "use_pt", "final_pt", "flop", "use_pt_min",
                 "flop_min", "setup_pt", "use_pt_ratio", "final_pt_ratio", "pt_min", "flop_min_direct")]


class EngineInfo(ctypes.Structure):
    """Mirror of ``mdp_engine_info``."""

    _fields_ = [
        ("n_devices", ctypes.c_int),
        ("npairs", c_u32),
        ("nuses", c_u32),
        ("ncoef", c_u32),
        ("npmax", c_u32),
        ("variant", c_u32),
    ]


# (name, restype, argtypes) for every function declared in include/midaspom.h
SIGNATURES = [
    ("mdp_model_load", ctypes.c_int,
     [ctypes.c_char_p, ctypes.c_double, ctypes.c_float, ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]),
    ("mdp_model_from_obs", ctypes.c_int,
     [c_i32_p, c_u32, c_u32, ctypes.c_double, ctypes.c_float, ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]),
    ("mdp_model_free", None, [ctypes.c_void_p]),
    ("mdp_model_problem", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Problem)]),
    ("mdp_grid", ctypes.c_double, [c_u32, ctypes.c_double, ctypes.c_double, c_dbl_p]),
    ("mdp_log_total", ctypes.c_double, [c_dbl_p, c_u32, ctypes.c_double]),
    ("mdp_write_posterior", ctypes.c_int, [ctypes.c_char_p, c_dbl_p, c_u32, ctypes.c_double, ctypes.c_int]),
    ("mdp_log_total_view", ctypes.c_double, [c_dbl_p, c_u32, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_double]),
    ("mdp_write_posterior_view", ctypes.c_int,
     [ctypes.c_char_p, c_dbl_p, c_u32, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_double, ctypes.c_int]),
    ("mdp_engine_create", ctypes.c_int,
     [ctypes.POINTER(Problem), ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("mdp_engine_create_opts", ctypes.c_int,
     [ctypes.POINTER(Problem), ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_char_p,
      ctypes.POINTER(ctypes.c_void_p)]),
    ("mdp_engine_destroy", None, [ctypes.c_void_p]),
    ("mdp_loglik_grid", ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_u32, c_dbl_p, c_u32, c_dbl_p]),
    ("mdp_loglik_grid_layout", ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_u32, c_dbl_p, c_u32, ctypes.c_int, c_dbl_p]),
    ("mdp_engine_set_grid", ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_u32, c_dbl_p, c_u32]),
    ("mdp_engine_run", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_u32, ctypes.c_void_p]),
    ("mdp_engine_set_layout", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("mdp_engine_set_cbound", ctypes.c_int, [ctypes.c_void_p, ctypes.c_double]),
    ("mdp_engine_set_profiling", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("mdp_engine_kernel_ms", ctypes.c_int, [ctypes.c_void_p, c_dbl_p, ctypes.c_int]),
    ("mdp_engine_time_kernels", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, c_dbl_p, ctypes.c_int]),
    ("mdp_engine_kernel_name", ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_int]),
    ("mdp_engine_work", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_dbl_p, c_dbl_p, c_dbl_p]),
    ("mdp_engine_work_fact", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(Work)]),
    ("mdp_engine_get_info", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(EngineInfo)]),
    ("mdp_engine_launched", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]),
    ("mdp_log_check", ctypes.c_int, [c_dbl_p, c_dbl_p, ctypes.c_size_t]),
    ("mdp_engine_diag_report", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]),
    ("mdp_last_error", ctypes.c_char_p, []),
    ("mdp_abi_version", ctypes.c_int, []),
    ("mdp_device_count", ctypes.c_int, []),
    ("mdp_kgrid", ctypes.c_double, [ctypes.c_uint32, ctypes.c_double, ctypes.c_double, c_dbl_p]),
    ("mdp_dgrid", ctypes.c_double, [ctypes.c_uint32, ctypes.c_double, ctypes.c_double, c_dbl_p]),
    ("mdp_scenario_create", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32, ctypes.c_double, ctypes.c_float, ctypes.c_double,
      ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("mdp_scenario_create_opts", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32, ctypes.c_double, ctypes.c_float, ctypes.c_double,
      ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    ("mdp_scenario_destroy", None, [ctypes.c_void_p]),
    ("mdp_scenario_lik", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_dbl_p, ctypes.c_uint32, c_dbl_p, ctypes.c_uint32, c_dbl_p,
      ctypes.c_uint32, c_dbl_p, ctypes.c_uint32, c_dbl_p]),
    ("mdp_scenario_set_grid", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_dbl_p, ctypes.c_uint32, c_dbl_p, ctypes.c_uint32, c_dbl_p,
      ctypes.c_uint32, c_dbl_p, ctypes.c_uint32]),
    ("mdp_scenario_run", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("mdp_scenario_time_kernels", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, c_dbl_p]),
    ("mdp_future_read_survey", ctypes.c_int,
     [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
      ctypes.POINTER(ctypes.POINTER(ctypes.c_int32))]),
    ("mdp_future_read_posterior", ctypes.c_int,
     [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(c_dbl_p)]),
    ("mdp_free", None, [ctypes.c_void_p]),
    ("mdp_future_create", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32, c_dbl_p, ctypes.c_uint32, ctypes.c_double, ctypes.c_double,
      ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("mdp_future_destroy", None, [ctypes.c_void_p]),
    ("mdp_future_simulate", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
      ctypes.POINTER(ctypes.c_uint64)]),
    ("mdp_future_simulate_device", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
      ctypes.c_void_p]),
    ("mdp_future_check", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("mdp_future_time_kernel", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, c_dbl_p]),
    ("mdp_future_philox", ctypes.c_int,
     [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
]

_lib = None


def lib() -> ctypes.CDLL:
    """Load libmidaspom.so (once).  Raises if the HIP build is missing."""
    global _lib
    if _lib is None:
        path = DIAG_LIB_PATH if os.environ.get("MIDASPOM_DIAG_LIB") == "1" else LIB_PATH
        if not path.exists():
            raise RuntimeError(
                f"{path} is missing: the HIP engine is not built "
                "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
        handle = ctypes.CDLL(str(path), mode=os.RTLD_NOW | ctypes.RTLD_GLOBAL)
        for name, res, args in SIGNATURES:
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int) -> int:
    """Raise MidaspomError on a negative ABI return code."""
    if rc < 0:
        raise MidaspomError(rc, lib().mdp_last_error().decode(errors="replace"))
    return rc


# Engine options (mdp_engine_create_opts).  The library reads
# no environment; the Python layer forwards these variables, when set, as the
# options of engines created without explicit ones -- the developer interface
# the tests and scripts/ use to pin kernel variants against each other.
ENGINE_OPTION_NAMES = (
    "MDP_JIT", "MDP_FUSED", "MDP_FUSED_COLS", "MDP_EPL", "MDP_JIT_SLOTS", "MDP_JIT_WINDOW", "MDP_JIT_XCD",
    "MDP_JIT_EFAST", "MDP_QROWS_XCD", "MDP_FWD", "MDP_WIDE", "MDP_VSPLIT", "MDP_VLDS_EPL", "MDP_VLDS_MAXUSES",
    "MDP_JIT_CHUNK", "MDP_JIT_GATHER", "MDP_QGLOBAL", "MDP_FAST_LOG", "MDP_JIT_KBLOCK", "MDP_WIDE_CB",
    "MDP_JIT_CHECK", "MDP_JIT_DUMP", "MDP_JIT_THREADS", "MDP_JIT_VERBOSE", "MDP_JIT_SPLIT", "MDP_JIT_ROT",
    "MDP_WIDE_MMA", "MDP_HS_RADIX", "MDP_HS_WAVES",
    # measurement-only: accepted by the diag build alone
    "MDP_DIAG", "MDP_JIT_HACK", "MDP_JIT_WPE", "MDP_HS_PROBE")
SCENARIO_OPTION_NAMES = ("MDP_SCN_BIG", "MDP_SCN_ROW")


DIAG_OPTION_NAMES = ("MDP_DIAG", "MDP_JIT_HACK", "MDP_JIT_WPE", "MDP_HS_PROBE")


def options_string(options=None, names=ENGINE_OPTION_NAMES) -> bytes | None:
    """The options argument of mdp_*_create_opts: a dict or "K=V;..." string
    as given, or (None) the MDP_* variables of `names` set in the environment.
    Measurement-only names (DIAG_OPTION_NAMES) are forwarded from the
    environment only to the diag library; with the default library they are
    skipped with a warning -- the C CLIs ignore the environment altogether,
    and a stale variable must not make every engine creation fail.  Passed
    explicitly, the default library refuses them (MDP_EINVAL)."""
    if options is None:
        diag_lib = os.environ.get("MIDASPOM_DIAG_LIB") == "1"
        options = {}
        for k in names:
            if k not in os.environ:
                continue
            if k in DIAG_OPTION_NAMES and not diag_lib:
                import warnings
                warnings.warn(f"{k} is measurement-only (libmidaspom_diag.so): ignored from the environment",
                              RuntimeWarning, stacklevel=3)
                continue
            options[k] = os.environ[k]
    if isinstance(options, dict):
        options = ";".join(f"{k}={v}" for k, v in options.items())
    return options.encode() if options else None
