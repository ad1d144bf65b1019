"""ctypes binding of libpert_hip.so (the C ABI declared in include/pert_hip.h).

There is no fallback: if the shared library is missing or fails to load, every
product entry point raises ``NativeLibraryError``.  Build it with
``python -m scdna_replication_tools_amd.build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_void_p

LIB_NAME = "libpert_hip.so"
DEFAULT_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# A/B measurement hook: PERT_LIB names another build of the same ABI (e.g. a previous
# kernel version compiled by tools/build_ab.sh); the product default is the in-tree build,
# whose provenance lib() checks.
LIB_PATH = os.environ.get("PERT_LIB", DEFAULT_LIB_PATH)

KIND_STEP1, KIND_STEP2, KIND_STEP3 = 1, 2, 3
MODE_STEP, MODE_GRAD, MODE_DECODE = 0, 1, 2
MAX_K1 = 8
MIN_P, MAX_P = 2, 16
BLOCK = 256

# every symbol include/pert_hip.h declares
EXPORTED_SYMBOLS = (
    "pert_make_layout", "pert_workspace_sizes", "pert_auto_bins_per_tile", "pert_enum_pass", "pert_obs_pass",
    "pert_finalize", "pert_adam", "pert_enum_step", "pert_adam_shared", "pert_stream_ceiling", "pert_selftest_nb_lgdiff_host",
    "pert_selftest_nb_lgdiff_device", "pert_selftest_enum_cellbin_host", "pert_selftest_enum_online_host", "pert_tau_binarize", "pert_svi_steps",
    "pert_svi_run", "pert_comm_load", "pert_comm_unique_id", "pert_comm_init", "pert_comm_destroy",
    "pert_comm_allreduce_sum_f64", "pert_svi_steps_sharded", "pert_svi_run_sharded", "pert_version",
    "pert_comm_init_host", "pert_comm_set_watchdog", "pert_comm_abort", "pert_comm_status", "pert_comm_wait_event",
    "pert_comm_inject_fault", "pert_finalize_shared", "pert_finalize_cells", "pert_comm_set_options",
    "pert_comm_overlap", "pert_comm_allreduce_async", "pert_comm_join",
)

# include/pert_hip.h status codes of a sharded fit's communicator
E_COMM_UNAVAILABLE, E_COMM_ABORTED, E_COMM_TIMEOUT, E_COMM_FAULT = 5, 6, 7, 8


class NativeLibraryError(RuntimeError):
    pass


class CommError(RuntimeError):
    """A sharded fit's communicator failed: this rank's collective, or a peer's abort
    (PERT_E_COMM_ABORTED), or a peer that did not arrive in time (PERT_E_COMM_TIMEOUT).
    ``code`` is the library's status."""

    def __init__(self, msg: str, code: int):
        super().__init__(msg)
        self.code = code


class PertLayout(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("off_rho", "off_a", "off_lam", "off_bstds", "off_bmeans",
                                       "n_shared", "off_u", "off_beta", "off_tau", "n_params")]


class PertProblem(ctypes.Structure):
    _fields_ = [
        ("kind", c_int32), ("L", c_int32), ("N", c_int32), ("P", c_int32), ("K1", c_int32),
        ("n_libs", c_int32), ("n_codes", c_int32), ("ldn", c_int32), ("is_root", c_int32),
        ("reads", c_void_p), ("gcf", c_void_p), ("libs", c_void_p), ("eta_code", c_void_p),
        ("eta_table", c_void_p), ("cn_obs", c_void_p), ("rep_obs", c_void_p),
        ("mean_reads", c_void_p), ("ploidy", c_void_p),
        ("lamb", c_float), ("log1m_lam", c_float), ("sum_reads", c_double), ("a_fixed", c_float),
        ("beta_means", c_void_p), ("rho_fixed", c_void_p),
    ]


class PertState(ctypes.Structure):
    _fields_ = [
        ("lay", PertLayout),
        ("params", c_void_p), ("adam_m", c_void_p), ("adam_v", c_void_p),
        ("grad_shared", c_void_p), ("grad_cell", c_void_p),
        ("z_pi", c_void_p), ("m_pi", c_void_p), ("v_pi", c_void_p), ("g_pi", c_void_p),
        ("cn_out", c_void_p), ("rep_out", c_void_p),
        ("cell_part", c_void_p), ("bin_part", c_void_p), ("blk_part", c_void_p),
        ("cellblk_part", c_void_p),
        ("bins_per_tile", c_int32), ("variant", c_int32),
        ("loop_ctl", c_void_p), ("loop_rec", c_void_p), ("loss_offset", c_void_p),
        ("loss_const", c_double), ("rel_tol", c_double), ("min_iter", c_int32), ("step", c_int32),
    ]


class PertTauParams(ctypes.Structure):
    _fields_ = [("first", c_int32), ("lloyd_max_iter", c_int32), ("em_max_iter", c_int32),
                ("q_lo", c_int32 * 5), ("q_hi", c_int32 * 5), ("pad_", c_int32), ("q_t", c_double * 5),
                ("u", c_double * 2), ("tie", c_double), ("pp_margin", c_double), ("fragile", c_double),
                ("em_margin", c_double), ("em_tol", c_double), ("reg_covar", c_double), ("mean_gap", c_double),
                ("early_skew", c_double), ("late_skew", c_double), ("fragile_abs", c_double),
                ("level_margin", c_double), ("eps32", c_double)]


class PertAdamHparams(ctypes.Structure):
    _fields_ = [(n, c_float) for n in ("lr", "beta1", "beta2", "eps", "step_size", "inv_bc2_sqrt")]


_lib = None
_lib_nogil = None


def lib():
    """Load libpert_hip.so once; raise loudly if it is absent, incomplete or stale (its
    embedded source hash differs from the sources of this tree, build.source_hash())."""
    global _lib
    if _lib is None:
        handle = load(LIB_PATH)
        check_provenance(handle)
        _lib = handle
    return _lib


def lib_nogil():
    """The same library bound through ``ctypes.CDLL``: its calls release the interpreter lock.
    For entry points that queue many launches at once (``pert_svi_steps``) or run a whole fit
    (``pert_svi_run``), so another thread of the fit runs Python meanwhile."""
    global _lib_nogil
    if _lib_nogil is None:
        lib()                                   # presence, symbols and provenance checked once
        _lib_nogil = load(LIB_PATH, gil=False)
    return _lib_nogil


def library_source_hash(handle) -> str:
    v = handle.pert_version().decode()
    return v.split("src=", 1)[1] if "src=" in v else ""


def check_provenance(handle):
    """The product library must be built from the sources beside it."""
    from . import build
    if os.path.abspath(LIB_PATH) != DEFAULT_LIB_PATH or not all(os.path.exists(d) for d in build.DEPS):
        return                      # sources not shipped: nothing to compare against
    want, got = build.source_hash(), library_source_hash(handle)
    if got != want:
        raise NativeLibraryError(
            "{} is stale: built from sources {} but the tree's sources hash to {} (rebuild with "
            "`python -m scdna_replication_tools_amd.build`)".format(LIB_PATH, got or "<unknown>", want))


def load(path: str, gil: bool = True):
    """Load and type one build of the C ABI (``lib()`` is the product one; A/B tools load
    a second build beside it).  ``gil=False``: bound through CDLL (calls release the GIL)."""
    # torch first: its bundled libamdhip64 (soname libamdhip64.so.7) must be the one HIP
    # runtime of the process, so our kernels and torch's allocations share a context.
    import torch  # noqa: F401
    if not os.path.exists(path):
        raise NativeLibraryError(
            "{} not found: the PERT HIP extension is not built (run "
            "`python -m scdna_replication_tools_amd.build`). There is no CPU fallback.".format(path))
    try:
        # PyDLL (gil=True): the calls keep the GIL.  Those entry points return in microseconds
        # (launches, no synchronisation), and a thread that drops the GIL around each launch
        # waits for it again behind whatever Python work another thread of the fit is doing.
        # The one entry point that waits on the device, pert_svi_run (a whole fit), and the
        # chunked pert_svi_steps go through the CDLL binding (gil=False, lib_nogil()).
        handle = ctypes.PyDLL(path) if gil else ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover
        raise NativeLibraryError("failed to load {}: {}".format(path, e))
    missing = [s for s in EXPORTED_SYMBOLS if not hasattr(handle, s)]
    if missing:
        raise NativeLibraryError("{} lacks symbols {}".format(LIB_PATH, missing))
    i32, i64 = c_int32, c_int64
    fp = POINTER(c_float)
    handle.pert_make_layout.argtypes = [i32, i32, i32, i32, POINTER(PertLayout)]
    handle.pert_workspace_sizes.argtypes = [i32, i32, i32, i32, i32, i32, POINTER(i64), POINTER(i64),
                                            POINTER(i64), POINTER(i64)]
    handle.pert_auto_bins_per_tile.argtypes = [POINTER(PertProblem), i32, POINTER(i32)]
    handle.pert_enum_pass.argtypes = [POINTER(PertProblem), POINTER(PertState), POINTER(PertAdamHparams),
                                      i32, c_void_p]
    handle.pert_obs_pass.argtypes = [POINTER(PertProblem), POINTER(PertState), c_void_p]
    handle.pert_finalize.argtypes = [POINTER(PertProblem), POINTER(PertState), c_void_p]
    handle.pert_adam.argtypes = [POINTER(PertProblem), POINTER(PertState), POINTER(PertAdamHparams), c_void_p]
    handle.pert_enum_step.argtypes = [POINTER(PertProblem), POINTER(PertState), POINTER(PertAdamHparams), i32,
                                      c_void_p]
    handle.pert_adam_shared.argtypes = [POINTER(PertProblem), POINTER(PertState), POINTER(PertAdamHparams),
                                        c_void_p]
    handle.pert_stream_ceiling.argtypes = [POINTER(PertProblem), POINTER(PertState), c_void_p]
    handle.pert_svi_steps.argtypes = [POINTER(PertProblem), POINTER(PertState), POINTER(PertAdamHparams), fp, fp,
                                      i32, i32, i32, c_void_p, c_void_p]
    handle.pert_svi_run.argtypes = [POINTER(PertProblem), POINTER(PertState), POINTER(PertAdamHparams), fp, fp,
                                    i32, i32, i32, i32, c_void_p, c_void_p, POINTER(i32), c_void_p]
    handle.pert_comm_load.argtypes = [c_char_p]
    handle.pert_comm_unique_id.argtypes = [c_void_p, i32]
    handle.pert_comm_init.argtypes = [c_void_p, i32, i32, i32, POINTER(c_void_p)]
    handle.pert_comm_destroy.argtypes = [c_void_p]
    handle.pert_comm_allreduce_sum_f64.argtypes = [c_void_p, c_void_p, c_void_p, i64, c_void_p]
    handle.pert_comm_init_host.argtypes = [c_char_p, i32, i32, i64, ctypes.c_double, POINTER(c_void_p)]
    handle.pert_comm_set_watchdog.argtypes = [c_void_p, c_char_p, ctypes.c_double]
    handle.pert_comm_abort.argtypes = [c_void_p, i32]
    handle.pert_comm_status.argtypes = [c_void_p]
    handle.pert_comm_wait_event.argtypes = [c_void_p, c_void_p, i32]
    handle.pert_comm_inject_fault.argtypes = [c_void_p, i64]
    handle.pert_comm_set_options.argtypes = [c_void_p, i32, ctypes.c_double]
    handle.pert_comm_overlap.argtypes = [c_void_p]
    handle.pert_comm_allreduce_async.argtypes = [c_void_p, c_void_p, c_void_p, i64, c_void_p]
    handle.pert_comm_join.argtypes = [c_void_p, c_void_p]
    handle.pert_finalize_shared.argtypes = [POINTER(PertProblem), POINTER(PertState), c_void_p]
    handle.pert_finalize_cells.argtypes = [POINTER(PertProblem), POINTER(PertState), c_void_p]
    handle.pert_svi_steps_sharded.argtypes = [POINTER(PertProblem), POINTER(PertState), POINTER(PertAdamHparams), fp,
                                              fp, i32, i32, i32, c_void_p, c_void_p, c_void_p, c_void_p]
    handle.pert_svi_run_sharded.argtypes = [POINTER(PertProblem), POINTER(PertState), POINTER(PertAdamHparams), fp,
                                            fp, i32, i32, i32, i32, c_void_p, c_void_p, c_void_p, c_void_p,
                                            POINTER(i32), c_void_p]
    handle.pert_selftest_nb_lgdiff_host.argtypes = [i64, fp, fp, fp, fp]
    handle.pert_selftest_nb_lgdiff_device.argtypes = [i64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    handle.pert_selftest_enum_cellbin_host.argtypes = [i32, i64, fp, fp, fp, fp, c_float, fp, fp, fp, fp,
                                                       fp, fp, fp, POINTER(i32)]
    handle.pert_selftest_enum_online_host.argtypes = [i32, i64, fp, fp, fp, fp, c_float, fp, fp, fp, fp]
    handle.pert_tau_binarize.argtypes = [i32, i32, c_void_p, POINTER(PertTauParams), c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p]
    handle.pert_version.restype = c_char_p
    for name in EXPORTED_SYMBOLS:
        if name != "pert_version":
            getattr(handle, name).restype = c_int32
    return handle


def check(code: int, what: str):
    if code != 0:
        if code >= 2000:
            raise CommError("{} failed: RCCL error {}".format(what, code - 2000), code)
        if code >= 1000:
            raise RuntimeError("{} failed: HIP error {}".format(what, code - 1000))
        if code == E_COMM_UNAVAILABLE:
            raise NativeLibraryError("{} failed: RCCL is not loaded (pert_comm_load)".format(what))
        if code in (E_COMM_ABORTED, E_COMM_TIMEOUT, E_COMM_FAULT):
            why = {E_COMM_ABORTED: "a rank of the fit failed and aborted it",
                   E_COMM_TIMEOUT: "a rank of the fit did not arrive before the deadline",
                   E_COMM_FAULT: "injected fault (pert_comm_inject_fault)"}[code]
            raise CommError("{} failed: {}".format(what, why), code)
        raise ValueError("{} failed: status {}".format(what, code))


def make_layout(L: int, N: int, K1: int, n_libs: int) -> PertLayout:
    lay = PertLayout()
    check(lib().pert_make_layout(L, N, K1, n_libs, ctypes.byref(lay)), "pert_make_layout")
    return lay


def workspace_sizes(kind: int, L: int, N: int, K1: int, n_libs: int, bins_per_tile: int = 0):
    out = [c_int64() for _ in range(4)]
    check(lib().pert_workspace_sizes(kind, L, N, K1, n_libs, bins_per_tile, *[ctypes.byref(o) for o in out]),
          "pert_workspace_sizes")
    return tuple(int(o.value) for o in out)


def auto_bins_per_tile(prob: PertProblem, variant: int = 0, handle=None) -> int:
    """pert_auto_bins_per_tile: occupancy-aware tile length on the current device."""
    out = c_int32()
    h = lib() if handle is None else handle
    check(h.pert_auto_bins_per_tile(ctypes.byref(prob), int(variant), ctypes.byref(out)),
          "pert_auto_bins_per_tile")
    return int(out.value)


def _fptr(a):
    return a.ctypes.data_as(POINTER(c_float))


def selftest_nb_lgdiff_host(d, x):
    """Host evaluation of pert_math.h nb_lgdiff (test-only)."""
    import numpy as np
    d = np.ascontiguousarray(d, dtype=np.float32)
    x = np.ascontiguousarray(x, dtype=np.float32)
    lam = np.empty_like(d)
    psi = np.empty_like(d)
    check(lib().pert_selftest_nb_lgdiff_host(d.size, _fptr(d), _fptr(x), _fptr(lam), _fptr(psi)),
          "pert_selftest_nb_lgdiff_host")
    return lam, psi


def selftest_enum_cellbin_host(P, x, em1, S1, z, log1m_lam, D, phi):
    """Host evaluation of pert_math.h enum_cellbin (test-only)."""
    import numpy as np
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)
    x, em1, S1, z, D, phi = map(f, (x, em1, S1, z, D, phi))
    n = x.size
    E, dirv, gD, gt = (np.empty(n, np.float32) for _ in range(4))
    gz = np.empty((n, P), np.float32)
    am = np.empty(n, np.int32)
    check(lib().pert_selftest_enum_cellbin_host(P, n, _fptr(x), _fptr(em1), _fptr(S1), _fptr(z),
                                                float(log1m_lam), _fptr(D), _fptr(phi), _fptr(E),
                                                _fptr(dirv), _fptr(gD), _fptr(gt), _fptr(gz),
                                                am.ctypes.data_as(POINTER(c_int32))),
          "pert_selftest_enum_cellbin_host")
    return dict(E=E, dirv=dirv, gD=gD, gt=gt, gz=gz, argmax=am)


def selftest_enum_online_host(P, x, em1, S1, z, log1m_lam, D, phi):
    """Host evaluation of the three-wave pass's arithmetic (enum_online + enum_jmax, test-only)."""
    import numpy as np
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)
    x, em1, S1, z, D, phi = map(f, (x, em1, S1, z, D, phi))
    n = x.size
    E = np.empty(n, np.float32)
    gz = np.empty((n, P), np.float32)
    check(lib().pert_selftest_enum_online_host(P, n, _fptr(x), _fptr(em1), _fptr(S1), _fptr(z), float(log1m_lam),
                                               _fptr(D), _fptr(phi), _fptr(E), _fptr(gz)),
          "pert_selftest_enum_online_host")
    return dict(E=E, gz=gz)
