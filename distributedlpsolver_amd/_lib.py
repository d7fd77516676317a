"""ctypes binding of libdlp.so (include/dlp.h).

The product path is the HIP library; there is no Python or CPU fallback.  If
libdlp.so is missing the import of anything that solves raises
``NativeLibraryMissing`` (build it with ``make`` or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdlp.so")

# status codes (dlp.h)
OK, INFEASIBLE, UNBOUNDED, PIVOT_LIMIT, RUNNING = 0, 1, 2, 3, 4
ERR_ARG, ERR_OOM, ERR_HIP, ERR_RCCL, ERR_NODEVICE, ERR_STATE, ERR_UNSUPPORTED = -1, -2, -3, -4, -5, -6, -7
PRICING_DANTZIG_BLAND, PRICING_BLAND = 0, 1
GEN_DENSE, GEN_DEGENERATE = 0, 1
MINIMIZE, MAXIMIZE = 1, -1
BUF_CAND_SEND, BUF_CAND_RECV, BUF_PROW_SEND, BUF_PROW_RECV = 0, 1, 2, 3
PHASE_RATIO, PHASE_EXCHANGE, PHASE_PROW, PHASE_UPDATE = 0, 1, 2, 3
XCHG_DEFAULT, XCHG_RCCL, XCHG_PEER, XCHG_HOST = 0, 1, 2, 3
NUM_PHASES = 4


class NativeLibraryMissing(RuntimeError):
    pass


class DLPError(RuntimeError):
    def __init__(self, status: int, where: str, msg: str):
        super().__init__(f"{where}: status {status}: {msg}")
        self.status = status


class Options(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("pricing", C.c_int32),
        ("tol_dj", C.c_double),
        ("tol_piv", C.c_double),
        ("max_pivots", C.c_int64),
        ("log_pivots", C.c_int32),
        ("check_interval", C.c_int32),
        ("timing", C.c_int32),
        ("nontemporal", C.c_int32),
        ("rows_per_block", C.c_int32),
        ("use_graph", C.c_int32),
        ("update_variant", C.c_int32),
        ("ld_align", C.c_int32),
        ("small_lp", C.c_int32),
        ("tol_feas", C.c_double),
        ("defer", C.c_int32),
        ("n_gpus", C.c_int32),
        ("lookahead", C.c_int32),
        ("exchange", C.c_int32),
        ("condensed", C.c_int32),
    ]


class Pivot(C.Structure):
    _fields_ = [
        ("q", C.c_int32),
        ("p", C.c_int32),
        ("leaving", C.c_int32),
        ("pad", C.c_int32),
        ("ratio", C.c_double),
        ("objective", C.c_double),
    ]


class Candidate(C.Structure):
    _fields_ = [
        ("ratio", C.c_double),
        ("basis_var", C.c_int32),
        ("row", C.c_int32),
        ("valid", C.c_int32),
        ("pad0", C.c_int32),
        ("pivot", C.c_double),
    ]


class MWOptions(C.Structure):
    _fields_ = [("device", C.c_int32), ("binary", C.c_int32), ("epsilon", C.c_double),
                ("tolerance", C.c_double), ("scale", C.c_double), ("intervals", C.c_int32),
                ("pad_", C.c_int32)]


class MWIter(C.Structure):
    _fields_ = [("dual_value", C.c_double), ("max_infeasibility", C.c_double),
                ("infeasible_advertiser", C.c_int32), ("search_levels", C.c_int32),
                ("min_weight", C.c_double), ("max_weight", C.c_double),
                ("weighted_budget", C.c_double)]


assert C.sizeof(Pivot) == 32 and C.sizeof(Candidate) == 32 and C.sizeof(MWIter) == 48
assert C.sizeof(MWOptions) == 40

_P = C.c_void_p
_I64 = C.c_int64
_I32 = C.c_int32
_DP = C.POINTER(C.c_double)

# (name, restype, argtypes) for every entry point declared in include/dlp.h
SIGNATURES = [
    ("dlp_options_default", None, [C.POINTER(Options)]),
    ("dlp_status_string", C.c_char_p, [C.c_int]),
    ("dlp_last_error", C.c_char_p, []),
    ("dlp_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("dlp_rank_rows", C.c_int, [_I64, C.c_int, C.c_int, C.POINTER(_I64), C.POINTER(_I64)]),
    ("dlp_candidate_select", C.c_int, [C.POINTER(Candidate), C.c_int, C.POINTER(C.c_int)]),
    ("dlp_tableau_ld", _I64, [_I64, _I64]),
    ("dlp_update_variants", C.c_int, []),
    ("dlp_problem_create_dense", C.c_int, [_I64, _I64, _DP, _DP, _DP, C.POINTER(_P)]),
    ("dlp_problem_create_random", C.c_int, [C.c_int, _I64, _I64, C.c_uint64, C.POINTER(_P)]),
    ("dlp_problem_create_adalloc", C.c_int,
     [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.POINTER(_P)]),
    ("dlp_problem_create_general", C.c_int,
     [_I64, _I64, _DP, _DP, _DP, _DP, _DP, _DP, C.c_double, C.c_int, C.POINTER(_P)]),
    ("dlp_problem_create_mps", C.c_int, [C.c_char_p, C.POINTER(_P)]),
    ("dlp_problem_get_general", C.c_int,
     [_P, _DP, _DP, _DP, _DP, _DP, _DP, _DP, C.POINTER(C.c_int)]),
    ("dlp_problem_std_dims", C.c_int,
     [_P, C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_I64)]),
    ("dlp_problem_dims", C.c_int, [_P, C.POINTER(_I64), C.POINTER(_I64)]),
    ("dlp_problem_get_dense", C.c_int, [_P, _DP, _DP, _DP]),
    ("dlp_problem_adalloc_bids", C.c_int,
     [_P, C.POINTER(_I64), C.POINTER(_I32), C.POINTER(_I32), _DP]),
    ("dlp_problem_free", None, [_P]),
    ("dlp_solve", C.c_int, [_P, C.POINTER(Options), C.POINTER(_P)]),
    ("dlp_session_create", C.c_int, [_P, C.POINTER(Options), C.POINTER(_P)]),
    ("dlp_session_create_rank", C.c_int,
     [_P, C.POINTER(Options), C.c_int, C.c_int, C.c_void_p, C.POINTER(_P)]),
    ("dlp_comm_unique_id", C.c_int, [C.c_void_p]),
    ("dlp_session_run", C.c_int, [_P, _I64, C.POINTER(_I64)]),
    ("dlp_session_step_candidate", C.c_int, [_P]),
    ("dlp_session_step_select", C.c_int, [_P]),
    ("dlp_session_step_update", C.c_int, [_P]),
    ("dlp_session_buffer", C.c_int, [_P, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    ("dlp_session_read_buffer", C.c_int, [_P, C.c_int, C.c_void_p, C.c_size_t]),
    ("dlp_session_write_buffer", C.c_int, [_P, C.c_int, C.c_void_p, C.c_size_t]),
    ("dlp_session_sync", C.c_int, [_P]),
    ("dlp_session_status", C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(_I64)]),
    ("dlp_session_timings", C.c_int, [_P, _DP, C.POINTER(_I64)]),
    ("dlp_session_reset_timings", C.c_int, [_P]),
    ("dlp_session_update_stats", C.c_int, [_P, C.POINTER(_I64), _DP, C.POINTER(C.c_int)]),
    ("dlp_session_set_defer_tuning", C.c_int, [_P, C.c_int, C.c_int]),
    ("dlp_session_set_fused_pivot", C.c_int, [_P, C.c_int]),
    ("dlp_session_get_lookahead", C.c_int, [_P, C.POINTER(C.c_int)]),
    ("dlp_session_set_exchange_timeout", C.c_int, [_P, C.c_double]),
    ("dlp_session_abort", C.c_int, [_P]),
    ("dlp_session_inject_fault", C.c_int, [_P, _I64]),
    ("dlp_sessions_connect", C.c_int, [C.POINTER(_P), C.c_int]),
    ("dlp_session_exchange_handle", C.c_int, [_P, C.c_void_p]),
    ("dlp_session_connect_ipc", C.c_int, [_P, C.c_void_p]),
    ("dlp_session_exchange_record", C.c_int, [_P, C.c_void_p]),
    ("dlp_session_connect_records", C.c_int, [_P, C.c_void_p]),
    ("dlp_session_colocated", C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("dlp_session_storage", C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int)]),
    ("dlp_session_set_exchange", C.c_int, [_P, C.c_int]),
    ("dlp_session_get_exchange", C.c_int, [_P, C.POINTER(C.c_int)]),
    ("dlp_session_exchange_reason", C.c_int, [_P, C.c_char_p, C.c_size_t]),
    ("dlp_sessions_run", C.c_int, [C.POINTER(_P), C.c_int, _I64, C.POINTER(_I64)]),
    ("dlp_session_get_defer_tuning", C.c_int,
     [_P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("dlp_session_set_tuning", C.c_int, [_P, C.c_int, C.c_int, C.c_int]),
    ("dlp_session_get_tuning", C.c_int,
     [_P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("dlp_session_small_lp", C.c_int, [_P, C.POINTER(C.c_int)]),
    ("dlp_session_chain_cus", C.c_int, [_P, C.POINTER(C.c_int)]),
    ("dlp_session_info", C.c_int,
     [_P, C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_I64)]),
    ("dlp_session_tableau", C.c_int, [_P, _DP]),
    ("dlp_session_read_rows", C.c_int, [_P, _I64, _I64, _DP]),
    ("dlp_session_result", C.c_int, [_P, C.POINTER(_P)]),
    ("dlp_sessions_result", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(_P)]),
    ("dlp_session_free", None, [_P]),
    ("dlp_mw_options_default", None, [C.POINTER(MWOptions)]),
    ("dlp_mw_create", C.c_int, [_P, C.POINTER(MWOptions), C.POINTER(_P)]),
    ("dlp_mw_run", C.c_int, [_P, C.c_int, C.POINTER(MWIter), _DP]),
    ("dlp_mw_solution", C.c_int, [_P, _DP, _DP, _DP]),
    ("dlp_mw_free", None, [_P]),
    ("dlp_result_status", C.c_int, [_P]),
    ("dlp_result_objective", C.c_double, [_P]),
    ("dlp_result_num_pivots", _I64, [_P]),
    ("dlp_result_x", C.c_int, [_P, _DP, _I64]),
    ("dlp_result_y", C.c_int, [_P, _DP, _I64]),
    ("dlp_result_basis", C.c_int, [_P, C.POINTER(_I32), _I64]),
    ("dlp_result_info", C.c_int, [_P, C.POINTER(_I64), C.POINTER(_I64)]),
    ("dlp_result_pivot_log", C.c_int, [_P, C.POINTER(Pivot), _I64, C.POINTER(_I64)]),
    ("dlp_result_timings", C.c_int, [_P, _DP]),
    ("dlp_result_exchange", C.c_int, [_P, C.POINTER(C.c_int), C.c_char_p, C.c_int64]),
    ("dlp_release_cached_memory", C.c_int, [C.c_int, C.POINTER(C.c_int64)]),
    ("dlp_batched_occupancy", C.c_int, [C.c_int64, C.c_int64, C.c_int, C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("dlp_result_free", None, [_P]),
    ("dlp_batched_solve", C.c_int,
     [C.c_int, _I64, _I64, _I64, C.c_uint64, C.POINTER(Options), _DP, C.POINTER(_I32),
      C.POINTER(_I64), C.POINTER(_I32), C.POINTER(Pivot), _I64, _DP]),
]

_lib = None


def lib() -> C.CDLL:
    """Load libdlp.so (once).  Raises NativeLibraryMissing when it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} not found: build the HIP library with `make` (there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error() -> str:
    msg = lib().dlp_last_error()
    return msg.decode() if msg else ""


def check(status: int, where: str, ok=(OK,)) -> int:
    if status in ok:
        return status
    s = lib().dlp_status_string(status).decode()
    raise DLPError(status, where, f"{s}: {last_error()}")


def default_options(**kw) -> Options:
    o = Options()
    lib().dlp_options_default(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise TypeError(f"unknown option {k}")
        setattr(o, k, v)
    return o
