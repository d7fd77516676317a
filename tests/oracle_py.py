"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so (the CPU
restatement of the pivot rule, oracle/oracle.h).  Imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg only — never by the
product package."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

PIVOT_DTYPE = np.dtype([("q", "<i4"), ("p", "<i4"), ("leaving", "<i4"), ("pad", "<i4"),
                        ("ratio", "<f8"), ("objective", "<f8")])
CAND_DTYPE = np.dtype([("ratio", "<f8"), ("basis_var", "<i4"), ("row", "<i4"), ("valid", "<i4"),
                       ("pad0", "<i4"), ("pivot", "<f8")])


class Opts(C.Structure):
    _fields_ = [("pricing", C.c_int32), ("tol_dj", C.c_double), ("tol_piv", C.c_double),
                ("max_pivots", C.c_int64), ("nthreads", C.c_int32)]


_lib = None
_D = C.POINTER(C.c_double)
_I32 = C.POINTER(C.c_int32)
_I64 = C.POINTER(C.c_int64)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_PATH):
            raise RuntimeError(f"{ORACLE_PATH} missing: run `make -C oracle`")
        L = C.CDLL(ORACLE_PATH)
        L.oracle_gen_dense.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_uint64, _D, _D, _D]
        L.oracle_gen_tableau.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_uint64, C.c_int64,
                                         C.c_int64, C.c_int64, _D, C.c_int32]
        L.oracle_ld.restype = C.c_int64
        L.oracle_ld.argtypes = [C.c_int64, C.c_int64]
        L.oracle_gen_adalloc.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, _I64, _I32,
                                         _I32, _D, _D, _I32, _D]
        L.oracle_solve_dense.argtypes = [C.c_int64, C.c_int64, _D, _D, _D, C.POINTER(Opts), _D, _D,
                                         _D, _I32, C.c_void_p, C.c_int64, _I64, C.POINTER(C.c_int)]
        L.oracle_slice_create.argtypes = [C.c_int64, C.c_int64, _D, _D, _D, C.c_int64, C.c_int64,
                                          C.POINTER(Opts), C.POINTER(C.c_void_p)]
        L.oracle_slice_candidate.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        L.oracle_slice_select.argtypes = [C.c_void_p, C.c_void_p, C.c_int, _I64, C.POINTER(C.c_int)]
        L.oracle_slice_update.argtypes = [C.c_void_p, _I64]
        L.oracle_slice_ld.restype = C.c_int64
        L.oracle_slice_ld.argtypes = [C.c_void_p]
        L.oracle_slice_npivots.restype = C.c_int64
        L.oracle_slice_npivots.argtypes = [C.c_void_p]
        L.oracle_slice_log.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.oracle_slice_tableau.argtypes = [C.c_void_p, _D]
        L.oracle_slice_free.argtypes = [C.c_void_p]
        L.oracle_bench_pivots.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_uint64, C.c_int64,
                                          C.c_int64, C.c_int32, _D, _I64, _D]
        L.oracle_run_generated.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_uint64, C.c_int64,
                                           C.c_int32, C.c_void_p, _I64, _I64, C.c_int64, _D, _I32]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(_D)


def gen_dense(m, n, seed, degenerate=False):
    A = np.zeros((m, n))
    b = np.zeros(m)
    c = np.zeros(n)
    rc = lib().oracle_gen_dense(1 if degenerate else 0, m, n, seed, _d(A), _d(b), _d(c))
    assert rc == 0
    return A, b, c


def ld(m, n):
    return int(lib().oracle_ld(m, n))


def gen_tableau(m, n, seed, degenerate=False, row_first=0, row_count=None, nthreads=4):
    row_count = m - row_first if row_count is None else row_count
    L_ = ld(m, n)
    T = np.zeros((row_count + 1, L_))
    rc = lib().oracle_gen_tableau(1 if degenerate else 0, m, n, seed, row_first, row_count, L_,
                                  _d(T), nthreads)
    assert rc == 0
    return T


def gen_adalloc(A, I, sparsity=0.1, scaling=0.25):
    nnz = C.c_int64()
    rc = lib().oracle_gen_adalloc(A, I, sparsity, scaling, C.byref(nnz), None, None, None, None,
                                  None, None)
    assert rc == 0
    adv = np.zeros(nnz.value, np.int32)
    imp = np.zeros(nnz.value, np.int32)
    bid = np.zeros(nnz.value)
    budgets = np.zeros(A)
    draws = np.zeros(A, np.int32)
    mb = C.c_double()
    rc = lib().oracle_gen_adalloc(A, I, sparsity, scaling, C.byref(nnz),
                                  adv.ctypes.data_as(_I32), imp.ctypes.data_as(_I32), _d(bid),
                                  _d(budgets), draws.ctypes.data_as(_I32), C.byref(mb))
    assert rc == 0
    return dict(adv=adv, imp=imp, bid=bid, budgets=budgets, draws=draws, max_bid=mb.value)


def adalloc_lp(A, I, sparsity=0.1, scaling=0.25):
    """Dense LP of the ad-allocation instance: rows [0,A) budgets, [A,A+I) assignment."""
    g = gen_adalloc(A, I, sparsity, scaling)
    nnz = len(g["bid"])
    M = np.zeros((A + I, nnz))
    M[g["adv"], np.arange(nnz)] = g["bid"]
    M[A + g["imp"], np.arange(nnz)] = 1.0
    b = np.concatenate([g["budgets"], np.ones(I)])
    return M, b, g["bid"].copy()


class Solution:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def solve_dense(A, b, c, pricing=0, tol_dj=1e-9, tol_piv=1e-9, max_pivots=1_000_000, nthreads=4,
                log_cap=None):
    A = np.ascontiguousarray(A, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    c = np.ascontiguousarray(c, dtype=np.float64)
    m, n = A.shape
    o = Opts(pricing, tol_dj, tol_piv, max_pivots, nthreads)
    x = np.zeros(n)
    y = np.zeros(m)
    obj = C.c_double()
    basis = np.zeros(m, np.int32)
    cap = max_pivots if log_cap is None else log_cap
    cap = min(cap, 2_000_000)
    log = np.zeros(cap, PIVOT_DTYPE)
    npiv = C.c_int64()
    st = C.c_int()
    rc = lib().oracle_solve_dense(m, n, _d(A), _d(b), _d(c), C.byref(o), _d(x), _d(y), C.byref(obj),
                                  basis.ctypes.data_as(_I32), log.ctypes.data, cap, C.byref(npiv),
                                  C.byref(st))
    assert rc == 0, "oracle_solve_dense rejected the problem"
    return Solution(status=st.value, objective=obj.value, x=x, y=y, basis=basis,
                    pivot_log=log[:min(npiv.value, cap)], num_pivots=npiv.value)


class OracleEngine:
    """A simulated rank (oracle row slice) with the rowblock engine interface."""

    def __init__(self, A, b, c, rank, nranks, row_first, row_count, pricing=0, tol_dj=1e-9,
                 tol_piv=1e-9):
        A = np.ascontiguousarray(A, dtype=np.float64)
        m, n = A.shape
        self._keep = (A, np.ascontiguousarray(b, float), np.ascontiguousarray(c, float))
        o = Opts(pricing, tol_dj, tol_piv, 1 << 40, 1)
        h = C.c_void_p()
        rc = lib().oracle_slice_create(m, n, _d(self._keep[0]), _d(self._keep[1]),
                                       _d(self._keep[2]), row_first, row_count, C.byref(o),
                                       C.byref(h))
        assert rc == 0
        self.h = h
        self.ld = int(lib().oracle_slice_ld(h))
        self.state = 4  # running

    def step_candidate(self):
        cand = np.zeros(1, CAND_DTYPE)
        opt = C.c_int()
        lib().oracle_slice_candidate(self.h, cand.ctypes.data, C.byref(opt))
        if opt.value:
            self.state = 0
        return cand

    def step_select(self, gathered):
        g = np.ascontiguousarray(gathered, dtype=CAND_DTYPE)
        out = np.zeros(self.ld, np.int64)
        unb = C.c_int()
        lib().oracle_slice_select(self.h, g.ctypes.data, len(g), out.ctypes.data_as(_I64),
                                  C.byref(unb))
        if unb.value:
            self.state = 2
        return out

    def step_update(self, prow_bits):
        p = np.ascontiguousarray(prow_bits, dtype=np.int64)
        lib().oracle_slice_update(self.h, p.ctypes.data_as(_I64))

    def status(self):
        return self.state, int(lib().oracle_slice_npivots(self.h))

    def log(self):
        n = int(lib().oracle_slice_npivots(self.h))
        out = np.zeros(n, PIVOT_DTYPE)
        lib().oracle_slice_log(self.h, out.ctypes.data, n)
        return out

    def close(self):
        if self.h:
            lib().oracle_slice_free(self.h)
            self.h = None


def bench_pivots(m, n, seed, warmup, k, nthreads, degenerate=False):
    secs = C.c_double()
    gen = C.c_double()
    done = C.c_int64()
    rc = lib().oracle_bench_pivots(1 if degenerate else 0, m, n, seed, warmup, k, nthreads,
                                   C.byref(secs), C.byref(done), C.byref(gen))
    assert rc == 0, f"oracle_bench_pivots rc={rc}"
    return secs.value, done.value, gen.value


def bench_windows(m, n, seed, runs, gen_threads, degenerate=False):
    """runs = [(threads, max_pivots, budget_seconds), ...] on one generated LP
    (oracle_bench_windows).  Returns ([(seconds, pivots), ...], generation seconds)."""
    L = lib()
    if not getattr(L, "_bw_bound", False):
        L.oracle_bench_windows.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_uint64, C.c_int32,
                                           C.c_int, _I32, _I64, _D, _D, _I64, _D]
        L._bw_bound = True
    thr = np.array([r[0] for r in runs], np.int32)
    kmax = np.array([r[1] for r in runs], np.int64)
    bud = np.array([r[2] for r in runs], np.float64)
    secs = np.zeros(len(runs))
    done = np.zeros(len(runs), np.int64)
    gen = C.c_double()
    rc = L.oracle_bench_windows(1 if degenerate else 0, m, n, seed, gen_threads, len(runs),
                                thr.ctypes.data_as(_I32), kmax.ctypes.data_as(_I64), _d(bud),
                                _d(secs), done.ctypes.data_as(_I64), C.byref(gen))
    assert rc == 0, f"oracle_bench_windows rc={rc}"
    return [(float(s), int(k)) for s, k in zip(secs, done)], gen.value


def bench_windows_defer(m, n, seed, K, runs, gen_threads, degenerate=False):
    """bench_windows with the deferred rank-K algorithm (oracle/oracle_defer.inc): windows of
    whole K-pivot blocks, each pass applied.  Returns ([(seconds, pivots), ...], generation s)."""
    L = lib()
    if not getattr(L, "_bwd_bound", False):
        L.oracle_bench_windows_defer.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_uint64, C.c_int32,
                                                 C.c_int, C.c_int, _I32, _I64, _D, _D, _I64, _D]
        L._bwd_bound = True
    thr = np.array([r[0] for r in runs], np.int32)
    kmax = np.array([r[1] for r in runs], np.int64)
    bud = np.array([r[2] for r in runs], np.float64)
    secs = np.zeros(len(runs))
    done = np.zeros(len(runs), np.int64)
    gen = C.c_double()
    rc = L.oracle_bench_windows_defer(1 if degenerate else 0, m, n, seed, gen_threads, K, len(runs),
                                      thr.ctypes.data_as(_I32), kmax.ctypes.data_as(_I64), _d(bud),
                                      _d(secs), done.ctypes.data_as(_I64), C.byref(gen))
    assert rc == 0, f"oracle_bench_windows_defer rc={rc}"
    return [(float(s), int(k)) for s, k in zip(secs, done)], gen.value


def run_generated_defer(m, n, seed, K, k, degenerate=False, nthreads=8):
    """k pivots of the deferred rank-K restatement on the generated tableau: (log, whole
    (m+1) x ld tableau after the last pass, basis)."""
    L = lib()
    if not getattr(L, "_rgd_bound", False):
        L.oracle_run_generated_defer.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_uint64, C.c_int,
                                                 C.c_int64, C.c_int32, C.c_void_p, C.POINTER(C.c_int64),
                                                 _D, _I32]
        L._rgd_bound = True
    log = np.zeros(k, PIVOT_DTYPE)
    npiv = C.c_int64()
    T = np.zeros((m + 1, ld(m, n)))
    basis = np.zeros(m, np.int32)
    rc = L.oracle_run_generated_defer(1 if degenerate else 0, m, n, seed, K, k, nthreads, log.ctypes.data,
                                      C.byref(npiv), _d(T), basis.ctypes.data_as(_I32))
    assert rc == 0, f"oracle_run_generated_defer rc={rc}"
    return log[:npiv.value], T, basis


def mw_scale(epsilon=0.01):
    """R/main.cpp:38 cr_transition_scale = 1 - epsilon * 0.001 in x87 long double, to fp64."""
    return float(np.longdouble(1) - np.longdouble(epsilon) * np.longdouble(0.001))


def mw_run(A, I, sparsity=0.1, scaling=0.25, epsilon=0.01, T=300, tol=1e-18, binary=False,
           scale=None, intervals=3):
    """fp64 MW spec (oracle/oracle_mw.cpp), sort or binary mode.  Returns a dict of
    per-iteration arrays (binary mode adds search `levels` and the final `interval`)."""
    L = lib()
    if not getattr(L, "_mw_bound", False):
        L.oracle_mw_run_mode.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                         C.c_int, C.c_double, C.c_int, C.c_double, C.c_int, _D, _D,
                                         _I32, _D, _D, _D, _D, _D, _I64, _I32, _D]
        L.oracle_sum_blocked.restype = C.c_double
        L.oracle_sum_blocked.argtypes = [_D, C.c_int64]
        L.oracle_dexp.restype = C.c_double
        L.oracle_dexp.argtypes = [C.c_double]
        L.oracle_sum_fixed.restype = C.c_double
        L.oracle_sum_fixed.argtypes = [_D, C.c_int64]
        L._mw_bound = True
    nnz = len(gen_adalloc(A, I, sparsity, scaling)["bid"])
    out = {k: np.zeros(T) for k in ("dual", "infeas", "wmin", "wmax", "budget")}
    idx = np.zeros(T, np.int32)
    xa = np.zeros(nnz)
    w = np.zeros(A)
    n = C.c_int64()
    levels = np.zeros(T, np.int32)
    interval = np.zeros((T, 2))
    if scale is None:
        scale = mw_scale(epsilon)
    rc = L.oracle_mw_run_mode(A, I, sparsity, scaling, epsilon, T, tol, 1 if binary else 0,
                              scale, intervals, _d(out["dual"]), _d(out["infeas"]),
                              idx.ctypes.data_as(_I32), _d(out["wmin"]), _d(out["wmax"]),
                              _d(out["budget"]), _d(xa), _d(w), C.byref(n),
                              levels.ctypes.data_as(_I32), _d(interval))
    assert rc == 0
    out.update(infeas_idx=idx, x_avg=xa, weights=w, nnz=n.value)
    if binary:
        out.update(levels=levels, interval=interval)
    return out


def dexp(x):
    L = lib()
    if not getattr(L, "_mw_bound", False):
        mw_run(2, 10, 0.5, 0.25, 0.01, 1)
    return L.oracle_dexp(x)


def run_generated(m, n, seed, k, rows, degenerate=False, nthreads=8):
    """k oracle pivots on the generated tableau; returns (log, sampled rows, basis)."""
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    log = np.zeros(k, PIVOT_DTYPE)
    npiv = C.c_int64()
    out = np.zeros((len(rows), ld(m, n)))
    basis = np.zeros(m, np.int32)
    rc = lib().oracle_run_generated(1 if degenerate else 0, m, n, seed, k, nthreads, log.ctypes.data,
                                    C.byref(npiv), rows.ctypes.data_as(_I64), len(rows), _d(out),
                                    basis.ctypes.data_as(_I32))
    assert rc == 0
    return log[:npiv.value], out, basis


STOP_CB = C.CFUNCTYPE(None, C.c_int64, C.POINTER(C.c_double), C.c_int64, C.c_int64, C.c_void_p,
                      C.POINTER(C.c_int32), C.c_void_p)


def run_generated_stops(m, n, seed, stops, fn, degenerate=False, nthreads=8):
    """Pivot the generated LP through the ascending `stops`; at each one call
    fn(npivots, T, log, basis) with zero-copy views of the oracle's whole
    tableau ((m+1) x ld, objective row last), its pivot log and basis."""
    L = lib()
    if not getattr(L, "_stops_bound", False):
        L.oracle_run_generated_stops.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_uint64, C.c_int32,
                                                 _I64, C.c_int, STOP_CB, C.c_void_p]
        L._stops_bound = True
    errs = []

    def _cb(k, T, ld_, rows, logp, basisp, _user):
        try:
            Tv = np.ctypeslib.as_array(T, shape=(rows, ld_))
            lg = np.frombuffer((C.c_char * (32 * k)).from_address(logp), dtype=PIVOT_DTYPE) if k else \
                np.zeros(0, PIVOT_DTYPE)
            bs = np.ctypeslib.as_array(basisp, shape=(m,))
            fn(int(k), Tv, lg, bs)
        except Exception as e:  # noqa: BLE001 - re-raised after the C call returns
            errs.append(e)

    cb = STOP_CB(_cb)
    st = np.ascontiguousarray(stops, dtype=np.int64)
    rc = L.oracle_run_generated_stops(1 if degenerate else 0, m, n, seed, nthreads,
                                      st.ctypes.data_as(_I64), len(st), cb, None)
    if errs:
        raise errs[0]
    assert rc == 0, f"oracle_run_generated_stops rc={rc}"


# ---- general LPs (include/dlp.h "general LPs", oracle/oracle_general.inc)
INF = float("inf")


class GeneralLP:
    """min/max c^T x + c0 s.t. row_lo <= A x <= row_hi, col_lo <= x <= col_hi (sense 1 = min)."""

    def __init__(self, A, row_lo, row_hi, col_lo, col_hi, c, c0=0.0, sense=1):
        self.A = np.ascontiguousarray(A, dtype=np.float64).reshape(len(row_lo), len(c))
        self.row_lo = np.ascontiguousarray(row_lo, dtype=np.float64)
        self.row_hi = np.ascontiguousarray(row_hi, dtype=np.float64)
        self.col_lo = np.ascontiguousarray(col_lo, dtype=np.float64)
        self.col_hi = np.ascontiguousarray(col_hi, dtype=np.float64)
        self.c = np.ascontiguousarray(c, dtype=np.float64)
        self.c0, self.sense = float(c0), int(sense)
        self.m, self.n = self.A.shape

    def args(self):
        return (self.m, self.n, _d(self.A), _d(self.row_lo), _d(self.row_hi), _d(self.col_lo),
                _d(self.col_hi), _d(self.c), self.c0, self.sense)


def _bind_general(L):
    if getattr(L, "_gen_bound", False):
        return
    base = [C.c_int64, C.c_int64, _D, _D, _D, _D, _D, _D, C.c_double, C.c_int]
    L.oracle_general_std_dims.argtypes = base + [_I64, _I64, _I64, _I64]
    L.oracle_solve_general.argtypes = base + [C.POINTER(Opts), C.c_double, _D, _D, _D, _I32,
                                              C.c_int64, C.c_void_p, C.c_int64, _I64, _I64,
                                              C.POINTER(C.c_int)]
    L._gen_bound = True


def general_std_dims(lp: GeneralLP):
    L = lib()
    _bind_general(L)
    v = [C.c_int64() for _ in range(4)]
    rc = L.oracle_general_std_dims(*lp.args(), *[C.byref(x) for x in v])
    assert rc == 0, rc
    return tuple(x.value for x in v)


def solve_general(lp: GeneralLP, pricing=0, tol_dj=1e-9, tol_piv=1e-9, tol_feas=1e-9,
                  max_pivots=1_000_000, nthreads=1, log_cap=200_000):
    L = lib()
    _bind_general(L)
    m_std, _, _, _ = general_std_dims(lp)
    o = Opts(pricing, tol_dj, tol_piv, max_pivots, nthreads)
    x = np.zeros(lp.n)
    y = np.zeros(lp.m)
    obj = C.c_double()
    basis = np.zeros(m_std, np.int32)
    log = np.zeros(log_cap, PIVOT_DTYPE)
    npiv, p1 = C.c_int64(), C.c_int64()
    st = C.c_int()
    rc = L.oracle_solve_general(*lp.args(), C.byref(o), tol_feas, _d(x), _d(y), C.byref(obj),
                                basis.ctypes.data_as(_I32), m_std, log.ctypes.data, log_cap,
                                C.byref(npiv), C.byref(p1), C.byref(st))
    assert rc == 0, rc
    return Solution(status=st.value, objective=obj.value, x=x, y=y, basis=basis,
                    pivot_log=log[:min(npiv.value, log_cap)], num_pivots=npiv.value,
                    phase1_pivots=p1.value)
