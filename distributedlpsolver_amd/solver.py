"""Python host API over the C ABI (include/dlp.h).

Mirrors the reference's problem-loading / solver-entry / result surface
(R/instance.h:41-57): ``Problem.adalloc`` regenerates the reference instance
(``Instance(...)`` + ``GenerateInstance()``), ``solve`` replaces
``RunMultiplicativeWeights`` with the exact GPU simplex, and ``Result`` exposes
what the reference keeps in the private ``solution_`` (R/instance.h:34) and
prints as "Dual Value" (R/global_problem.cpp:320-322).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L

STATUS_NAMES = {L.OK: "optimal", L.INFEASIBLE: "infeasible", L.UNBOUNDED: "unbounded",
                L.PIVOT_LIMIT: "pivot limit", L.RUNNING: "running"}

PIVOT_DTYPE = np.dtype([("q", "<i4"), ("p", "<i4"), ("leaving", "<i4"), ("pad", "<i4"),
                        ("ratio", "<f8"), ("objective", "<f8")])
CAND_DTYPE = np.dtype([("ratio", "<f8"), ("basis_var", "<i4"), ("row", "<i4"), ("valid", "<i4"),
                       ("pad0", "<i4"), ("pivot", "<f8")])


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


XREC_BYTES = 256   # include/dlp.h DLP_XREC_BYTES

class Problem:
    """An LP owned by libdlp: dense / random / ad-allocation problems are
    max c^T x s.t. A x <= b, x >= 0 (b >= 0); general problems
    (``Problem.general`` / ``Problem.mps``) have row and column bounds and are
    solved in two phases (include/dlp.h, "general LPs")."""

    def __init__(self, handle: int, kind: str):
        self._h = C.c_void_p(handle)
        self.kind = kind
        m, n = C.c_int64(), C.c_int64()
        L.check(L.lib().dlp_problem_dims(self._h, C.byref(m), C.byref(n)), "dlp_problem_dims")
        self.m, self.n = m.value, n.value

    @classmethod
    def dense(cls, A, b, c) -> "Problem":
        A = np.ascontiguousarray(A, dtype=np.float64)
        b = np.ascontiguousarray(b, dtype=np.float64)
        c = np.ascontiguousarray(c, dtype=np.float64)
        m, n = A.shape
        if b.shape != (m,) or c.shape != (n,):
            raise ValueError("shape mismatch: A (m,n), b (m,), c (n,)")
        h = C.c_void_p()
        L.check(L.lib().dlp_problem_create_dense(m, n, _dptr(A), _dptr(b), _dptr(c), C.byref(h)),
                "dlp_problem_create_dense")
        return cls(h.value, "dense")

    @classmethod
    def random(cls, m: int, n: int, seed: int, degenerate: bool = False) -> "Problem":
        h = C.c_void_p()
        kind = L.GEN_DEGENERATE if degenerate else L.GEN_DENSE
        L.check(L.lib().dlp_problem_create_random(kind, m, n, seed, C.byref(h)),
                "dlp_problem_create_random")
        return cls(h.value, "random")

    @classmethod
    def adalloc(cls, num_advertisers: int, num_impressions: int, num_slots: int = 1,
                bid_sparsity: float = 0.1, scaling_factor: float = 0.25) -> "Problem":
        """The reference's generated instance (R/instance.cpp:32-57), as an exact LP."""
        h = C.c_void_p()
        L.check(L.lib().dlp_problem_create_adalloc(num_advertisers, num_impressions, num_slots,
                                                   bid_sparsity, scaling_factor, C.byref(h)),
                "dlp_problem_create_adalloc")
        p = cls(h.value, "adalloc")
        p.num_advertisers, p.num_impressions = num_advertisers, num_impressions
        return p

    @classmethod
    def general(cls, A, row_lo, row_hi, col_lo, col_hi, c, c0: float = 0.0,
                sense: int = L.MINIMIZE) -> "Problem":
        """min (sense=MINIMIZE) or max c^T x + c0 s.t. row_lo <= A x <= row_hi,
        col_lo <= x <= col_hi; +-inf (or |v| >= 1e30) for missing bounds."""
        c = np.ascontiguousarray(c, dtype=np.float64)
        n = c.shape[0]
        row_lo = np.ascontiguousarray(row_lo, dtype=np.float64)
        row_hi = np.ascontiguousarray(row_hi, dtype=np.float64)
        m = row_lo.shape[0]
        A = np.ascontiguousarray(np.asarray(A, dtype=np.float64).reshape(m, n))
        col_lo = np.ascontiguousarray(np.broadcast_to(np.asarray(col_lo, np.float64), (n,)))
        col_hi = np.ascontiguousarray(np.broadcast_to(np.asarray(col_hi, np.float64), (n,)))
        if row_hi.shape != (m,):
            raise ValueError("row_lo / row_hi must have one entry per row of A")
        h = C.c_void_p()
        L.check(L.lib().dlp_problem_create_general(m, n, _dptr(A), _dptr(row_lo), _dptr(row_hi),
                                                   _dptr(col_lo), _dptr(col_hi), _dptr(c),
                                                   float(c0), int(sense), C.byref(h)),
                "dlp_problem_create_general")
        return cls(h.value, "general")

    @classmethod
    def mps(cls, path: str) -> "Problem":
        """Load a free- or fixed-format MPS file (dlp_problem_create_mps)."""
        h = C.c_void_p()
        L.check(L.lib().dlp_problem_create_mps(str(path).encode(), C.byref(h)),
                "dlp_problem_create_mps")
        return cls(h.value, "general")

    def to_general(self):
        """(A, row_lo, row_hi, col_lo, col_hi, c, c0, sense) of this problem."""
        m, n = self.m, self.n
        A, rl, rh = np.zeros((m, n)), np.zeros(m), np.zeros(m)
        cl, ch, c = np.zeros(n), np.zeros(n), np.zeros(n)
        c0, sense = C.c_double(), C.c_int()
        L.check(L.lib().dlp_problem_get_general(self._h, _dptr(A), _dptr(rl), _dptr(rh), _dptr(cl),
                                                _dptr(ch), _dptr(c), C.byref(c0), C.byref(sense)),
                "dlp_problem_get_general")
        return A, rl, rh, cl, ch, c, c0.value, sense.value

    def std_dims(self):
        """(standard-form rows, tableau columns, priced columns, artificial columns)."""
        v = [C.c_int64() for _ in range(4)]
        L.check(L.lib().dlp_problem_std_dims(self._h, *[C.byref(x) for x in v]),
                "dlp_problem_std_dims")
        return tuple(x.value for x in v)

    def to_dense(self):
        A = np.zeros((self.m, self.n))
        b = np.zeros(self.m)
        c = np.zeros(self.n)
        L.check(L.lib().dlp_problem_get_dense(self._h, _dptr(A), _dptr(b), _dptr(c)),
                "dlp_problem_get_dense")
        return A, b, c

    def adalloc_bids(self):
        nnz = C.c_int64()
        L.check(L.lib().dlp_problem_adalloc_bids(self._h, C.byref(nnz), None, None, None),
                "dlp_problem_adalloc_bids")
        adv = np.zeros(nnz.value, np.int32)
        imp = np.zeros(nnz.value, np.int32)
        bid = np.zeros(nnz.value)
        L.check(L.lib().dlp_problem_adalloc_bids(
            self._h, C.byref(nnz), adv.ctypes.data_as(C.POINTER(C.c_int32)),
            imp.ctypes.data_as(C.POINTER(C.c_int32)), _dptr(bid)), "dlp_problem_adalloc_bids")
        return adv, imp, bid

    def close(self):
        if self._h:
            L.lib().dlp_problem_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class Result:
    status: int
    objective: float
    num_pivots: int
    x: np.ndarray
    y: np.ndarray
    basis: np.ndarray
    pivot_log: np.ndarray
    timings_ms: np.ndarray = field(default_factory=lambda: np.zeros(4))
    phase1_pivots: int = 0
    exchange: int = 0            # dlp_solve(n_gpus): L.XCHG_PEER / L.XCHG_RCCL (0 otherwise)
    exchange_reason: str = ""    # why not the peer exchange (dlp_result_exchange)

    @property
    def status_name(self) -> str:
        return STATUS_NAMES.get(self.status, str(self.status))


def _result_from_handle(h: C.c_void_p, m: int, n: int) -> Result:
    lib = L.lib()
    try:
        x = np.zeros(n)
        y = np.zeros(m)
        mb, p1 = C.c_int64(), C.c_int64()
        L.check(lib.dlp_result_info(h, C.byref(mb), C.byref(p1)), "dlp_result_info")
        basis = np.zeros(mb.value, np.int32)
        L.check(lib.dlp_result_x(h, _dptr(x), n), "dlp_result_x")
        L.check(lib.dlp_result_y(h, _dptr(y), m), "dlp_result_y")
        L.check(lib.dlp_result_basis(h, basis.ctypes.data_as(C.POINTER(C.c_int32)), mb.value),
                "dlp_result_basis")
        cnt = C.c_int64()
        L.check(lib.dlp_result_pivot_log(h, None, 0, C.byref(cnt)), "dlp_result_pivot_log")
        log = np.zeros(cnt.value, PIVOT_DTYPE)
        if cnt.value:
            L.check(lib.dlp_result_pivot_log(h, log.ctypes.data_as(C.POINTER(L.Pivot)), cnt.value,
                                             C.byref(cnt)), "dlp_result_pivot_log")
        tm = np.zeros(L.NUM_PHASES)
        L.check(lib.dlp_result_timings(h, _dptr(tm)), "dlp_result_timings")
        xm, xr = C.c_int(), C.create_string_buffer(512)
        L.check(lib.dlp_result_exchange(h, C.byref(xm), xr, 512), "dlp_result_exchange")
        return Result(status=lib.dlp_result_status(h), objective=lib.dlp_result_objective(h),
                      num_pivots=lib.dlp_result_num_pivots(h), x=x, y=y, basis=basis,
                      pivot_log=log, timings_ms=tm, phase1_pivots=p1.value, exchange=xm.value,
                      exchange_reason=xr.value.decode())
    finally:
        lib.dlp_result_free(h)


def options(**kw) -> L.Options:
    return L.default_options(**kw)


def solve(problem: Problem, **opts) -> Result:
    """One-shot solve (dlp_solve): one GPU, or n_gpus=N devices of this process
    (row-block partition, one host thread + one RCCL rank per device)."""
    o = options(**opts)
    h = C.c_void_p()
    L.check(L.lib().dlp_solve(problem._h, C.byref(o), C.byref(h)), "dlp_solve")
    return _result_from_handle(h, problem.m, problem.n)


class Session:
    """HBM-resident tableau (dlp_session_*): single GPU, or one row-block rank."""

    def __init__(self, problem: Problem, rank: int = 0, nranks: int = 1, rccl_id: bytes | None = None,
                 **opts):
        self.problem = problem
        self.rank, self.nranks = rank, nranks
        self.exchange = nranks > 1 or rccl_id is not None
        self.opts = options(**opts)
        h = C.c_void_p()
        uid = C.create_string_buffer(rccl_id, 128) if rccl_id is not None else None
        L.check(L.lib().dlp_session_create_rank(problem._h, C.byref(self.opts), rank, nranks, uid,
                                                C.byref(h)), "dlp_session_create_rank")
        self._h = h
        rows, first, ld, ncols = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        L.check(L.lib().dlp_session_info(h, C.byref(rows), C.byref(first), C.byref(ld),
                                         C.byref(ncols)), "dlp_session_info")
        self.rows, self.row_first, self.ld, self.ncols = rows.value, first.value, ld.value, ncols.value
        # the tableau as stored: row stride, RHS column, condensed or full
        sld, snc, cond = C.c_int64(), C.c_int64(), C.c_int()
        L.check(L.lib().dlp_session_storage(h, C.byref(sld), C.byref(snc), C.byref(cond)), "dlp_session_storage")
        self.storage_ld, self.storage_ncols, self.condensed = sld.value, snc.value, bool(cond.value)

    def run(self, max_pivots: int) -> tuple[int, int]:
        done = C.c_int64()
        st = L.lib().dlp_session_run(self._h, max_pivots, C.byref(done))
        L.check(st, "dlp_session_run",
                ok=(L.OK, L.INFEASIBLE, L.UNBOUNDED, L.PIVOT_LIMIT, L.RUNNING))
        return st, done.value

    # caller-driven exchange (host-side communicators, see rowblock.py)
    def step_candidate(self) -> np.ndarray:
        L.check(L.lib().dlp_session_step_candidate(self._h), "dlp_session_step_candidate")
        out = np.zeros(1, CAND_DTYPE)
        L.check(L.lib().dlp_session_read_buffer(self._h, L.BUF_CAND_SEND, out.ctypes.data, 32),
                "dlp_session_read_buffer")
        return out

    def step_select(self, gathered: np.ndarray) -> np.ndarray:
        g = np.ascontiguousarray(gathered, dtype=CAND_DTYPE)
        if self.exchange:
            L.check(L.lib().dlp_session_write_buffer(self._h, L.BUF_CAND_RECV, g.ctypes.data,
                                                     g.nbytes), "dlp_session_write_buffer")
        L.check(L.lib().dlp_session_step_select(self._h), "dlp_session_step_select")
        out = np.zeros(self.storage_ld, np.int64)
        L.check(L.lib().dlp_session_read_buffer(self._h, L.BUF_PROW_SEND, out.ctypes.data,
                                                out.nbytes), "dlp_session_read_buffer")
        return out

    def step_update(self, prow_bits: np.ndarray) -> None:
        p = np.ascontiguousarray(prow_bits, dtype=np.int64)
        if self.exchange:
            L.check(L.lib().dlp_session_write_buffer(self._h, L.BUF_PROW_RECV, p.ctypes.data,
                                                     p.nbytes), "dlp_session_write_buffer")
        L.check(L.lib().dlp_session_step_update(self._h), "dlp_session_step_update")

    def status(self) -> tuple[int, int]:
        st, n = C.c_int(), C.c_int64()
        L.check(L.lib().dlp_session_status(self._h, C.byref(st), C.byref(n)), "dlp_session_status")
        return st.value, n.value

    def timings(self) -> tuple[np.ndarray, int]:
        tm = np.zeros(L.NUM_PHASES)
        ns = C.c_int64()
        L.check(L.lib().dlp_session_timings(self._h, _dptr(tm), C.byref(ns)), "dlp_session_timings")
        return tm, ns.value

    def set_tuning(self, update_variant: int, rows_per_block: int = 0, nontemporal: int = 1):
        L.check(L.lib().dlp_session_set_tuning(self._h, update_variant, rows_per_block, nontemporal),
                "dlp_session_set_tuning")

    def get_tuning(self) -> tuple[int, int, int]:
        v, rb, nt = C.c_int(), C.c_int(), C.c_int()
        L.check(L.lib().dlp_session_get_tuning(self._h, C.byref(v), C.byref(rb), C.byref(nt)),
                "dlp_session_get_tuning")
        return v.value, rb.value, nt.value

    def chain_cus(self) -> int:
        """Lookahead: CUs the selection chain's stream runs on (the pass on the rest; 0 = unmasked)."""
        v = C.c_int()
        L.check(L.lib().dlp_session_chain_cus(self._h, C.byref(v)), "dlp_session_chain_cus")
        return v.value

    def small_lp(self) -> bool:
        """True when this session solves in the one-launch LDS path (options.small_lp)."""
        v = C.c_int()
        L.check(L.lib().dlp_session_small_lp(self._h, C.byref(v)), "dlp_session_small_lp")
        return bool(v.value)

    def update_stats(self) -> tuple[int, float, int]:
        """(timed update launches, their total ms, pivots per tableau pass)."""
        n, ms, k = C.c_int64(), C.c_double(), C.c_int()
        L.check(L.lib().dlp_session_update_stats(self._h, C.byref(n), C.byref(ms), C.byref(k)),
                "dlp_session_update_stats")
        return n.value, ms.value, k.value

    def set_fused_pivot(self, on: bool = True):
        """Deferred single-rank sessions: ratio test + selection + pivot row as one launch."""
        L.check(L.lib().dlp_session_set_fused_pivot(self._h, 1 if on else 0),
                "dlp_session_set_fused_pivot")

    def lookahead(self) -> bool:
        """True while block b+1 is selected during the pass of block b (dlp_options.lookahead)."""
        on = C.c_int()
        L.check(L.lib().dlp_session_get_lookahead(self._h, C.byref(on)), "dlp_session_get_lookahead")
        return bool(on.value)

    def set_exchange_timeout(self, seconds: float):
        """RCCL sessions: abort the exchange after `seconds` without progress (0 = never)."""
        L.check(L.lib().dlp_session_set_exchange_timeout(self._h, float(seconds)),
                "dlp_session_set_exchange_timeout")

    def abort(self):
        """Request an abort of the RCCL exchange (any thread): the run returns DLP_ERR_RCCL."""
        L.check(L.lib().dlp_session_abort(self._h), "dlp_session_abort")

    def inject_fault(self, after_polls: int = 0):
        """Tests: the (after_polls + 1)-th window wait fails as if the exchange had died."""
        L.check(L.lib().dlp_session_inject_fault(self._h, int(after_polls)), "dlp_session_inject_fault")

    # owner-rooted peer exchange (include/dlp.h "peer exchange")
    @staticmethod
    def connect_peers(sessions) -> None:
        """Connect the rank sessions of one solve that live in this process
        (dlp_sessions_connect): candidates and the pivot row then travel by direct
        stores into each rank's exchange block.  Ranks that share a device must be
        run together with Session.run_ranks."""
        arr = (C.c_void_p * len(sessions))(*[s._h for s in sessions])
        L.check(L.lib().dlp_sessions_connect(arr, len(sessions)), "dlp_sessions_connect")

    @staticmethod
    def run_ranks(sessions, max_pivots: int) -> tuple[int, int]:
        """dlp_sessions_run: every connected rank from this thread, phase-interleaved."""
        arr = (C.c_void_p * len(sessions))(*[s._h for s in sessions])
        done = C.c_int64()
        st = L.lib().dlp_sessions_run(arr, len(sessions), max_pivots, C.byref(done))
        L.check(st, "dlp_sessions_run", ok=(L.OK, L.INFEASIBLE, L.UNBOUNDED, L.PIVOT_LIMIT, L.RUNNING))
        return st, done.value

    def exchange_handle(self) -> bytes:
        """64-B IPC handle of this rank's exchange block (one process per GPU)."""
        buf = C.create_string_buffer(64)
        L.check(L.lib().dlp_session_exchange_handle(self._h, buf), "dlp_session_exchange_handle")
        return buf.raw

    def connect_ipc(self, handles) -> None:
        """Every rank's exchange_handle(), in rank order (gathered by the caller)."""
        raw = b"".join(handles)
        if len(raw) != 64 * self.nranks:
            raise ValueError("connect_ipc needs nranks 64-byte handles")
        buf = C.create_string_buffer(raw, len(raw))
        L.check(L.lib().dlp_session_connect_ipc(self._h, buf), "dlp_session_connect_ipc")

    def exchange_record(self) -> bytes:
        """This rank's 256-B exchange record: its block's IPC handle and its device's PCI bus id."""
        buf = C.create_string_buffer(XREC_BYTES)
        L.check(L.lib().dlp_session_exchange_record(self._h, buf), "dlp_session_exchange_record")
        return buf.raw

    def connect_records(self, records) -> None:
        """Every rank's exchange_record(), in rank order (gathered by the caller): the peer connect
        that also learns which ranks share this session's device (their chains get disjoint CUs)."""
        raw = b"".join(records)
        if len(raw) != XREC_BYTES * self.nranks:
            raise ValueError("connect_records needs nranks 256-byte records")
        buf = C.create_string_buffer(raw, len(raw))
        L.check(L.lib().dlp_session_connect_records(self._h, buf), "dlp_session_connect_records")

    def colocated(self) -> tuple[int, int]:
        """(ranks of this exchange on this session's device, this rank's index among them)."""
        n, i = C.c_int(), C.c_int()
        L.check(L.lib().dlp_session_colocated(self._h, C.byref(n), C.byref(i)), "dlp_session_colocated")
        return n.value, i.value

    def set_exchange(self, mode: int) -> None:
        """L.XCHG_RCCL or L.XCHG_PEER (PEER over a communicator: an all-gather of IPC handles)."""
        L.check(L.lib().dlp_session_set_exchange(self._h, int(mode)), "dlp_session_set_exchange")

    def get_exchange(self) -> int:
        m = C.c_int()
        L.check(L.lib().dlp_session_get_exchange(self._h, C.byref(m)), "dlp_session_get_exchange")
        return m.value

    def exchange_reason(self) -> str:
        """Why the auto exchange (XCHG_DEFAULT) fell back to RCCL ("" when it did not)."""
        buf = C.create_string_buffer(512)
        L.check(L.lib().dlp_session_exchange_reason(self._h, buf, 512), "dlp_session_exchange_reason")
        return buf.value.decode()

    def set_defer_tuning(self, occupancy: int, form: int = -1):
        """Deferred pass: workgroups/CU cap (0 = none) and form (0 wide, 1/2 narrow x 2/4 rows;
        scalar-coefficient 3 = 1 double x 4 rows, 4 = 2 doubles x 2 rows, 5 = 1 double x 8 rows)."""
        L.check(L.lib().dlp_session_set_defer_tuning(self._h, occupancy, form),
                "dlp_session_set_defer_tuning")

    def get_defer_tuning(self) -> tuple[int, int, int]:
        """(pass workgroups/CU cap, pass form (-1 when eager), pivots per pass K)."""
        occ, form, k = C.c_int(), C.c_int(), C.c_int()
        L.check(L.lib().dlp_session_get_defer_tuning(self._h, C.byref(occ), C.byref(form), C.byref(k)),
                "dlp_session_get_defer_tuning")
        return occ.value, form.value, k.value

    def defer_form(self) -> int:
        return self.get_defer_tuning()[1]

    def reset_timings(self):
        L.check(L.lib().dlp_session_reset_timings(self._h), "dlp_session_reset_timings")

    def tableau(self) -> np.ndarray:
        T = np.zeros((self.rows + 1, self.ld))
        L.check(L.lib().dlp_session_tableau(self._h, _dptr(T)), "dlp_session_tableau")
        return T

    def read_rows(self, first: int, count: int) -> np.ndarray:
        T = np.zeros((count, self.ld))
        L.check(L.lib().dlp_session_read_rows(self._h, first, count, _dptr(T)),
                "dlp_session_read_rows")
        return T

    def result(self) -> Result:
        h = C.c_void_p()
        L.check(L.lib().dlp_session_result(self._h, C.byref(h)), "dlp_session_result")
        return _result_from_handle(h, self.problem.m, self.problem.n)

    @staticmethod
    def merged_result(sessions) -> Result:
        """One result for the rank sessions of a row-block solve that all live in
        this process (dlp_sessions_result): x covers every basic variable."""
        arr = (C.c_void_p * len(sessions))(*[s._h for s in sessions])
        h = C.c_void_p()
        L.check(L.lib().dlp_sessions_result(arr, len(sessions), C.byref(h)), "dlp_sessions_result")
        p = sessions[0].problem
        return _result_from_handle(h, p.m, p.n)

    def close(self):
        if self._h:
            L.lib().dlp_session_free(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class BatchResult:
    objective: np.ndarray
    status: np.ndarray
    num_pivots: np.ndarray
    basis: np.ndarray | None
    logs: np.ndarray | None
    kernel_ms: float


def batched_solve(nlp: int, m: int, n: int, seed: int, degenerate: bool = False,
                  want_basis: bool = False, log_cap: int = 0, **opts) -> BatchResult:
    """C5: nlp independent generated LPs, one LDS-resident workgroup each."""
    o = options(**opts)
    obj = np.zeros(nlp)
    st = np.zeros(nlp, np.int32)
    npv = np.zeros(nlp, np.int64)
    basis = np.zeros((nlp, m), np.int32) if want_basis else None
    logs = np.zeros((nlp, log_cap), PIVOT_DTYPE) if log_cap > 0 else None
    ms = C.c_double()
    L.check(L.lib().dlp_batched_solve(
        L.GEN_DEGENERATE if degenerate else L.GEN_DENSE, nlp, m, n, seed, C.byref(o), _dptr(obj),
        st.ctypes.data_as(C.POINTER(C.c_int32)), npv.ctypes.data_as(C.POINTER(C.c_int64)),
        basis.ctypes.data_as(C.POINTER(C.c_int32)) if basis is not None else None,
        logs.ctypes.data_as(C.POINTER(L.Pivot)) if logs is not None else None, log_cap,
        C.byref(ms)), "dlp_batched_solve")
    return BatchResult(obj, st, npv, basis, logs, ms.value)


def batched_occupancy(m: int, n: int, device: int = 0) -> dict:
    """dlp_batched_occupancy: the batch kernel's lanes per LP and LPs resident per CU."""
    a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
    L.check(L.lib().dlp_batched_occupancy(m, n, device, C.byref(a), C.byref(b), C.byref(c)),
            "dlp_batched_occupancy")
    return {"lps_per_cu": a.value, "threads_per_lp": b.value, "register_kernel": bool(c.value)}


MW_ITER_DTYPE = np.dtype([("dual_value", "<f8"), ("max_infeasibility", "<f8"),
                          ("infeasible_advertiser", "<i4"), ("search_levels", "<i4"), ("min_weight", "<f8"),
                          ("max_weight", "<f8"), ("weighted_budget", "<f8")])


class MW:
    """The reference's multiplicative-weights loop on the GPU (dlp_mw_*):
    replaces Instance::RunMultiplicativeWeights(T, tol, binary[, scale,
    intervals]), R/instance.cpp:117-141.  binary=False is sort mode
    (R/global_problem.cpp:224-255), binary=True the threshold search
    (R/global_problem.cpp:46-222) that R/main.cpp:36 runs; scale=None derives
    cr_transition_scale = 1 - epsilon * 0.001 (R/main.cpp:38).  Needs a
    Problem.adalloc problem."""

    def __init__(self, problem: Problem, epsilon: float = 0.01, tolerance: float = 1e-18,
                 device: int = 0, binary: bool = False, scale: float | None = None,
                 intervals: int = 3):
        o = L.MWOptions()
        L.lib().dlp_mw_options_default(C.byref(o))
        o.epsilon, o.tolerance, o.device = epsilon, tolerance, device
        o.binary, o.intervals = (1 if binary else 0), intervals
        o.scale = 0.0 if scale is None else scale
        self.problem = problem
        h = C.c_void_p()
        L.check(L.lib().dlp_mw_create(problem._h, C.byref(o), C.byref(h)), "dlp_mw_create")
        self._h = h

    def run(self, iterations: int):
        """Run iterations; returns (per-iteration log array, device ms)."""
        log = np.zeros(iterations, MW_ITER_DTYPE)
        ms = C.c_double()
        L.check(L.lib().dlp_mw_run(self._h, iterations, log.ctypes.data_as(C.POINTER(L.MWIter)),
                                   C.byref(ms)), "dlp_mw_run")
        return log, ms.value

    def solution(self, current: bool = False):
        """(averaged x in the problem's variable order, advertiser weights); with
        current=True also the last iteration's x: (x_avg, weights, x_current)."""
        x = np.zeros(self.problem.n)
        xc = np.zeros(self.problem.n) if current else None
        w = np.zeros(self.problem.num_advertisers)
        L.check(L.lib().dlp_mw_solution(self._h, _dptr(x), _dptr(xc) if current else None, _dptr(w)),
                "dlp_mw_solution")
        return (x, w, xc) if current else (x, w)

    def close(self):
        if self._h:
            L.lib().dlp_mw_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rank_rows(m: int, rank: int, nranks: int) -> tuple[int, int]:
    first, count = C.c_int64(), C.c_int64()
    L.check(L.lib().dlp_rank_rows(m, rank, nranks, C.byref(first), C.byref(count)), "dlp_rank_rows")
    return first.value, count.value


def candidate_select(cands: np.ndarray) -> int:
    c = np.ascontiguousarray(cands, dtype=CAND_DTYPE)
    w = C.c_int()
    L.check(L.lib().dlp_candidate_select(c.ctypes.data_as(C.POINTER(L.Candidate)), len(c),
                                         C.byref(w)), "dlp_candidate_select")
    return w.value


def tableau_ld(m: int, n: int) -> int:
    return int(L.lib().dlp_tableau_ld(m, n))


def device_count() -> int:
    n = C.c_int()
    L.check(L.lib().dlp_device_count(C.byref(n)), "dlp_device_count")
    return n.value


def release_cached_memory(device: int = -1) -> int:
    """Free the buffers finished sessions left in the per-process cache (-1: every device);
    returns the bytes freed (dlp_release_cached_memory)."""
    n = C.c_int64()
    L.check(L.lib().dlp_release_cached_memory(int(device), C.byref(n)), "dlp_release_cached_memory")
    return n.value


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    L.check(L.lib().dlp_comm_unique_id(buf), "dlp_comm_unique_id")
    return buf.raw
