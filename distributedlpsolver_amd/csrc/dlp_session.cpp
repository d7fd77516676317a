// dlp_session.cpp — host runtime behind the C ABI (include/dlp.h): problem
// objects, the HBM-resident tableau session, the pivot loop with device-side
// decisions (no host round trip per pivot), RCCL row-block exchange, results.
//
// Replaces the reference's solver entry and result store:
//   Instance::RunMultiplicativeWeights  R/instance.cpp:117-134  -> dlp_solve
//   AllocationMW::RunAllocationMW loop  R/allocation_mw.cpp:271-326 -> dlp_session_run
//   Instance::solution_                 R/instance.h:34 -> dlp_result_x / _y
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "dlp_host.h"
#include "dlp_internal.h"

namespace dlp {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace dlp

using dlp::set_error;

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                \
            return DLP_ERR_HIP;                                                          \
        }                                                                                \
    } while (0)

#define NCCL_TRY(expr)                                                                   \
    do {                                                                                 \
        ncclResult_t r_ = (expr);                                                        \
        if (r_ != ncclSuccess) {                                                         \
            set_error(std::string(#expr) + ": " + ncclGetErrorString(r_));               \
            return DLP_ERR_RCCL;                                                         \
        }                                                                                \
    } while (0)

#define CALL_TRY(expr)                                                                   \
    do {                                                                                 \
        int rc_ = (expr);                                                                \
        if (rc_ != DLP_OK) return rc_;                                                   \
    } while (0)

struct dlp_session {
    dlp_options opt{};
    int device = 0, rank = 0, nranks = 1;
    int64_t m = 0, n = 0, N = 0, ld = 0, width = 0, row_first = 0, rows = 0;
    bool streaming = false;         // tableau >> Infinity Cache (auto-tuning regime)
    hipStream_t stream = nullptr;
    dlp::Geometry g{};
    double* T = nullptr;
    double* colq = nullptr;
    int64_t* prow_send = nullptr;
    int64_t* prow_recv = nullptr;   // == prow_send when nranks == 1
    dlp::Cand* partials = nullptr;
    int ratio_blocks = 0;
    int ratio_blocks_max = 0;       // partials capacity (eager or deferred ratio kernel)
    dlp::Cand* cand_send = nullptr;
    dlp::Cand* cand_recv = nullptr;
    dlp::PricePart* pp = nullptr;
    int32_t* basis = nullptr;
    dlp::DevState* st = nullptr;
    dlp_pivot* log = nullptr;
    int64_t log_cap = 0;
    dlp::DevState* host_st = nullptr;   // pinned
    ncclComm_t comm = nullptr;
    bool use_rccl = false;
    // how the exchange travels (exchange sessions): X_HOST = the caller (step API),
    // X_RCCL = all-gather + MAX all-reduce, X_PEER = direct stores into the ranks'
    // exchange blocks (dlp_sessions_connect / dlp_session_connect_ipc /
    // dlp_session_set_exchange)
    enum XMode { X_RCCL = DLP_XCHG_RCCL, X_PEER = DLP_XCHG_PEER, X_HOST = DLP_XCHG_HOST };
    int xmode = X_HOST;
    uint64_t* xblk = nullptr;            // this rank's exchange block (uncached device memory)
    bool xblk_uncached = false;
    dlp::XPeers* xpeers = nullptr;       // device copy of the peer table (X_PEER)
    dlp::XPeers xpeers_host{};
    std::vector<void*> ipc_open;         // peers' blocks opened through IPC
    uint32_t* xabort = nullptr;          // pinned host word the device waits read (abort)
    uint32_t xseq_c = 0, xseq_r = 0;     // exchange counters, identical on every rank
    // failure containment on the exchange path: a window's wait polls the
    // stream, the communicator's async error, the caller's / the in-process group's abort
    // word and a stall limit, and aborts the communicator instead of blocking forever
    std::atomic<int> abort_req{0};               // dlp_session_abort (any thread)
    std::atomic<int>* group_failed = nullptr;    // solve_in_process: the first failed rank, -1
    double stall_limit_s = 600.0;                // dlp_session_set_exchange_timeout (0 = none)
    int64_t fault_after_polls = -1;              // dlp_session_inject_fault (tests)
    int64_t npolls = 0;
    // deferred, single rank: one launch for ratio + selection + pivot row (opt-in: measured
    // equal to two launches, C2 24.7 vs 25.0 us/pivot, profiles/r02c/tune_*_fused.txt)
    bool fuse_pivot = false;
    bool fuse_fits = false;   // ... when K <= 32 and the whole grid is resident at once
    // small LPs: the whole window in one launch, tableau in the LDS of cl_wg workgroups
    bool cluster = false;
    int cl_wg = 0, cl_cw = 0;
    uint64_t* cl_gran = nullptr;   // hand-off granules of the cluster launch
    bool exchange = false;          // candidate all-gather + prow all-reduce path
    int64_t launched = 0;
    int status = DLP_RUNNING;
    int64_t npivots = 0;
    // timing (HIP events on the session stream)
    int ev_per_pivot = 0;
    std::vector<hipEvent_t> ev;
    int64_t ev_pending = 0;   // pivots with recorded events since the last poll
    double timings[DLP_NUM_PHASES] = {0, 0, 0, 0};
    int64_t nsamples = 0;
    // graph replay of one poll window (single rank, no events)
    hipGraphExec_t gexec = nullptr;
    hipGraph_t graph = nullptr;
    int64_t graph_chunk = 0;
    // problem copy for results
    dlp_problem prob_dims{};
    // general LPs (two-phase): phase 1 / 2, the carried Phase II objective row
    // (local index, -1 elsewhere), artificial drive-out queue, caller-driven step kind
    bool general = false;
    int phase = 2;
    int64_t carry_local = -1;
    int64_t nprice = 0;
    double bmax = 0.0;
    std::vector<int32_t> drive;
    size_t drive_next = 0;
    bool carry_pending = false;
    int64_t phase1_pivots = 0;
    enum StepKind { STEP_PIVOT, STEP_FORCED, STEP_CARRY } step_kind = STEP_PIVOT;
    bool step_void = false;
    // deferred rank-k update (dlp_defer.hip): block arrays, pivots enqueued since
    // the last tableau pass, pass geometry; update-kernel launch accounting
    dlp::Defer d;
    int since_flush = 0;
    int defer_rb = 64, defer_occ = 0;   // pass band rows (auto_defer_rb), WG/CU cap
    int defer_rb_req = 0;               // the caller's band rows (0 = auto: follows the form)
    std::vector<uint8_t> ev_flush;   // per timed slot: a pass ran in it
    int64_t upd_launches = 0;
    // lookahead: two tableau buffers; the pass of block b reads Tb[tcur]
    // and writes the other buffer on pstream while block b+1 is selected on Tb[tread]
    // (the pass's source) replaying block b's sealed steps first.  dslot: the block
    // arrays of the two blocks in flight (rhs shared); zbuf: the buffer whose objective
    // row is current.
    bool la = false;
    double* Tb[2] = {nullptr, nullptr};
    // band publication of the lookahead pass (dlp::BandPub): [2][band_stride] counts
    uint32_t* band_cnt = nullptr;
    int64_t band_stride = 0;
    int tread = 0, tcur = 0, zbuf = 0, cur = 0;
    bool la_pending = false;   // a pass is in flight: Tb[tread] lacks block (1 - cur)
    dlp::Defer dslot[2];
    hipStream_t pstream = nullptr;
    hipEvent_t ev_seal = nullptr, ev_pass = nullptr;
    int prio_chain = 0, prio_pass = 0;   // the two streams' priorities (stream pool key)
    // auto policies: lookahead (opt.lookahead < 0) and the pass form (no set_defer_tuning form);
    // an exchange session's lookahead follows its exchange (la_policy)
    bool la_auto = false;
    bool form_auto = true;
    // peer exchange, deferred: the selection inside the ratio launch and the commit inside the
    // pivot-row launch (dlp::launch_ratio_defer's xfuse); off while dlp_sessions_run drives ranks
    // that share a device (their phases must stay in separate launches)
    bool xfuse = true;
    std::string xreason;   // why an auto exchange fell back to RCCL (empty: it did not)
    // allocations from the buffer pool (size class per pointer), returned to it at free
    std::vector<std::pair<void*, size_t>> pooled;
    bool pool_ok = true;   // false once the stream failed: its buffers are freed, not pooled
    int chain_cus = 0;     // lookahead: CUs of the chain's stream (0 = unmasked; chain_cus_policy)
    // ranks of this session's exchange on its device (itself included) and this rank's index among
    // them, from the device of every rank the peer connect saw (install_peers); 1 / 0 otherwise
    int coloc_n = 1, coloc_i = 0;
    int64_t ld_full = 0;   // condensed tableau: the row stride the full layout would have (read-outs)
};

extern "C" int flush_pending(dlp_session* s);   // defined with the C entry points

namespace {

int64_t round16(int64_t v) { return (v + 15) / 16 * 16; }

// Streams are reused across sessions: creating a HIP stream costs ~1.7-2.3 ms and
// destroying one ~1.6-1.9 ms on MI355X (ROCm 7.2, DLP_TRACE_CREATE), against ~0.05 ms for all
// of a small session's allocations: C1 (200 x 400, 353 pivots) spent 4 of its 10 ms end to
// end there (profiles/r03f/).  A freed session's streams (drained without error) go back to a
// per-(device, priority) pool of at most kStreamPoolMax; a new session takes one from it.
constexpr size_t kStreamPoolMax = 16;
// Streams on a CU mask (the lookahead's chain / pass split, chain_cus_policy): a pooled stream key
// >= kMaskedKey names one, key = kMaskedKey + (first mask bit << 10) + bit count.
constexpr int kMaskedKey = 1 << 20;
struct PooledStream {
    int device, prio;
    hipStream_t s;
};
std::mutex g_stream_mu;
std::vector<PooledStream> g_stream_pool;

hipError_t acquire_stream(int device, int prio, hipStream_t* out) {
    {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        for (size_t k = g_stream_pool.size(); k-- > 0;)
            if (g_stream_pool[k].device == device && g_stream_pool[k].prio == prio) {
                *out = g_stream_pool[k].s;
                g_stream_pool.erase(g_stream_pool.begin() + (ptrdiff_t)k);
                return hipSuccess;
            }
    }
    if (prio >= kMaskedKey) {
        if (std::getenv("DLP_TEST_MASK_FAIL")) return hipErrorNotSupported;   // tests: no CU-masked queues
        const int first = (prio - kMaskedKey) >> 10, n = (prio - kMaskedKey) & 1023;
        uint32_t mask[8] = {};
        for (int b = first; b < first + n && b < 256; ++b) mask[b / 32] |= 1u << (b % 32);
        (void)hipGetLastError();
        return hipExtStreamCreateWithCUMask(out, 8, mask);
    }
    return hipStreamCreateWithPriority(out, hipStreamNonBlocking, prio);
}

// Destroy the pooled streams of `device` (< 0: all), e.g. before the process exits: CU-masked queues
// left to the runtime's own teardown crashed a rocprofv3-traced process at exit (profiles/r06i/).
void streams_drain(int device) {
    std::vector<PooledStream> out;
    {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        for (size_t k = g_stream_pool.size(); k-- > 0;)
            if (device < 0 || g_stream_pool[k].device == device) {
                out.push_back(g_stream_pool[k]);
                g_stream_pool.erase(g_stream_pool.begin() + (ptrdiff_t)k);
            }
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (const auto& e : out) {
        (void)hipSetDevice(e.device);
        (void)hipStreamDestroy(e.s);
    }
    (void)hipSetDevice(cur);
    (void)hipGetLastError();
}

// the caller has set the device; a stream whose work failed is destroyed, not pooled
void release_stream(int device, int prio, hipStream_t s) {
    if (!s) return;
    if (hipStreamSynchronize(s) == hipSuccess) {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        if (g_stream_pool.size() < kStreamPoolMax) {
            g_stream_pool.push_back({device, prio, s});
            return;
        }
    }
    (void)hipGetLastError();
    (void)hipStreamDestroy(s);
}

// Small device buffers (and the pinned state copy) are reused across sessions the same way:
// C1 (200 x 400) spent 0.6 ms of its 6.7 ms end to end in the ~18 hipFree calls of a session's
// teardown and ~0.2 ms in the allocations (DLP_TRACE_CREATE, profiles/r03g/).  Freed buffers of at
// most kBufPoolMax bytes go to a per-device pool keyed by their power-of-two size class (at most
// kBufPoolTotal bytes and kBufPoolCount entries cached); a session takes an exact class match.
// Buffers above kBufPoolMax (the tableau of every streaming LP) are never pooled; a small LP's
// tableau is.  Contents are not cleared: every buffer is initialised by the session before it
// is read, as a fresh hipMalloc's would have to be.  When an allocation fails, the device's
// cached buffers are freed and it is retried (pool_alloc); dlp_release_cached_memory empties
// the pool explicitly, and pool_bytes lets the free-memory checks count cached bytes as free.
constexpr size_t kBufPoolMax = (size_t)32 << 20;     // (the default pivot log: 1 M x 32 B)
constexpr size_t kBufPoolTotal = (size_t)512 << 20;
constexpr size_t kBufPoolCount = 256;
struct PooledBuf {
    int device;   // -1: pinned host memory
    size_t cls;
    void* p;
};
std::mutex g_buf_mu;
std::vector<PooledBuf> g_buf_pool;
size_t g_buf_total = 0;

size_t size_class(size_t bytes) {
    size_t c = 256;
    while (c < bytes) c <<= 1;
    return c;
}

// Free every cached buffer of `device` (-1: pinned host memory; kAllDevices: every entry);
// returns the bytes freed.
constexpr int kAllDevices = -2;
size_t pool_drain(int device) {
    std::vector<PooledBuf> out;
    {
        std::lock_guard<std::mutex> lk(g_buf_mu);
        for (size_t k = g_buf_pool.size(); k-- > 0;)
            if (device == kAllDevices || g_buf_pool[k].device == device) {
                out.push_back(g_buf_pool[k]);
                g_buf_total -= g_buf_pool[k].cls;
                g_buf_pool.erase(g_buf_pool.begin() + (ptrdiff_t)k);
            }
    }
    size_t freed = 0;
    for (const auto& b : out) {
        if (b.device < 0) {
            (void)hipHostFree(b.p);
        } else {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(b.device);
            (void)hipFree(b.p);
            (void)hipSetDevice(cur);
        }
        freed += b.cls;
    }
    return freed;
}

// Device bytes the pool holds for `device` (free memory as far as a session is concerned).
size_t pool_bytes(int device) {
    std::lock_guard<std::mutex> lk(g_buf_mu);
    size_t n = 0;
    for (const auto& b : g_buf_pool)
        if (b.device == device) n += b.cls;
    return n;
}

// device < 0: pinned host memory (hipHostMallocDefault)
hipError_t pool_alloc(dlp_session* s, int device, void** p, size_t bytes) {
    const size_t cls = size_class(bytes);
    if (cls <= kBufPoolMax) {
        std::lock_guard<std::mutex> lk(g_buf_mu);
        for (size_t k = g_buf_pool.size(); k-- > 0;)
            if (g_buf_pool[k].device == device && g_buf_pool[k].cls == cls) {
                *p = g_buf_pool[k].p;
                g_buf_total -= cls;
                g_buf_pool.erase(g_buf_pool.begin() + (ptrdiff_t)k);
                s->pooled.push_back({*p, cls});
                return hipSuccess;
            }
    }
    const bool pool = cls <= kBufPoolMax;
    auto alloc = [&]() {
        return device < 0 ? hipHostMalloc(p, pool ? cls : bytes, hipHostMallocDefault)
                          : hipMalloc(p, pool ? cls : bytes);
    };
    hipError_t e = alloc();
    if (e != hipSuccess && pool_drain(device) > 0) {   // cached buffers of this device hold memory
        (void)hipGetLastError();
        e = alloc();
    }
    if (e == hipSuccess && pool) s->pooled.push_back({*p, cls});
    return e;
}

// Free p (a session buffer): back to the pool when it came from it and the session is healthy.
// DLP_TRACE_CREATE: buffers the calling thread's last teardown freed instead of pooling (per
// thread: sessions may be freed from several threads at once)
thread_local int g_pool_freed = 0;
thread_local std::string g_pool_freed_why;
void pool_release(dlp_session* s, int device, void* p) {
    if (!p) return;
    size_t cls = 0;
    for (auto& e : s->pooled)
        if (e.first == p) {
            cls = e.second;
            e.first = nullptr;
            break;
        }
    if (cls && s->pool_ok) {
        std::lock_guard<std::mutex> lk(g_buf_mu);
        if (g_buf_total + cls <= kBufPoolTotal && g_buf_pool.size() < kBufPoolCount) {
            g_buf_pool.push_back({device, cls, p});
            g_buf_total += cls;
            return;
        }
    }
    ++g_pool_freed;
    if (std::getenv("DLP_TRACE_CREATE"))
        g_pool_freed_why += " " + std::to_string(cls) + (cls == 0 ? "(unpooled)" : s->pool_ok ? "(full)" : "(failed)");
    if (device < 0)
        (void)hipHostFree(p);
    else
        (void)hipFree(p);
}

// DLP_TRACE_CREATE=1: milliseconds of each stage of session creation / free on stderr
// (tools/c1_overhead.py; diagnostics only)
struct StageClock {
    bool on = std::getenv("DLP_TRACE_CREATE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "dlp stage %-22s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

int auto_rows_per_block(const dlp_session* s) { return s->streaming ? 8 : 4; }
// deferred pass band rows: 64 on a cache-resident tableau, 256 streaming; 768 for the K = 64
// streaming pass over >= 16k local rows (form 21 reads P once per band: C3 7,227 / 7,361 / 7,433
// pivots/s at 256 / 512 / 768 rows on one box, 768 best on two, profiles/r02q/).  Fewer rows (a
// rank of a multi-GPU C3) keep 256: at 4096 rows, 768-row bands would be 6 x 257 workgroups,
// two rounds of the chip's 768 pass slots plus a few, a long tail.  Only the register-resident
// forms (3/4/5/20/21/22) take tall bands: forms 0-2 stage the band's coefficients in LDS
// (fit_defer_rb).
bool tall_band_form(int form) {
    return form == 3 || form == 4 || form == 5 || form == 20 || form == 21 || form == 22 || form == 23;
}
// Forms 0-2 hold the band's K coefficients per row + a row index in dynamic LDS and s_pl[K]
// statically: K * rb * 8 + rb * 4 + K * 4 <= 160 KiB.  Bands only change the work split, never
// the result (every element sees the same K-step sequence), so the clamp is exact.
int fit_defer_rb(const dlp_session* s, int rb) {
    if (s->d.form <= 2) {
        const int K = std::max(s->d.K, 1);
        const int cap = (160 * 1024 - 4 * K) / (8 * K + 4);
        rb = std::min(rb, cap);
    }
    return std::max(1, std::min(rb, 1024));
}
int auto_defer_rb(const dlp_session* s) {
    if (!s->streaming) return fit_defer_rb(s, 64);
    const bool tall = s->d.K == 64 && s->rows >= 16384 && tall_band_form(s->d.form);
    return fit_defer_rb(s, tall ? 768 : 256);
}

// Row i of a general LP's standard-form tableau (include/dlp.h, "general LPs").
void std_row(const dlp::StdForm& f, int64_t i, double* r) {
    std::memcpy(r, f.A.data() + i * f.ns, sizeof(double) * f.ns);
    if (f.slack_col[i] >= 0) r[f.slack_col[i]] = f.type[i] == dlp::ROW_G ? -1.0 : 1.0;
    if (f.art_col[i] >= 0) r[f.art_col[i]] = 1.0;
    r[f.ncols()] = f.b[i];
}

// Host build of a tableau slice (dense / ad-allocation / general problems).
// General LPs with artificials: `rows` includes the carried Phase II
// objective row at local index carry_local (>= 0 on the last rank only).
void host_tableau(const dlp_problem* p, int64_t row_first, int64_t rows, int64_t ld,
                  std::vector<double>& T, int64_t carry_local = -1) {
    const int64_t m = p->m, n = p->n, N = n + m;
    T.assign((size_t)(rows + 1) * ld, 0.0);
    if (p->kind == dlp::PROB_GENERAL) {
        const dlp::StdForm& f = p->sf;
        const int64_t NG = f.ncols();
        for (int64_t il = 0; il < rows; ++il) {
            double* r = T.data() + il * ld;
            if (il == carry_local) {
                for (int64_t j = 0; j < f.ns; ++j) r[j] = -f.c[j];
            } else {
                std_row(f, row_first + il, r);
            }
        }
        double* z = T.data() + rows * ld;
        if (f.nart == 0) {
            for (int64_t j = 0; j < f.ns; ++j) z[j] = -f.c[j];
        } else {   // Phase I: z_j = fold over artificial rows ascending of (z_j - T[i][j])
            std::vector<double> r(NG + 1);
            for (int64_t i = 0; i < f.m; ++i) {
                if (f.art_col[i] < 0) continue;
                std::fill(r.begin(), r.end(), 0.0);
                std_row(f, i, r.data());
                for (int64_t j = 0; j < f.nprice(); ++j) z[j] = z[j] - r[j];
                z[NG] = z[NG] - r[NG];
            }
        }
        return;
    }
    if (p->kind == dlp::PROB_DENSE) {
        for (int64_t il = 0; il < rows; ++il) {
            const int64_t i = row_first + il;
            double* r = T.data() + il * ld;
            std::memcpy(r, p->A.data() + i * n, sizeof(double) * n);
            r[n + i] = 1.0;
            r[N] = p->b[i];
        }
        double* z = T.data() + rows * ld;
        for (int64_t j = 0; j < n; ++j) z[j] = -p->c[j];
    } else {   // PROB_ADALLOC: rows [0,A) budgets, rows [A, A+I) assignment
        const auto& ad = p->ad;
        const int64_t A = ad.num_advertisers;
        for (int64_t k = 0; k < (int64_t)ad.adv.size(); ++k) {
            const int64_t ib = ad.adv[k] - row_first;
            if (ib >= 0 && ib < rows) T[ib * ld + k] = ad.bid[k];
            const int64_t ia = A + ad.imp[k] - row_first;
            if (ia >= 0 && ia < rows) T[ia * ld + k] = 1.0;
        }
        for (int64_t il = 0; il < rows; ++il) {
            const int64_t i = row_first + il;
            T[il * ld + n + i] = 1.0;
            T[il * ld + N] = (i < A) ? ad.budget[i] : 1.0;
        }
        double* z = T.data() + rows * ld;
        for (int64_t k = 0; k < n; ++k) z[k] = -ad.bid[k];
    }
}

void free_session(dlp_session* s) {
    if (!s) return;
    StageClock clk;
    if (s->device >= 0) (void)hipSetDevice(s->device);
    if (s->stream && hipStreamSynchronize(s->stream) != hipSuccess) s->pool_ok = false;
    if (s->pstream && hipStreamSynchronize(s->pstream) != hipSuccess) s->pool_ok = false;
    (void)hipGetLastError();
    clk.mark("free: sync");
    // diagnostics: DLP_CHAIN_STAMPS=<file> dumps the chain kernels' phase stamps (tools only)
    if (const char* path = std::getenv("DLP_CHAIN_STAMPS")) {
        std::vector<uint64_t> h(64 * 16, 0);
        if (dlp::chain_stamps_dump(h.data()) == hipSuccess)
            if (FILE* f = std::fopen(path, "wb")) {
                std::fwrite(h.data(), sizeof(uint64_t), h.size(), f);
                std::fclose(f);
            }
        std::vector<uint64_t> w(1024 * 8, 0);   // per-workgroup stamps of the grouped-ring selection
        if (dlp::chain_wg_stamps_dump(w.data()) == hipSuccess)
            if (FILE* f = std::fopen((std::string(path) + ".wg").c_str(), "wb")) {
                std::fwrite(w.data(), sizeof(uint64_t), w.size(), f);
                std::fclose(f);
            }
    }
    if (s->gexec) (void)hipGraphExecDestroy(s->gexec);
    clk.mark(s->gexec ? "free: graph exec" : "free: (no graph)");
    if (s->graph) (void)hipGraphDestroy(s->graph);
    clk.mark("free: graph");
    for (auto e : s->ev) (void)hipEventDestroy(e);
    clk.mark("free: events");
    if (s->comm) (void)ncclCommDestroy(s->comm);
    if (s->pstream) (void)hipStreamSynchronize(s->pstream);
    clk.mark("free: comm");
    void* dev[] = {s->Tb[0] ? s->Tb[0] : s->T, s->Tb[1], s->colq, s->prow_send, s->partials,
                   s->cand_send, s->cand_recv, s->pp, s->basis, s->st, s->log, s->d.C, s->d.Cc,
                   s->d.P, s->d.rhs, s->d.nzc, s->cl_gran, s->band_cnt, s->g.cd.slot_of, s->g.cd.var_of,
                   s->g.cd.rst};
    for (void* p : dev) pool_release(s, s->device, p);
    if (s->la || s->dslot[1].C) {   // slot 0 aliases s->d
        void* sl[] = {s->dslot[1].C, s->dslot[1].Cc, s->dslot[1].P, s->dslot[1].nzc};
        for (void* p : sl) pool_release(s, s->device, p);
    }
    clk.mark(g_pool_freed ? ("free: pooled buffers, freed:" + g_pool_freed_why).c_str() : "free: pooled buffers");
    g_pool_freed = 0;
    g_pool_freed_why.clear();
    if (s->ev_seal) (void)hipEventDestroy(s->ev_seal);
    if (s->ev_pass) (void)hipEventDestroy(s->ev_pass);
    if (s->pstream) release_stream(s->device, s->prio_pass, s->pstream);
    if (s->prow_recv && s->prow_recv != s->prow_send) pool_release(s, s->device, s->prow_recv);
    for (void* p : s->ipc_open) (void)hipIpcCloseMemHandle(p);
    if (s->xblk) (void)hipFree(s->xblk);
    if (s->xpeers) (void)hipFree(s->xpeers);
    if (s->xabort) (void)hipHostFree(s->xabort);
    pool_release(s, -1, s->host_st);
    clk.mark("free: buffers");
    if (s->stream) release_stream(s->device, s->prio_chain, s->stream);
    clk.mark("free: stream");
    delete s;
}

int validate_options(const dlp_options* o) {
    if (!o) { set_error("options is NULL"); return DLP_ERR_ARG; }
    if (o->pricing != DLP_PRICING_DANTZIG_BLAND && o->pricing != DLP_PRICING_BLAND) {
        set_error("unknown pricing rule");
        return DLP_ERR_ARG;
    }
    if (!(o->tol_dj >= 0.0) || !(o->tol_piv >= 0.0) || !(o->tol_feas >= 0.0) || o->max_pivots < 0 ||
        o->check_interval <= 0) {
        set_error("invalid tolerance / pivot limit / check interval");
        return DLP_ERR_ARG;
    }
    if (o->exchange != DLP_XCHG_DEFAULT && o->exchange != DLP_XCHG_RCCL && o->exchange != DLP_XCHG_PEER) {
        set_error("exchange must be DLP_XCHG_DEFAULT, DLP_XCHG_RCCL or DLP_XCHG_PEER");
        return DLP_ERR_ARG;
    }
    return DLP_OK;
}

// The K = 64 streaming pass form, when the caller has not set one: form 21 (DPP coefficients
// from registers) under lookahead, form 23 (LDS ring) with nothing beside the pass: C3 7.9 vs
// 8.2 ms per pass in situ without lookahead, but under lookahead the ring's deeper memory queue
// slows the selection chain beside it more than it speeds the pass (C3 6,578 vs 7,685 pivots/s,
// profiles/r03d/)
void pick_form(dlp_session* s) {
    if (!s->form_auto || s->d.K != 64 || !s->streaming || (s->d.form != 21 && s->d.form != 23)) return;
    // lookahead: form 21 beside the chain (its waves fit the 32 VGPRs three form-21 waves leave);
    // on a CU split of more than 4,096 rows the LDS-ring pass (form 23), which streams faster per
    // CU and no longer slows a chain on other CUs: c3r2 13.9-14.3 k vs 12.6 k pivots/s, c3r4
    // 20.6 k (chain on 128 CUs) vs 20.0-20.3 k (form 21 on 96); c3r8 24.4-24.5 k vs 24.7 k, so
    // form 21 there (profiles/r04ag/, r04ah/)
    s->d.form = !s->la ? 23 : (s->chain_cus > 0 && s->rows > 4096) ? 23 : 21;
    s->dslot[0].form = s->dslot[1].form = s->d.form;
}

int flush_pending_block(dlp_session* s);

// Lanes per deferred ratio workgroup (one lane per row; the replay's coefficient chain streams
// through each wave's LDS-DMA ring, whose rate is per CU): fixed at creation, since the peer
// exchange's candidate slots are one per ratio workgroup of every rank (xslots), identical on
// every rank — so the rule reads the global m and the rank count, not the local rows.  128 lanes
// up to 8,192 rows per rank: twice the workgroups spread the replay over more CUs (c3r8 25.3-25.4 k
// vs 24.8-25.0 k pivots/s, c3r4 21.0 k vs 20.7-20.9 k, profiles/r05d/; C2 44.7 k vs 42.7 k,
// profiles/r05o/; 64 lanes gain nothing more), else 256 (C3 at P = 1: no difference,
// profiles/r05e/).  DLP_RATIO_THREADS=64/128/256 overrides.
// Condensed tableau by default (dlp_options.condensed = 0); DLP_CONDENSED=0 / 1 overrides the
// auto choice (A/B and tests).
bool condensed_auto() {
    static const int v = std::getenv("DLP_CONDENSED") ? std::atoi(std::getenv("DLP_CONDENSED")) : 1;
    return v == 1;
}

int ratio_threads_policy(const dlp_session* s) {
    if (const char* e = std::getenv("DLP_RATIO_THREADS")) {
        const int n = std::atoi(e);
        if (n == 64 || n == 128 || n == 256) return n;
    }
    const int64_t per_rank = s->m / std::max(s->nranks, 1);
    return per_rank <= 8192 ? 128 : dlp::kRatioDeferThreads;
}

// Lookahead on: a second tableau buffer holding the same bytes, a second set of
// block arrays (rhs shared), band counters, the pass stream.  Called at session creation or
// between runs (la_policy): a pending block is applied first.  Silently stays off where it does
// not apply (the form has no out-of-place pass, general LPs, the small-LP launch, per-phase
// timing, a host-driven rank unless forced, too little free memory).
// The lookahead's CU split.  Beside the pass, the selection chain of a rank-sized tableau is the
// longer of the two and runs 2-3x slower than alone, its waves sharing every CU with three pass
// waves.  On disjoint CU masks (chain on the top n mask bits, the pass on the rest) the block
// balances: measured on the rank geometries with the form-21 pass (profiles/r04x/, alternating
// runs), c3r8 (4,096 rows) n = 128: 24.3-24.5 k vs 22.65 k pivots/s; c3r4 (8,192) n = 80-96:
// 19.9-20.0 k vs 17.0-17.1 k; c3r2 (16,384) n = 48-64: 12.5-12.6 k vs 11.97 k; C3 (32,768 rows,
// pass-bound) loses with any split (form 21 n = 32: 7.63 k, form 23 n = 32: 8.05 k vs 8.22 k
// unmasked on one box, profiles/r04ai/).  With the form-23 pass on the split (pick_form) the
// best n moves: c3r4 128 (20.6 k), c3r2 64 (13.9-14.3 k), c3r8 128 (profiles/r04ah/).  Auto: 128
// CUs for the chain up to 8,192 local rows, 64 below 32,768, at most half the CUs, 0 (no masks)
// from 32,768; DLP_CHAIN_CUS=n overrides (0 = off).
// Ranks that share a device (several rank processes or rank sessions on one GPU: install_peers
// learns it from the devices of the connected ranks) split that budget into disjoint slices, one
// per rank, the pass of each on the CUs no chain uses: with one shared mask the spinning chain
// workgroups of the waiting ranks filled those CUs and the owner's could not be placed (3+ rank
// processes on one GPU hit the exchange timeout, profiles/r05w/).  A slice under 32 CUs (mask
// bits act in groups of 32) turns the masks off for those ranks.  Returns this rank's slice.
int chain_cus_policy(const dlp_session* s) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device) != hipSuccess || cus < 64)
        return 0;
    int n = 0;
    if (const char* e = std::getenv("DLP_CHAIN_CUS")) {
        n = std::atoi(e);
        n = n > 0 && n < cus ? n : 0;
    } else if (s->rows < 32768 || s->g.cd.on) {
        // (mask bits act in groups of 32: 112 and 128 chain bits, or 144 and 160, give the pass the
        // same time, profiles/r04ah/).  The condensed tableau halves the pass, so at C3 (32,768
        // rows) the chain is the longer part too: 64 chain CUs with form 23 on the other 192 take
        // the block from 5.62 to 4.73-4.79 ms (13.4-13.5 k vs 11.4 k pivots/s; 32 CUs 12.7 k, 96
        // 12.6 k; profiles/r06f/)
        n = std::min(s->rows > 8192 ? 64 : 128, cus / 2);
        // A rank alone on its device, condensed, moved the balance again (alternating pairs,
        // profiles/r06zh/, r06zi/): up to 8,192 rows 96 chain CUs (c3r8 27.99-28.36 k vs 27.58-27.64 k
        // pivots/s with 128; c3r4 24.30-24.55 k vs 23.90-24.05 k; 64 equal to 96), 16,384 rows 128
        // (c3r2 19.10-19.46 k vs 18.71-18.74 k with 64; 160 loses), C3 64.  Ranks sharing a device keep
        // the budget above for their slices.
        if (s->g.cd.on && s->coloc_n <= 1)
            n = std::min(s->rows <= 8192 ? 96 : (s->rows < 32768 ? 128 : 64), cus / 2);
    }
    const int nco = std::max(1, s->coloc_n);
    if (n <= 0 || nco == 1) return n;
    const int slice = n / nco / 32 * 32;
    return slice >= 32 ? slice : 0;
}

// Put the chain's stream on n CU-mask bits (n = 0: an unmasked stream at the chain's priority) —
// the top n, or with ranks sharing the device this rank's slice of the top coloc_n x n — and name
// the pass's stream key accordingly (the bits below every chain slice; acquired by the caller).
// Results do not depend on where a kernel runs.
int chain_cus_apply(dlp_session* s, int n) {
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device) != hipSuccess) cus = 256;
    const int nco = std::max(1, s->coloc_n);
    if (n > 0 && n * nco > cus) n = 0;   // (chain_cus_policy never asks for more)
    const int first = cus - n * (s->coloc_i + 1);
    if (n == s->chain_cus && s->stream && (n == 0 || s->prio_chain == kMaskedKey + (first << 10) + n))
        return DLP_OK;
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (s->pstream) {
        HIP_TRY(hipStreamSynchronize(s->pstream));
        release_stream(s->device, s->prio_pass, s->pstream);
        s->pstream = nullptr;
    }
    release_stream(s->device, s->prio_chain, s->stream);
    s->stream = nullptr;
    int lo = 0, hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    s->prio_chain = n > 0 ? kMaskedKey + (first << 10) + n : hi;
    s->prio_pass = n > 0 ? kMaskedKey + (cus - n * nco) : lo;
    if (n > 0 && acquire_stream(s->device, s->prio_chain, &s->stream) != hipSuccess) {
        (void)hipGetLastError();   // no CU-masked queue here: both streams unmasked, as before round 4
        s->stream = nullptr;
        s->prio_chain = hi;
        s->prio_pass = lo;
        n = 0;
    }
    if (!s->stream) HIP_TRY(acquire_stream(s->device, s->prio_chain, &s->stream));
    s->chain_cus = n;
    return DLP_OK;
}

// The lookahead's two streams on the split chain_cus_policy asks for (re-applied when the exchange
// changes what it asks for: a peer connect that finds ranks sharing the device).
int la_streams(dlp_session* s) {
    CALL_TRY(chain_cus_apply(s, chain_cus_policy(s)));   // releases the pass stream when the split changes
    if (!s->pstream && acquire_stream(s->device, s->prio_pass, &s->pstream) != hipSuccess) {
        (void)hipGetLastError();   // no CU-masked queue for the pass: back to unmasked streams
        s->pstream = nullptr;
        CALL_TRY(chain_cus_apply(s, 0));
        HIP_TRY(acquire_stream(s->device, s->prio_pass, &s->pstream));
    }
    return DLP_OK;
}

int la_enable(dlp_session* s, bool forced) {
    if (s->la) return DLP_OK;
    const bool host_driven = s->nranks > 1 && !s->use_rccl && s->xmode != dlp_session::X_PEER;
    bool ok = s->d.K > 1 && 2 * s->d.K <= dlp::kMaxReplay && dlp::lookahead_form(s->d.form) &&
              !s->general && !s->cluster && (!host_driven || forced) && s->opt.timing < 2;
    const size_t tbytes = (size_t)(s->rows + 1) * s->ld * sizeof(double);
    size_t freeb = 0, totalb = 0;
    if (ok && hipMemGetInfo(&freeb, &totalb) == hipSuccess) {
        freeb += pool_bytes(s->device);   // cached by earlier sessions: released on demand (pool_alloc)
        ok = (s->Tb[1] ? freeb + tbytes : freeb) > tbytes + tbytes / 8 + ((size_t)1 << 30);
    }
    else
        ok = false;
    if (!ok) return DLP_OK;
    CALL_TRY(flush_pending_block(s));
    const int c = (s->Tb[1] && s->T == s->Tb[1]) ? 1 : 0;   // the current buffer
    if (!s->Tb[0]) s->Tb[0] = s->T;
    if (!s->Tb[1 - c] && pool_alloc(s, s->device, (void**)&s->Tb[1 - c], tbytes) != hipSuccess) {
        set_error("hipMalloc of the second tableau buffer failed");
        return DLP_ERR_OOM;
    }
    // the whole buffer, padding included, so both hold the same bytes everywhere
    HIP_TRY(hipMemcpyAsync(s->Tb[1 - c], s->Tb[c], tbytes, hipMemcpyDeviceToDevice, s->stream));
    s->tread = s->tcur = s->zbuf = c;
    s->cur = 0;
    s->la_pending = false;
    const dlp::Defer keep1 = s->dslot[1];
    s->dslot[0] = s->d;
    s->dslot[1] = s->d;
    dlp::Defer& d1 = s->dslot[1];
    const int64_t rows_total = s->rows + 1;
    if (keep1.C) {   // arrays of an earlier lookahead period (their stale contents are never read)
        d1.C = keep1.C;
        d1.Cc = keep1.Cc;
        d1.P = keep1.P;
        d1.nzc = keep1.nzc;
    } else {
        const int64_t kt = s->d.K <= 4 ? 4 : s->d.K <= 8 ? 8 : s->d.K <= 16 ? 16 : s->d.K <= 32 ? 32 : 64;
        d1.C = d1.Cc = d1.P = nullptr;
        d1.nzc = nullptr;
        HIP_TRY(pool_alloc(s, s->device, (void**)&d1.C, sizeof(double) * s->d.K * (rows_total + 1)));
        HIP_TRY(pool_alloc(s, s->device, (void**)&d1.Cc, sizeof(double) * s->d.K * s->d.ldcc));
        HIP_TRY(pool_alloc(s, s->device, (void**)&d1.P, sizeof(double) * kt * s->ld));
        HIP_TRY(pool_alloc(s, s->device, (void**)&d1.nzc, sizeof(int32_t) * (s->rows + 1)));
        HIP_TRY(hipMemsetAsync(d1.C, 0, sizeof(double) * s->d.K * (rows_total + 1), s->stream));
        HIP_TRY(hipMemsetAsync(d1.Cc, 0, sizeof(double) * s->d.K * s->d.ldcc, s->stream));
        HIP_TRY(hipMemsetAsync(d1.P, 0, sizeof(double) * kt * s->ld, s->stream));
    }
    if (!s->band_cnt) {
        s->band_stride = (s->rows + 63) / 64 + 1;   // bands of >= 64 rows
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->band_cnt, sizeof(uint32_t) * 2 * s->band_stride));
    }
    HIP_TRY(hipMemsetAsync(s->band_cnt, 0, sizeof(uint32_t) * 2 * s->band_stride, s->stream));
    CALL_TRY(la_streams(s));
    if (!s->ev_seal) HIP_TRY(hipEventCreateWithFlags(&s->ev_seal, hipEventDisableTiming));
    if (!s->ev_pass) HIP_TRY(hipEventCreateWithFlags(&s->ev_pass, hipEventDisableTiming));
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->la = true;
    s->opt.lookahead = 1;
    if (s->gexec) { (void)hipGraphExecDestroy(s->gexec); s->gexec = nullptr; }
    if (s->graph) { (void)hipGraphDestroy(s->graph); s->graph = nullptr; }
    return DLP_OK;
}

// comm_in: a communicator made by the caller (dlp_solve's in-process multi-device
// path, ncclCommInitAll); the session then owns it.  uid: a unique id shared by
// P processes (ncclCommInitRank here).  Either one means the RCCL exchange.
int session_init(const dlp_problem* prob, const dlp_options* opt, int rank, int nranks,
                 const void* uid, dlp_session* s, ncclComm_t comm_in = nullptr) {
    const bool rccl = uid != nullptr || comm_in != nullptr;
    // the caller's choice, before the "auto" values below are resolved into s->opt
    const bool variant_auto = opt->update_variant < 0;
    s->opt = *opt;
    s->device = opt->device;
    s->rank = rank;
    s->nranks = nranks;
    s->m = prob->m;
    s->n = prob->n;
    s->N = prob->n + prob->m;
    s->nprice = s->N;
    s->general = prob->kind == dlp::PROB_GENERAL;
    if (s->general) {   // standard-form dimensions; the carried row goes to the last rank
        s->m = prob->sf.m;
        s->n = prob->sf.ns;
        s->N = prob->sf.ncols();
        s->nprice = prob->sf.nprice();
        s->phase = prob->sf.nart > 0 ? 1 : 2;
        for (double v : prob->sf.b) s->bmax = std::max(s->bmax, v);
    }
    s->width = round16(s->N + 1);
    CALL_TRY(dlp_rank_rows(s->m, rank, nranks, &s->row_first, &s->rows));
    int64_t rows_elig = s->rows;
    if (s->phase == 1 && rank == nranks - 1) {
        s->carry_local = s->rows;
        s->rows += 1;
    }
    // "auto" tuning (negative / zero option values), from the interleaved A/B
    // sweeps of tools/tune_update.py on MI355X (update kernel):
    //  - tableaus far beyond the 256 MiB Infinity Cache stream from HBM: the
    //    row-serial kernel capped at 4 workgroups/CU, 8-row bands, nt stores;
    //  - smaller ones stay partly cache-resident: uncapped, 4-row bands,
    //    default cache policy;
    //  - rows of >= 4096 doubles are aligned to 4 KiB (whole-tile alignment) for the eager
    //    update, to 1 KiB for the deferred pass of a streaming tableau (C3 ld 65,664 vs
    //    66,048: 7,716-7,737 vs 7,620-7,632 pivots/s, alternating runs on one box; the
    //    LDS-ring copy probe 6.2 vs 7.0 ms: profiles/r03g/)
    const bool streaming = (double)(s->rows + 1) * (double)s->width * 8.0 > (double)(1ll << 30);
    if (s->opt.ld_align <= 0)
        s->opt.ld_align = s->width >= 4096 ? ((streaming && s->opt.defer != 1) ? 128 : 512) : 16;
    if (s->opt.update_variant < 0) s->opt.update_variant = streaming ? 22 : 26;
    if (s->opt.nontemporal < 0) s->opt.nontemporal = streaming ? 1 : 0;
    s->streaming = streaming;
    const int64_t align = s->opt.ld_align;
    if (align % 16 != 0) {
        set_error("ld_align must be a multiple of 16 doubles");
        return DLP_ERR_ARG;
    }
    s->ld = (s->width + align - 1) / align * align;
    opt = &s->opt;
    s->prob_dims.m = prob->m;
    s->prob_dims.n = prob->n;
    s->prob_dims.kind = prob->kind;
    if (s->general) {   // back-mapping for results (the matrix itself is not kept)
        s->prob_dims.sf = prob->sf;
        s->prob_dims.sf.A.clear();
        s->prob_dims.sf.A.shrink_to_fit();
    }

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("no HIP device visible (libdlp has no CPU fallback)");
        return DLP_ERR_NODEVICE;
    }
    if (s->device < 0 || s->device >= ndev) { set_error("device ordinal out of range"); return DLP_ERR_ARG; }
    StageClock clk;
    HIP_TRY(hipSetDevice(s->device));
    if (std::getenv("DLP_CHAIN_STAMPS")) HIP_TRY(dlp::chain_stamps_enable());   // diagnostics
    // the pivot chain runs at the highest stream priority: under lookahead its small
    // launches share the device with the pass (pstream, lowest priority)
    int prio_least = 0, prio_greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
    s->prio_chain = prio_greatest;
    s->prio_pass = prio_least;
    HIP_TRY(acquire_stream(s->device, prio_greatest, &s->stream));
    clk.mark("create: stream");

    const int64_t rows_total = s->rows + 1;
    dlp::Geometry& g = s->g;
    g.ld = s->ld;
    g.width = s->width;
    g.rows = s->rows;
    g.row_first = s->row_first;
    g.ncols = s->N;
    g.nprice = s->nprice;
    g.rows_elig = rows_elig;
    g.rthreads = ratio_threads_policy(s);
    if (opt->update_variant < 0 || opt->update_variant >= dlp::update_variants()) {
        set_error("update_variant out of range");
        return DLP_ERR_ARG;
    }
    const int tile = dlp::update_tile(opt->update_variant);
    g.ntiles = (int)((s->width + tile - 1) / tile);
    // deferred rank-k update: auto = 32 pivots per tableau pass on a streaming
    // (HBM-resident) tableau, 16 on a cache-resident one, eager on a tiny one; eager when the
    // caller drives the exchange itself (dlp_session_step_*) or when the chosen
    // rank-1 variant tiles pricing differently from the deferred kernels
    {
        const bool host_driven = nranks > 1 && !rccl;
        int K = opt->defer;
        if (K < 0 || K > dlp::kMaxDefer) {
            set_error("defer must be 0 (auto) or 1..64");
            return DLP_ERR_ARG;
        }
        // a tableau under 32 MiB stays eager: its rank-1 update is a few-µs launch, and
        // the replayed ratio / pivot-row kernels cost more than the passes they save
        // (C4 256x512: 14.2 µs/pivot eager vs 19.0 at K = 16; 1024x1024: 18.0 vs 20.8;
        // C2 4096x8192, 268 MB: K = 16 is 2.3x eager; profiles/r01j/tune_small_defer.txt)
        const bool tiny = (double)(s->rows + 1) * (double)s->width * 8.0 < (double)(32ll << 20);
        // small LPs (auto: tiny, default kernels; or forced by small_lp = 1): one launch per
        // window with the tableau in LDS, when it fits the CUs' LDS (dlp_cluster.hip)
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device) != hipSuccess)
            cus = 0;
        if (!s->general && nranks == 1 && !rccl && s->m < (1 << 30) && s->N < (1 << 30) &&
            (opt->small_lp == 1 ||
             (opt->small_lp == 0 && K == 0 && tiny && variant_auto))) {
            s->cl_wg = dlp::cluster_plan(s->m, s->N, cus, &s->cl_cw);
            // tuning only: DLP_CLUSTER_WG=G forces the workgroup count (if the slices fit)
            if (const char* e = std::getenv("DLP_CLUSTER_WG")) {
                const int gw = std::atoi(e);
                const int cw = gw > 0 ? (int)((s->N + gw) / gw) : 0;
                if (gw > 0 && gw <= cus && (int64_t)(gw - 1) * cw < s->N + 1 &&
                    dlp::cluster_lds_bytes(s->m, cw) <= 160 * 1024 - 1024) {
                    s->cl_wg = gw;
                    s->cl_cw = cw;
                }
            }
            s->cluster = s->cl_wg > 0;
        }
        // streaming tableaus: 64-step blocks through the DPP-coefficient pass (form 21: C3
        // 8.4 ms per 64-step pass = 0.131 ms per step against 0.197 for form 4's 32-step
        // pass, 6,100 vs 4,500 pivots/s; profiles/r02j/)
        // a host-driven rank (the step API) takes the geometry the same rank would run over
        // RCCL, so the multi-GPU split can be exercised without RCCL (general LPs stay eager)
        if (K == 0)
            K = ((host_driven && s->general) || tile != dlp::kDeferTile || tiny || s->cluster)
                    ? 1
                    : (s->streaming ? 64 : 16);
        if (s->cluster && K != 1) s->cluster = false;
        if (K > 1 && tile != dlp::kDeferTile) {
            set_error("defer > 1 needs a 512-column update variant");
            return DLP_ERR_ARG;
        }
        if (K > 1 && host_driven && s->general) {
            set_error("a host-driven (step API) general-LP session is eager: create it with defer = 1");
            return DLP_ERR_ARG;
        }
        s->d.K = K;
        s->opt.defer = K;
        // pass form 4 (2 doubles x 2 rows per lane; a window's partial last block runs the
        // full-block code with zeroed coefficients: C3 20-pivot partial pass 6.93 ms vs a
        // 6.30 ms full pass, 7.58 for the streamed kernel's (form 14), 12.7 before,
        // profiles/r02c/) at K = 32 on a streaming tableau and K = 16 on a cache-resident one
        // (C2: pass 0.116 vs 0.128 ms for form 3, profiles/r02b/tune_c2_forms.txt); 1 double
        // x 4 rows elsewhere (K = 16 streaming: form 3 6.1 ms vs form 4 6.4, r01g)
        s->d.form = (K == 64 && s->streaming) ? 21
                    : ((K == 32 && s->streaming) || (K == 16 && !s->streaming)) ? 4 : 3;
        // condensed tableau: a deferred session of a dense / random /
        // ad-allocation LP stores only the n nonbasic columns + the RHS (the m basic columns are
        // unit vectors); the size-based policies above keep the full tableau's scale
        const int creq = opt->condensed;
        if (creq < -1 || creq > 1) {
            set_error("condensed must be -1 (off), 0 (auto) or 1 (on)");
            return DLP_ERR_ARG;
        }
        if ((creq == 1 || (creq == 0 && condensed_auto())) && K > 1 && !s->general && !s->cluster) {
            s->g.cd.on = 1;
            s->ld_full = s->ld;   // (the read-outs keep the full layout's stride)
            s->width = round16(s->n + 1);
            s->ld = (s->width + align - 1) / align * align;
            g.ld = s->ld;
            g.width = s->width;
            g.ncols = s->n;
            g.nprice = s->n;
            g.ntiles = (int)((s->width + tile - 1) / tile);
        }
    }
    g.rows_per_block = opt->rows_per_block > 0 ? opt->rows_per_block : auto_rows_per_block(s);
    g.rows_per_block = std::min(g.rows_per_block, dlp::kMaxBandLdsHost);
    const size_t tbytes = (size_t)rows_total * s->ld * sizeof(double);
    if (s->g.cd.on) {
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->g.cd.slot_of, sizeof(int32_t) * s->N));
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->g.cd.var_of, sizeof(int32_t) * s->ld));
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->g.cd.rst, sizeof(int32_t) * s->ld));
    }
    if (pool_alloc(s, s->device, (void**)&s->T, tbytes) != hipSuccess) {
        set_error("hipMalloc of the tableau failed (" + std::to_string(tbytes) + " bytes)");
        return DLP_ERR_OOM;
    }
    g.T = s->T;
    clk.mark("create: plan + tableau");
    if (s->cluster) {
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->cl_gran, sizeof(uint64_t) * dlp::cluster_granules(s->m, s->cl_wg)));
    }
    s->ratio_blocks = dlp::ratio_blocks(g);
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device) != hipSuccess)
            cus = 0;
        // (the kernel's real occupancy, not an assumed 2 per CU: ADVICE r02)
        s->fuse_fits = s->d.K > 1 && s->d.K <= 32 &&
                       dlp::fused_pivot_blocks(g) <= std::min(2 * cus, dlp::fused_pivot_capacity(s->d.K, cus));
    }
    s->ratio_blocks_max = std::max(s->ratio_blocks, dlp::ratio_defer_blocks(g));
    HIP_TRY(pool_alloc(s, s->device, (void**)&s->colq, sizeof(double) * (rows_total + dlp::kColqPad)));
    HIP_TRY(hipMemsetAsync(s->colq, 0, sizeof(double) * (rows_total + dlp::kColqPad), s->stream));
    s->exchange = nranks > 1 || rccl;
    HIP_TRY(pool_alloc(s, s->device, (void**)&s->prow_send, sizeof(int64_t) * s->ld));
    if (s->exchange)
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->prow_recv, sizeof(int64_t) * s->ld));
    else
        s->prow_recv = s->prow_send;
    HIP_TRY(pool_alloc(s, s->device, (void**)&s->partials, sizeof(dlp::Cand) * s->ratio_blocks_max));
    HIP_TRY(pool_alloc(s, s->device, (void**)&s->cand_send, sizeof(dlp::Cand)));
    HIP_TRY(pool_alloc(s, s->device, (void**)&s->cand_recv, sizeof(dlp::Cand) * nranks));
    HIP_TRY(pool_alloc(s, s->device, (void**)&s->pp, sizeof(dlp::PricePart) * ((s->ld + 511) / 512)));
    HIP_TRY(pool_alloc(s, s->device, (void**)&s->basis, sizeof(int32_t) * s->m));
    HIP_TRY(pool_alloc(s, s->device, (void**)&s->st, sizeof(dlp::DevState)));
    s->log_cap = opt->log_pivots ? std::max<int64_t>(1, opt->max_pivots) : 0;
    if (s->log_cap > 0) HIP_TRY(pool_alloc(s, s->device, (void**)&s->log, sizeof(dlp_pivot) * s->log_cap));
    HIP_TRY(pool_alloc(s, -1, (void**)&s->host_st, sizeof(dlp::DevState)));
    if (s->d.K > 1) {
        s->d.ldc = s->d.K;
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->d.C, sizeof(double) * s->d.K * (rows_total + 1)));
        s->d.ldcc = (rows_total + 1 + 63) / 64 * 64;
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->d.Cc, sizeof(double) * s->d.K * s->d.ldcc));
        HIP_TRY(hipMemsetAsync(s->d.Cc, 0, sizeof(double) * s->d.K * s->d.ldcc, s->stream));
        // P is sized for the pass template's block (K rounded up to 4/8/16/32/64), so a
        // kernel instance never addresses past it, whatever the session's K
        const int64_t kt = s->d.K <= 4 ? 4 : s->d.K <= 8 ? 8 : s->d.K <= 16 ? 16 : s->d.K <= 32 ? 32 : 64;
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->d.P, sizeof(double) * kt * s->ld));
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->d.rhs, sizeof(double) * (s->rows + 1)));
        HIP_TRY(pool_alloc(s, s->device, (void**)&s->d.nzc, sizeof(int32_t) * (s->rows + 1)));
        HIP_TRY(hipMemsetAsync(s->d.C, 0, sizeof(double) * s->d.K * (rows_total + 1), s->stream));
        HIP_TRY(hipMemsetAsync(s->d.P, 0, sizeof(double) * kt * s->ld, s->stream));
        s->defer_rb_req = opt->rows_per_block > 0 ? opt->rows_per_block : 0;
        s->defer_rb = s->defer_rb_req > 0 ? fit_defer_rb(s, s->defer_rb_req) : auto_defer_rb(s);
    }
    HIP_TRY(hipMemsetAsync(s->prow_send, 0, sizeof(int64_t) * s->ld, s->stream));
    clk.mark("create: side arrays");

    // tableau
    if (prob->kind == dlp::PROB_RANDOM) {
        HIP_TRY(dlp::launch_generate(g, prob->gen_kind, s->m, s->n, prob->seed, s->stream));
    } else {
        std::vector<double> host;
        if (s->g.cd.on) {   // the full rows, then only the structural columns and the RHS kept
            const int64_t ldf = round16(s->N + 1);
            std::vector<double> full;
            host_tableau(prob, s->row_first, s->rows, ldf, full, s->carry_local);
            host.assign((size_t)rows_total * s->ld, 0.0);
            for (int64_t i = 0; i < rows_total; ++i) {
                std::memcpy(host.data() + i * s->ld, full.data() + i * ldf, sizeof(double) * s->n);
                host[(size_t)(i * s->ld + s->n)] = full[(size_t)(i * ldf + s->N)];
            }
        } else {
            host_tableau(prob, s->row_first, s->rows, s->ld, host, s->carry_local);
        }
        HIP_TRY(hipMemcpyAsync(s->T, host.data(), tbytes, hipMemcpyHostToDevice, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
    }
    std::vector<int32_t> basis(s->m);
    for (int64_t i = 0; i < s->m; ++i)
        basis[i] = s->general ? (prob->sf.art_col[i] >= 0 ? prob->sf.art_col[i] : prob->sf.slack_col[i])
                              : (int32_t)(s->n + i);
    HIP_TRY(hipMemcpyAsync(s->basis, basis.data(), sizeof(int32_t) * s->m, hipMemcpyHostToDevice,
                           s->stream));
    dlp::DevState st0{};
    for (int l = 0; l < dlp::kMaxDefer; ++l) st0.pl[l] = -1;
    st0.status = DLP_RUNNING;
    st0.q = -1;
    st0.p = -1;
    st0.p_local = -1;
    st0.leaving = -1;
    st0.bland = opt->pricing == DLP_PRICING_BLAND ? 1 : 0;
    st0.sq = -1;
    st0.bser = 0;
    st0.seal[0].ser = st0.seal[1].ser = -1;
    *s->host_st = st0;
    HIP_TRY(hipMemcpyAsync(s->st, s->host_st, sizeof(st0), hipMemcpyHostToDevice, s->stream));
    HIP_TRY(dlp::launch_cond_init(g, s->N, s->st, s->stream));
    HIP_TRY(dlp::launch_price_init(g, s->pp, opt->tol_dj, opt->update_variant, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->Tb[0] = s->T;
    clk.mark("create: fill + state");

    // lookahead: forced on, or auto at K = 64 on a streaming (> 1 GiB) tableau,
    // where the 64-step pass is long enough to hide the selection chain: C3 17 GB 4,492 -> 4,935
    // pivots/s (round 2), and round 4's rank geometries with the faster chain, 2.15 / 4.3 / 8.6 GB:
    // +8 / +8 / +18 % (profiles/r04g/).  Smaller K (cache-resident tableaus) stays off: the chain,
    // slowed by the concurrent pass and by replaying two blocks, costs more than the pass it hides
    // (C2 268 MB, K = 16: 39.0k -> 30.2k; profiles/r02h/).  An exchange session decides once its
    // exchange is known (la_policy): on with the peer exchange, off with RCCL.
    s->la_auto = opt->lookahead < 0;
    if (opt->lookahead == 1 || (s->la_auto && !s->exchange && s->d.K == 64 && streaming))
        CALL_TRY(la_enable(s, opt->lookahead == 1));
    s->opt.lookahead = s->la ? 1 : 0;
    pick_form(s);

    if (comm_in) {
        s->comm = comm_in;
        s->use_rccl = true;
    } else if (uid) {
        ncclUniqueId id;
        std::memcpy(&id, uid, sizeof(id));
        NCCL_TRY(ncclCommInitRank(&s->comm, nranks, id, rank));
        s->use_rccl = true;
    }
    s->xmode = s->use_rccl ? dlp_session::X_RCCL : dlp_session::X_HOST;
    s->ev_per_pivot = opt->timing == 1 ? 2 : (opt->timing >= 2 ? 5 : 0);
    if (s->ev_per_pivot) {
        s->ev.resize((size_t)s->ev_per_pivot * opt->check_interval);
        for (auto& e : s->ev) HIP_TRY(hipEventCreate(&e));
        s->ev_flush.assign(opt->check_interval, 0);
    }
    clk.mark("create: lookahead + comm");
    return DLP_OK;
}

// ---- one pivot, as stream-ordered launches ------------------------------
int enqueue_candidate(dlp_session* s) {
    const dlp_options& o = s->opt;
    HIP_TRY(dlp::launch_ratio(s->g, s->basis, s->basis, s->pp, s->st, s->colq, s->partials,
                              s->ratio_blocks, s->cand_send, s->exchange ? 2 : 1, o.tol_dj,
                              o.tol_piv,
                              o.pricing, s->log, s->log_cap, s->stream));
    return DLP_OK;
}
int enqueue_select(dlp_session* s) {
    const dlp_options& o = s->opt;
    if (s->exchange)
        HIP_TRY(dlp::launch_select(s->g, s->cand_recv, s->nranks, s->basis, s->st, o.pricing,
                                   s->log, s->log_cap, s->stream));
    return DLP_OK;
}
int enqueue_prow(dlp_session* s) {
    HIP_TRY(dlp::launch_prow(s->g, s->st, s->prow_send, s->nranks, s->stream));
    return DLP_OK;
}
int enqueue_update(dlp_session* s) {
    const dlp_options& o = s->opt;
    HIP_TRY(dlp::launch_update(s->g, s->colq, (const double*)s->prow_recv, s->st, s->pp, o.tol_dj,
                               s->log, s->log_cap, o.nontemporal != 0, o.update_variant,
                               s->stream));
    return DLP_OK;
}

// Deferred mode: the tableau pass of the pivots enqueued since the last one
// (a no-op on the device when the block is empty).
int enqueue_flush(dlp_session* s) {
    if (s->d.K <= 1) return DLP_OK;
    HIP_TRY(dlp::launch_flush_defer(s->g, s->d, s->st, s->opt.nontemporal != 0, s->defer_rb,
                                    s->defer_occ, s->stream));
    s->since_flush = 0;
    return DLP_OK;
}

// ---- lookahead --------------------------------------------
// The objective row lives in one buffer at a time (the pivot-row kernels update it
// in place, passes never touch it): move it along when the selections change buffer.
int la_move_z(dlp_session* s, int to) {
    if (s->zbuf == to) return DLP_OK;
    HIP_TRY(hipMemcpyAsync(s->Tb[to] + s->rows * s->ld, s->Tb[s->zbuf] + s->rows * s->ld,
                           sizeof(double) * s->width, hipMemcpyDeviceToDevice, s->stream));
    s->zbuf = to;
    return DLP_OK;
}

// Wait for the pass in flight; the selections then read its output, current again.
int la_drain(dlp_session* s) {
    if (!s->la_pending) return DLP_OK;
    HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_pass, 0));
    s->tread = s->tcur;
    s->la_pending = false;
    CALL_TRY(la_move_z(s, s->tread));
    s->T = s->g.T = s->Tb[s->tread];
    return DLP_OK;
}

// The lookahead pass's band publication: the form-21 pass counts its
// finished workgroups per band; the next block's selections read a finished band's rows
// from the pass's output (Tn) and replay their own block only.  DLP_BAND_PUB=0: off (A/B).
dlp::BandPub band_pub(const dlp_session* s) {
    static const bool off = std::getenv("DLP_BAND_PUB") && std::atoi(std::getenv("DLP_BAND_PUB")) == 0;
    dlp::BandPub b;
    if (!s->band_cnt || off) return b;
    b.cnt = s->band_cnt;
    b.stride = s->band_stride;
    b.rb = s->defer_rb;
    b.ntiles = dlp::band_pub_tiles(s->d.form, s->g.width);
    b.Tn = s->la_pending ? s->Tb[s->tcur] : nullptr;   // the pass in flight writes Tb[tcur]
    return b;
}

// End of a block: seal it, start its pass (Tb[tcur] -> the other buffer) on pstream
// behind the seal, and move the selections to the pass's source, which the previous
// pass (if one is in flight) must have finished writing.  drain: also wait for
// this pass (a window's end).
int la_block_end(dlp_session* s, bool drain, hipEvent_t* evp) {
    const dlp::BandPub bp = band_pub(s);
    HIP_TRY(dlp::launch_seal_defer(s->st, s->cur, s->stream, &bp));
    HIP_TRY(hipEventRecord(s->ev_seal, s->stream));
    HIP_TRY(hipStreamWaitEvent(s->pstream, s->ev_seal, 0));
    if (evp) HIP_TRY(hipEventRecord(evp[0], s->pstream));
    dlp::Geometry gp = s->g;
    gp.T = s->Tb[s->tcur];
    HIP_TRY(dlp::launch_flush_defer(gp, s->dslot[s->cur], s->st, s->opt.nontemporal != 0, s->defer_rb,
                                    s->defer_occ, s->pstream, s->Tb[1 - s->tcur], s->cur, &bp));
    if (evp) HIP_TRY(hipEventRecord(evp[1], s->pstream));
    if (s->la_pending) HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_pass, 0));   // previous pass
    HIP_TRY(hipEventRecord(s->ev_pass, s->pstream));                            // this pass
    s->tread = s->tcur;
    s->tcur = 1 - s->tcur;
    s->la_pending = true;
    s->cur = 1 - s->cur;
    s->since_flush = 0;
    CALL_TRY(la_move_z(s, s->tread));
    s->T = s->g.T = s->Tb[s->tread];
    if (drain) CALL_TRY(la_drain(s));
    return DLP_OK;
}

// Back to the single-buffer path (step API, a pass form without an out-of-place
// instance): finish what is in flight; slot 0's arrays serve the in-place blocks.
int la_disable(dlp_session* s) {
    if (!s->la) return DLP_OK;
    if (s->since_flush > 0) CALL_TRY(la_block_end(s, true, nullptr));
    CALL_TRY(la_drain(s));
    HIP_TRY(hipStreamSynchronize(s->stream));
    const int form = s->d.form;
    s->d = s->dslot[0];
    s->d.form = form;
    s->la = false;
    s->opt.lookahead = 0;
    CALL_TRY(chain_cus_apply(s, 0));   // the pass runs on the chain's stream again: every CU
    pick_form(s);
    return DLP_OK;
}

// The single-buffer path's pending block applied (la_enable's precondition).
int flush_pending_block(dlp_session* s) {
    if (!s->la && s->d.K > 1 && s->since_flush > 0) CALL_TRY(enqueue_flush(s));
    return DLP_OK;
}

// An exchange session's auto lookahead, once its exchange is known (creation, connect,
// dlp_session_set_exchange; between runs): with the peer exchange, the single-rank rule (K = 64 on
// a streaming tableau), where every per-pivot kernel fits beside the form-21 pass (the LEAN ratio
// and pivot-row launches, with the selection and the commit inside: <= 32 VGPRs,
// tests/test_isa.py).  Measured on the C3 rank geometries at P = 8 / 4 / 2 (c3r8 / c3r4 / c3r2):
// 23,012 vs 21,358, 17,098 vs 15,881, 11,980 vs 10,183 pivots/s (profiles/r04g/).  With RCCL only
// where the chain gets CUs of its own (chain_cus_policy > 0: a rank of up to 32k rows): RCCL's
// collective kernels need more registers than the pass leaves on a CU and would each wait for pass
// workgroups to drain, but on a disjoint CU mask they never share a CU with the pass
// (round 5; profiles/r05*/).  That RCCL case is measured and tested only on a
// 1-rank communicator (bench.py --workload c3r8, test_rccl_rank_session_lookahead_on_cu_split):
// RCCL collectives on a CU-masked chain stream beside the pass across real ranks have never run,
// and RCCL is the path a multi-GPU run falls back to, so with nranks > 1 it is opt-in
// (DLP_RCCL_LOOKAHEAD=1).  A caller's explicit lookahead setting is kept.
bool rccl_lookahead_ok(const dlp_session* s) {
    if (s->nranks == 1) return true;
    const char* e = std::getenv("DLP_RCCL_LOOKAHEAD");
    return e && std::atoi(e) == 1;
}

int la_policy(dlp_session* s) {
    if (!s->la_auto || !s->exchange) return DLP_OK;
    const bool rccl_split = s->xmode == dlp_session::X_RCCL && rccl_lookahead_ok(s) && chain_cus_policy(s) > 0;
    const bool want = (s->xmode == dlp_session::X_PEER || rccl_split) && s->d.K == 64 && s->streaming &&
                      !s->general;
    if (want && !s->la) CALL_TRY(la_enable(s, false));
    if (s->la && s->pstream) CALL_TRY(la_streams(s));   // (the split may have changed with the exchange)
    // RCCL beside the pass only on a CU split that really exists (a masked queue may be refused)
    if (s->la && s->xmode == dlp_session::X_RCCL && s->chain_cus == 0) CALL_TRY(la_disable(s));
    if (!want && s->la) CALL_TRY(la_disable(s));
    pick_form(s);
    return DLP_OK;
}

// DLP_PEER_ONELAUNCH=1: a peer pivot as one launch (read per pivot, so tests can switch it)
bool peer_onelaunch() {
    const char* e = std::getenv("DLP_PEER_ONELAUNCH");
    return e && std::atoi(e) == 1;
}

// The one-launch peer pivot applies: 256-lane ratio workgroups, or 128-lane ones when the chain owns
// its CUs (the ring instance covers them with 256 lanes); the condensed tableau's entering slot
// travels in the selection record
bool onelaunch_ok(const dlp_session* s) {
    if (!peer_onelaunch()) return false;
    if (s->chain_cus > 0 && s->d.K == 64)   // the ring instance (launch_pivot_x)
        return s->g.rthreads == 128 || s->g.rthreads == dlp::kRatioDeferThreads;
    // the LEAN instance beside the pass (lookahead on shared CUs) has no condensed build
    return s->g.rthreads == dlp::kRatioDeferThreads && !(s->g.cd.on && s->la);
}

// The exchange kernels' peer table (X_PEER) or NULL.
inline const dlp::XPeers* xp_of(const dlp_session* s) {
    return s->xmode == dlp_session::X_PEER ? s->xpeers : nullptr;
}

// One deferred pivot: replayed ratio test, exchange, replayed pivot row (+
// objective row and pricing), and the pass when the block is full or `last`.
// Three phases, so that dlp_sessions_run can interleave the ranks of one device
// (every rank's phase p is enqueued before any rank's phase p + 1: a wait for a
// peer's message is then always queued after the launch that sends it):
//   0 ratio test (+ candidate send) | 1 select (+ wait) + pivot row (+ send) |
//   2 commit (+ wait) + pass
int pivot_defer_phase(dlp_session* s, int phase, int64_t slot, bool last) {
    const dlp_options& o = s->opt;
    const dlp::XPeers* xp = xp_of(s);
    const bool xf = xp && s->xfuse;   // selection + commit inside the chain launches
    // timing 2: 5 events per pivot (every phase); timing 1: 2 events around the pass only
    hipEvent_t* ev = s->ev_per_pivot == 5 ? &s->ev[(size_t)slot * 5] : nullptr;
    hipEvent_t* evp = s->ev_per_pivot == 2 ? &s->ev[(size_t)slot * 2] : nullptr;
    // lookahead: the selections read Tb[tread] and replay the sealed block in flight first
    dlp::Geometry gsel = s->g;
    const dlp::Defer* dcur = &s->d;
    const dlp::Defer* dprev = nullptr;
    int pseal = -1;
    const dlp::BandPub bp = band_pub(s);
    if (s->la) {
        gsel.T = s->Tb[s->tread];
        dcur = &s->dslot[s->cur];
        if (s->la_pending) {
            dprev = &s->dslot[1 - s->cur];
            pseal = 1 - s->cur;
        }
    }
    if (phase == 0) {
        if (ev) HIP_TRY(hipEventRecord(ev[0], s->stream));
        if (!s->la && !s->exchange && s->fuse_pivot && s->fuse_fits && !s->g.cd.on && !ev) {
            // single rank: ratio test, selection and pivot row in one launch
            HIP_TRY(dlp::launch_pivot_defer(s->g, s->d, s->basis, s->pp, s->st, s->partials,
                                            s->ratio_blocks_max, o.tol_dj, o.tol_piv, o.pricing, s->log,
                                            s->log_cap, s->stream));
            return DLP_OK;
        }
        // peer exchange, DLP_PEER_ONELAUNCH=1 (opt-in): the whole pivot in ONE launch (ratio test,
        // selection, the selection record to the pivot-row workgroups, row push, commit).  Bit-exact,
        // but 1-3 % slower than two launches at the C3 rank geometries: the record's hand-off and its
        // ~130 pollers cost what the launch boundary did (profiles/r04i/, r04j/)
        if (xf && onelaunch_ok(s)) {
            s->xseq_c += 1;
            s->xseq_r += 1;   // (equal: every pivot, drive-out and carry step advances both)
            HIP_TRY(dlp::launch_pivot_x(gsel, *dcur, s->basis, s->pp, s->st, o.tol_dj, o.tol_piv, o.pricing, s->log,
                                        s->log_cap, s->stream, dprev, pseal, xp, s->xseq_c, &bp, s->chain_cus > 0));
            if (ev) HIP_TRY(hipEventRecord(ev[1], s->stream));
            return DLP_OK;
        }
        if (xp) s->xseq_c += 1;
        HIP_TRY(dlp::launch_ratio_defer(gsel, *dcur, s->basis, s->pp, s->st, s->partials,
                                        s->ratio_blocks_max, s->cand_send, s->exchange ? 2 : 1, o.tol_dj,
                                        o.tol_piv, o.pricing, s->log, s->log_cap, s->stream, dprev,
                                        pseal, xp, s->xseq_c, &bp, xf, s->chain_cus > 0));
        if (ev) HIP_TRY(hipEventRecord(ev[1], s->stream));
        if (s->xmode == dlp_session::X_RCCL)
            NCCL_TRY(ncclAllGather(s->cand_send, s->cand_recv, sizeof(dlp::Cand), ncclUint8, s->comm,
                                   s->stream));
        return DLP_OK;
    }
    if (phase == 1) {
        if (!s->la && !s->exchange && s->fuse_pivot && s->fuse_fits && !s->g.cd.on && !ev) return DLP_OK;
        if (xf && onelaunch_ok(s)) {   // (the whole pivot ran in phase 0's launch)
            if (ev) HIP_TRY(hipEventRecord(ev[2], s->stream));
            return DLP_OK;
        }
        if (s->exchange && !xf)
            HIP_TRY(dlp::launch_select(s->g, s->cand_recv, s->nranks, s->basis, s->st, o.pricing,
                                       s->log, s->log_cap, s->stream, false, true, xp, s->xseq_c));
        if (ev) HIP_TRY(hipEventRecord(ev[2], s->stream));
        if (xp) s->xseq_r += 1;
        HIP_TRY(dlp::launch_prow_defer(gsel, *dcur, s->st, s->prow_send, s->pp, o.tol_dj, s->log,
                                       s->log_cap, s->exchange ? 2 : 1, s->stream, dprev, pseal, xp,
                                       s->xseq_r, &bp, xf, s->chain_cus > 0));
        if (s->xmode == dlp_session::X_RCCL)
            NCCL_TRY(ncclAllReduce(s->prow_send, s->prow_recv, (size_t)s->ld, ncclInt64, ncclMax,
                                   s->comm, s->stream));
        return DLP_OK;
    }
    if (s->exchange && !xf)
        HIP_TRY(dlp::launch_commit_defer(gsel, *dcur, s->st, s->prow_recv, s->pp, o.tol_dj, s->log,
                                         s->log_cap, s->stream, xp, s->xseq_r));
    if (ev) HIP_TRY(hipEventRecord(ev[3], s->stream));
    s->since_flush += 1;
    const bool flush = last || s->since_flush >= s->d.K;
    if (flush && s->la) {
        CALL_TRY(la_block_end(s, last, evp));
    } else {
        if (flush && evp) HIP_TRY(hipEventRecord(evp[0], s->stream));
        if (flush) CALL_TRY(enqueue_flush(s));
        if (flush && evp) HIP_TRY(hipEventRecord(evp[1], s->stream));
    }
    if (ev) HIP_TRY(hipEventRecord(ev[4], s->stream));
    if (ev || evp) s->ev_flush[slot] = flush ? 1 : 0;
    return DLP_OK;
}

// Small LPs: `count` pivots in one launch, the tableau in LDS; the HBM tableau,
// basis, log and state are current afterwards, and the pricing partials are
// rebuilt so that the multi-kernel path (the step API) can continue from it.
int enqueue_cluster(dlp_session* s, int64_t count) {
    const dlp_options& o = s->opt;
    hipEvent_t* ev = s->ev_per_pivot ? &s->ev[0] : nullptr;
    if (ev)
        for (int k = 0; k < s->ev_per_pivot - 1; ++k) HIP_TRY(hipEventRecord(ev[k], s->stream));
    // diagnostic: DLP_CLUSTER_STAMPS=<file> dumps s_memtime per phase of the first 64 pivots
    // of the first window (tools only; never set in a timed run)
    static const char* stamp_path = std::getenv("DLP_CLUSTER_STAMPS");
    uint64_t* stamps = nullptr;
    if (stamp_path) {
        HIP_TRY(hipMalloc(&stamps, sizeof(uint64_t) * 16 * 64 * s->cl_wg));
        HIP_TRY(hipMemsetAsync(stamps, 0, sizeof(uint64_t) * 16 * 64 * s->cl_wg, s->stream));
    }
    HIP_TRY(dlp::launch_cluster(s->g, s->m, s->n, s->cl_wg, s->cl_cw, s->st, s->basis, s->log,
                                s->log_cap, s->cl_gran, count, o.pricing, o.tol_dj, o.tol_piv,
                                s->stream, stamps));
    if (stamps) {
        std::vector<uint64_t> h(16 * 64 * s->cl_wg);
        HIP_TRY(hipMemcpyAsync(h.data(), stamps, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost,
                               s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        HIP_TRY(hipFree(stamps));
        if (FILE* f = std::fopen(stamp_path, "wb")) {
            std::fwrite(h.data(), sizeof(uint64_t), h.size(), f);
            std::fclose(f);
        }
    }
    if (ev) HIP_TRY(hipEventRecord(ev[s->ev_per_pivot - 1], s->stream));
    HIP_TRY(dlp::launch_price_init(s->g, s->pp, o.tol_dj, o.update_variant, s->stream));
    s->ev_pending = ev ? 1 : 0;
    return DLP_OK;
}

// One eager pivot in the same three phases (pivot_defer_phase).
int pivot_eager_phase(dlp_session* s, int phase, int64_t slot) {
    const dlp::XPeers* xp = xp_of(s);
    hipEvent_t* ev = s->ev_per_pivot ? &s->ev[(size_t)slot * s->ev_per_pivot] : nullptr;
    const bool all = s->ev_per_pivot == 5;
    if (phase == 0) {
        if (all) HIP_TRY(hipEventRecord(ev[0], s->stream));
        CALL_TRY(enqueue_candidate(s));
        if (xp) HIP_TRY(dlp::launch_xcand_send(xp, ++s->xseq_c, s->cand_send, s->st, s->stream));
        if (all) HIP_TRY(hipEventRecord(ev[1], s->stream));
        if (s->xmode == dlp_session::X_RCCL)
            NCCL_TRY(ncclAllGather(s->cand_send, s->cand_recv, sizeof(dlp::Cand), ncclUint8, s->comm,
                                   s->stream));
        return DLP_OK;
    }
    if (phase == 1) {
        if (s->exchange)
            HIP_TRY(dlp::launch_select(s->g, s->cand_recv, s->nranks, s->basis, s->st, s->opt.pricing,
                                       s->log, s->log_cap, s->stream, false, false, xp, s->xseq_c));
        if (all) HIP_TRY(hipEventRecord(ev[2], s->stream));
        CALL_TRY(enqueue_prow(s));
        if (xp)
            HIP_TRY(dlp::launch_xrow_send(xp, ++s->xseq_r, s->prow_send, s->ld, s->st, -1, s->rank,
                                          s->stream));
        if (s->xmode == dlp_session::X_RCCL)
            NCCL_TRY(ncclAllReduce(s->prow_send, s->prow_recv, (size_t)s->ld, ncclInt64, ncclMax,
                                   s->comm, s->stream));
        return DLP_OK;
    }
    if (xp) HIP_TRY(dlp::launch_xrow_recv(xp, s->xseq_r, s->ld, s->prow_recv, s->st, s->stream));
    if (all) HIP_TRY(hipEventRecord(ev[3], s->stream));
    if (s->ev_per_pivot == 2) HIP_TRY(hipEventRecord(ev[0], s->stream));
    CALL_TRY(enqueue_update(s));
    if (all) HIP_TRY(hipEventRecord(ev[4], s->stream));
    if (s->ev_per_pivot == 2) HIP_TRY(hipEventRecord(ev[1], s->stream));
    return DLP_OK;
}

int pivot_phase(dlp_session* s, int phase, int64_t slot, bool last) {
    return s->d.K > 1 ? pivot_defer_phase(s, phase, slot, last) : pivot_eager_phase(s, phase, slot);
}

int enqueue_pivot(dlp_session* s, int64_t slot, bool last = true) {
    for (int ph = 0; ph < 3; ++ph) CALL_TRY(pivot_phase(s, ph, slot, last));
    return DLP_OK;
}

// General LPs: forced drive-out pivot on global row `row` (same exchange shape
// as a pivot: candidate exchange, pivot-row exchange), in the same three phases.
int enqueue_forced_candidate(dlp_session* s, int64_t row) {
    const dlp_options& o = s->opt;
    HIP_TRY(dlp::launch_drive(s->g, row, s->basis, s->st, o.tol_piv, s->cand_send,
                              s->exchange ? 2 : 1, o.pricing, s->log, s->log_cap, s->colq,
                              s->stream));
    return DLP_OK;
}
int enqueue_forced_select(dlp_session* s) {
    if (s->exchange) {
        HIP_TRY(dlp::launch_select(s->g, s->cand_recv, s->nranks, s->basis, s->st, s->opt.pricing,
                                   s->log, s->log_cap, s->stream, true, false, xp_of(s), s->xseq_c));
        HIP_TRY(dlp::launch_gather_q(s->g, s->st, s->colq, s->stream));
    }
    return enqueue_prow(s);
}
int forced_phase(dlp_session* s, int phase, int64_t row) {
    const dlp::XPeers* xp = xp_of(s);
    if (phase == 0) {
        CALL_TRY(enqueue_forced_candidate(s, row));
        if (xp) HIP_TRY(dlp::launch_xcand_send(xp, ++s->xseq_c, s->cand_send, s->st, s->stream));
        if (s->xmode == dlp_session::X_RCCL)
            NCCL_TRY(ncclAllGather(s->cand_send, s->cand_recv, sizeof(dlp::Cand), ncclUint8, s->comm,
                                   s->stream));
        return DLP_OK;
    }
    if (phase == 1) {
        CALL_TRY(enqueue_forced_select(s));
        if (xp)
            HIP_TRY(dlp::launch_xrow_send(xp, ++s->xseq_r, s->prow_send, s->ld, s->st, -1, s->rank,
                                          s->stream));
        if (s->xmode == dlp_session::X_RCCL)
            NCCL_TRY(ncclAllReduce(s->prow_send, s->prow_recv, (size_t)s->ld, ncclInt64, ncclMax,
                                   s->comm, s->stream));
        return DLP_OK;
    }
    if (xp) HIP_TRY(dlp::launch_xrow_recv(xp, s->xseq_r, s->ld, s->prow_recv, s->st, s->stream));
    return enqueue_update(s);
}
int enqueue_forced(dlp_session* s, int64_t row) {
    for (int ph = 0; ph < 3; ++ph) CALL_TRY(forced_phase(s, ph, row));
    return DLP_OK;
}
// Carried Phase II objective row -> objective row on every rank.
int enqueue_carry_out(dlp_session* s) {
    HIP_TRY(dlp::launch_carry_out(s->g, s->carry_local, s->prow_send, s->stream));
    return DLP_OK;
}
int enqueue_carry_in(dlp_session* s) {
    HIP_TRY(dlp::launch_carry_in(s->g, s->prow_recv, s->st, s->opt.pricing, s->stream));
    HIP_TRY(dlp::launch_price_init(s->g, s->pp, s->opt.tol_dj, s->opt.update_variant, s->stream));
    return DLP_OK;
}
// Peer exchange: the carried row may only overwrite a rank's row region after that rank
// has read the previous pivot row, so the carry starts with an empty candidate exchange
// (a barrier: every rank's select-wait sees every rank's message).
int carry_phase(dlp_session* s, int phase) {
    const dlp::XPeers* xp = xp_of(s);
    if (phase == 0) {
        // the last drive-out pivot may have left the skip status (a redundant row): the
        // carry runs whatever it is (carry_in sets "running" again), and the peer kernels
        // below act only while running
        HIP_TRY(dlp::launch_set_status(s->st, DLP_RUNNING, s->stream));
        if (xp) {
            HIP_TRY(hipMemsetAsync(s->cand_send, 0, sizeof(dlp::Cand), s->stream));
            HIP_TRY(dlp::launch_xcand_send(xp, ++s->xseq_c, s->cand_send, s->st, s->stream));
        }
        return DLP_OK;
    }
    if (phase == 1) {
        if (xp) HIP_TRY(dlp::launch_xwait(xp, s->xseq_c, s->st, s->stream));
        CALL_TRY(enqueue_carry_out(s));
        if (xp)
            HIP_TRY(dlp::launch_xrow_send(xp, ++s->xseq_r, s->prow_send, s->ld, s->st, s->nranks - 1,
                                          s->rank, s->stream));
        if (s->xmode == dlp_session::X_RCCL)
            NCCL_TRY(ncclAllReduce(s->prow_send, s->prow_recv, (size_t)s->ld, ncclInt64, ncclMax,
                                   s->comm, s->stream));
        return DLP_OK;
    }
    if (xp) HIP_TRY(dlp::launch_xrow_recv(xp, s->xseq_r, s->ld, s->prow_recv, s->st, s->stream));
    return enqueue_carry_in(s);
}
int enqueue_carry(dlp_session* s) {
    for (int ph = 0; ph < 3; ++ph) CALL_TRY(carry_phase(s, ph));
    return DLP_OK;
}

int poll(dlp_session* s);

// Phase I optimum reached (device status "optimal" in phase 1): decide
// infeasibility from the Phase I objective, queue the drive-out pivots of the
// rows whose basic variable is artificial (replicated basis: every rank
// queues the same rows) and the carried-row switch.
int begin_phase2(dlp_session* s) {
    double zN = 0.0;
    std::vector<int32_t> basis(s->m);
    HIP_TRY(hipMemcpyAsync(&zN, s->T + s->rows * s->ld + s->N, sizeof(double),
                           hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipMemcpyAsync(basis.data(), s->basis, sizeof(int32_t) * s->m, hipMemcpyDeviceToHost,
                           s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->phase1_pivots = s->npivots;
    s->step_void = true;   // a caller-driven step begun in Phase I is void
    if (zN < -s->opt.tol_feas * (1.0 + s->bmax)) {
        s->status = DLP_INFEASIBLE;
        s->phase = 3;
        return DLP_OK;
    }
    s->drive.clear();
    for (int64_t i = 0; i < s->m; ++i)
        if (basis[i] >= s->nprice) s->drive.push_back((int32_t)i);
    s->drive_next = 0;
    s->carry_pending = true;
    s->phase = 2;
    s->status = DLP_RUNNING;
    HIP_TRY(dlp::launch_set_status(s->st, DLP_RUNNING, s->stream));
    return DLP_OK;
}

// After the carry-in: the Phase I pivot count (drive-out included) is final.
int finish_phase1(dlp_session* s) {
    s->carry_pending = false;
    CALL_TRY(poll(s));
    s->phase1_pivots = s->npivots;
    return DLP_OK;
}

// Abort the RCCL communicator (its kernels in flight return) and fail the window.
int abort_exchange(dlp_session* s, const std::string& why) {
    if (s->xabort) __atomic_store_n(s->xabort, 1u, __ATOMIC_SEQ_CST);   // ends the device waits
    if (s->comm) {
        (void)ncclCommAbort(s->comm);   // frees the communicator; pending collectives exit
        s->comm = nullptr;
    }
    s->use_rccl = false;
    s->status = DLP_ERR_RCCL;
    set_error("exchange aborted: " + why);
    return DLP_ERR_RCCL;
}

// Wait for the session stream.  A single-GPU session blocks in hipStreamSynchronize; an
// exchange session polls hipStreamQuery, so that a peer that never arrives (a failed rank,
// a dead process) ends the wait: ncclCommGetAsyncError, the in-process group's failure word,
// dlp_session_abort and a stall limit each abort the communicator and return DLP_ERR_RCCL.
int wait_stream(dlp_session* s) {
    if (s->fault_after_polls >= 0 && s->npolls++ >= s->fault_after_polls) {
        s->fault_after_polls = -1;
        (void)hipStreamSynchronize(s->stream);
        if (s->exchange && s->xmode != dlp_session::X_HOST)
            return abort_exchange(s, "injected fault (dlp_session_inject_fault)");
        set_error("injected fault (dlp_session_inject_fault)");
        return DLP_ERR_HIP;
    }
    if (!s->exchange || s->xmode == dlp_session::X_HOST) {
        HIP_TRY(hipStreamSynchronize(s->stream));
        return DLP_OK;
    }
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (int64_t spin = 0;; ++spin) {
        const hipError_t e = hipStreamQuery(s->stream);
        if (e == hipSuccess) return DLP_OK;
        if (e != hipErrorNotReady) {   // a device error, not an exchange one: DLP_ERR_HIP
            (void)abort_exchange(s, hipGetErrorString(e));
            s->status = DLP_ERR_HIP;
            set_error(std::string("hipStreamQuery: ") + hipGetErrorString(e));
            return DLP_ERR_HIP;
        }
        if (s->abort_req.load(std::memory_order_relaxed)) return abort_exchange(s, "dlp_session_abort");
        if (s->group_failed) {
            const int f = s->group_failed->load(std::memory_order_relaxed);
            if (f >= 0 && f != s->rank) return abort_exchange(s, "rank " + std::to_string(f) + " failed");
        }
        if (s->comm && (spin & 63) == 0) {
            ncclResult_t ae = ncclSuccess;
            if (ncclCommGetAsyncError(s->comm, &ae) == ncclSuccess && ae != ncclSuccess &&
                ae != ncclInProgress)
                return abort_exchange(s, std::string("RCCL async error: ") + ncclGetErrorString(ae));
        }
        const double el = std::chrono::duration<double>(clk::now() - t0).count();
        if (s->stall_limit_s > 0 && el > s->stall_limit_s)
            return abort_exchange(s, "window not complete after " + std::to_string(el) +
                                         " s (exchange timeout)");
        if (spin < 2000)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Sync, read the device state, fold event timings of pivots that really ran.
int poll(dlp_session* s) {
    const int64_t before = s->npivots;
    HIP_TRY(hipMemcpyAsync(s->host_st, s->st, sizeof(dlp::DevState), hipMemcpyDeviceToHost,
                           s->stream));
    CALL_TRY(wait_stream(s));
    s->npivots = s->host_st->npivots;
    if (s->host_st->status == dlp::kStatusXFail) {   // an exchange failure, as every other one
        s->status = DLP_ERR_RCCL;
        set_error("exchange aborted: a peer-exchange wait for another rank timed out or was aborted (rank " +
                  std::to_string(s->rank) + ")");
        return DLP_ERR_RCCL;
    }
    if (s->host_st->status != DLP_RUNNING && s->host_st->status != dlp::kStatusSkip &&
        s->status == DLP_RUNNING)
        s->status = s->host_st->status;
    if (s->cluster && s->ev_per_pivot && s->ev_pending > 0) {   // one launch per window
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, s->ev[0], s->ev[s->ev_per_pivot - 1]));
        s->timings[DLP_PHASE_UPDATE] += ms;
        s->nsamples += s->npivots - before;
        s->upd_launches += 1;
        s->ev_pending = 0;
    }
    if (s->ev_per_pivot && s->ev_pending > 0) {
        const int64_t real = std::min<int64_t>(s->ev_pending, s->npivots - before);
        for (int64_t k = 0; k < real; ++k) {
            hipEvent_t* ev = &s->ev[(size_t)k * s->ev_per_pivot];
            float ms = 0.f;
            if (s->ev_per_pivot == 2) {
                // deferred: only slots that ended with a pass recorded their events
                if (s->d.K <= 1 || s->ev_flush[k]) {
                    HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[1]));
                    s->timings[DLP_PHASE_UPDATE] += ms;
                }
            } else {
                for (int ph = 0; ph < 4; ++ph) {
                    HIP_TRY(hipEventElapsedTime(&ms, ev[ph], ev[ph + 1]));
                    s->timings[ph] += ms;
                }
            }
            s->upd_launches += (s->d.K > 1) ? s->ev_flush[k] : 1;
        }
        // deferred, solve ended inside the window: the pass that applied the last real
        // pivots ran in a later slot (the window's closing one), fold that one too
        if (s->d.K > 1 && s->ev_per_pivot == 2 && real > 0 && real < s->ev_pending &&
            !s->ev_flush[real - 1]) {
            for (int64_t k = real; k < s->ev_pending; ++k) {
                if (!s->ev_flush[k]) continue;
                hipEvent_t* ev = &s->ev[(size_t)k * 2];
                float ms = 0.f;
                HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[1]));
                s->timings[DLP_PHASE_UPDATE] += ms;
                s->upd_launches += 1;
                break;
            }
        }
        s->nsamples += real;
    }
    s->ev_pending = 0;
    if (s->general && s->phase == 1 && s->status == DLP_OK) CALL_TRY(begin_phase2(s));
    return DLP_OK;
}

int run_window_graph(dlp_session* s, int64_t chunk) {
    if (!s->gexec || s->graph_chunk != chunk) {
        if (s->gexec) { (void)hipGraphExecDestroy(s->gexec); s->gexec = nullptr; }
        if (s->graph) { (void)hipGraphDestroy(s->graph); s->graph = nullptr; }
        StageClock clk;
        HIP_TRY(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
        int rc = DLP_OK;
        for (int64_t k = 0; k < chunk && rc == DLP_OK; ++k) rc = enqueue_pivot(s, 0, k == chunk - 1);
        hipGraph_t gr = nullptr;
        hipError_t e = hipStreamEndCapture(s->stream, &gr);
        if (rc != DLP_OK) return rc;
        HIP_TRY(e);
        clk.mark("run: graph capture");
        s->graph = gr;
        HIP_TRY(hipGraphInstantiate(&s->gexec, s->graph, nullptr, nullptr, 0));
        clk.mark("run: graph instantiate");
        s->graph_chunk = chunk;
    }
    HIP_TRY(hipGraphLaunch(s->gexec, s->stream));
    return DLP_OK;
}

// General LP results in user terms (include/dlp.h, "general LPs": results).
// Before Phase II has started (infeasible, or a pivot limit in Phase I) the
// objective is NaN and y is zero; x is the current (Phase I) point.
int general_result(dlp_session* s, const std::vector<double>& z, const std::vector<double>& rhs,
                   dlp_result* r, int64_t row_first, int64_t rows_elig) {
    const dlp::StdForm& f = s->prob_dims.sf;
    const int64_t mu = s->prob_dims.m, nu = s->prob_dims.n;
    r->m = mu;
    r->n = nu;
    r->phase1_pivots = s->phase == 1 ? s->npivots : s->phase1_pivots;
    std::vector<double> xs(f.ns, 0.0);
    for (int64_t il = 0; il < rows_elig; ++il) {
        const int32_t v = r->basis[row_first + il];
        if (v < f.ns) xs[v] = rhs[il];
    }
    r->x.resize(nu);
    for (int64_t j = 0; j < nu; ++j) {
        const int32_t k = f.var_col[j];
        switch (f.var_kind[j]) {
            case dlp::VAR_LO: r->x[j] = f.var_const[j] + xs[k]; break;
            case dlp::VAR_HI: r->x[j] = f.var_const[j] - xs[k]; break;
            default: r->x[j] = xs[k] - xs[k + 1]; break;
        }
    }
    r->y.assign(mu, 0.0);
    const bool phase2 = s->phase == 2 && !s->carry_pending;
    if (!phase2) {
        r->objective = NAN;
        return DLP_OK;
    }
    r->objective = f.obj_sign * z[s->N] + f.obj_const;
    for (int64_t i = 0; i < f.m; ++i) {
        if (f.user_row[i] < 0) continue;
        const int32_t ident = f.type[i] == dlp::ROW_L ? f.slack_col[i] : f.art_col[i];
        r->y[f.user_row[i]] += f.obj_sign * f.row_sign[i] * z[ident];
    }
    return DLP_OK;
}

// The RHS column entries of this rank's ratio-eligible rows (the values of their
// basic variables).
// Condensed tableau: the slot of every variable (-1: basic).
int cond_slots(dlp_session* s, std::vector<int32_t>& slot_of) {
    slot_of.resize(s->N);
    HIP_TRY(hipMemcpyAsync(slot_of.data(), s->g.cd.slot_of, sizeof(int32_t) * s->N, hipMemcpyDeviceToHost,
                           s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return DLP_OK;
}

// z (the stored objective row, ld doubles) -> the full row in variable order (basic: +0, RHS at N).
int cond_expand_z(dlp_session* s, std::vector<double>& z) {
    std::vector<int32_t> so;
    CALL_TRY(cond_slots(s, so));
    std::vector<double> f(std::max<int64_t>(round16(s->N + 1), s->N + 1), 0.0);
    for (int64_t v = 0; v < s->N; ++v)
        if (so[v] >= 0) f[v] = z[so[v]];
    f[s->N] = z[s->g.ncols];
    z.swap(f);
    return DLP_OK;
}

// Rows [first, first + count) of a condensed session (the objective row is local row `rows`) in
// the full tableau's layout, ldl doubles per row: a nonbasic variable's entry from its slot, a
// basic one's unit entry (1 in its row, +0 elsewhere and in the objective row), the RHS at N.
int cond_read_rows(dlp_session* s, int64_t first, int64_t count, double* host, int64_t ldl) {
    std::vector<double> c((size_t)count * s->ld);
    HIP_TRY(hipMemcpyAsync(c.data(), s->T + first * s->ld, sizeof(double) * count * s->ld,
                           hipMemcpyDeviceToHost, s->stream));
    std::vector<int32_t> basis(s->m);
    HIP_TRY(hipMemcpyAsync(basis.data(), s->basis, sizeof(int32_t) * s->m, hipMemcpyDeviceToHost, s->stream));
    std::vector<int32_t> so;
    CALL_TRY(cond_slots(s, so));   // (synchronises the stream)
    for (int64_t k = 0; k < count; ++k) {
        const double* src = c.data() + k * s->ld;
        double* dst = host + k * ldl;
        for (int64_t v = 0; v < ldl; ++v) dst[v] = 0.0;
        for (int64_t v = 0; v < s->N; ++v)
            if (so[v] >= 0) dst[v] = src[so[v]];
        dst[s->N] = src[s->g.ncols];
        const int64_t il = first + k;
        if (il < s->rows) {
            const int32_t bv = basis[s->row_first + il];
            if (bv >= 0 && bv < s->N) dst[bv] = 1.0;
        }
    }
    return DLP_OK;
}

int local_rhs(dlp_session* s, std::vector<double>& rhs) {
    HIP_TRY(hipSetDevice(s->device));
    rhs.assign(s->g.rows_elig, 0.0);
    if (s->g.rows_elig > 0) {
        HIP_TRY(dlp::launch_gather_column(s->T, s->ld, s->rows, s->g.ncols, s->colq, s->stream));
        HIP_TRY(hipMemcpyAsync(rhs.data(), s->colq, sizeof(double) * s->g.rows_elig,
                               hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
    }
    return DLP_OK;
}

// rhs_all != NULL: the eligible rows of EVERY rank in global row order (an
// in-process row-block solve), so x covers all basic variables; else this
// rank's rows only.
int extract_result(dlp_session* s, dlp_result* r, const std::vector<double>* rhs_all = nullptr) {
    HIP_TRY(hipSetDevice(s->device));
    CALL_TRY(poll(s));
    r->m = s->m;
    r->n = s->n;
    r->status = s->status == DLP_RUNNING ? DLP_PIVOT_LIMIT : s->status;
    r->npivots = s->npivots;
    std::vector<double> z(s->ld), rhs(s->rows);
    HIP_TRY(hipMemcpyAsync(z.data(), s->T + s->rows * s->ld, sizeof(double) * s->ld,
                           hipMemcpyDeviceToHost, s->stream));
    if (s->rows > 0) {
        HIP_TRY(dlp::launch_gather_column(s->T, s->ld, s->rows, s->g.ncols, s->colq, s->stream));
        HIP_TRY(hipMemcpyAsync(rhs.data(), s->colq, sizeof(double) * s->rows,
                               hipMemcpyDeviceToHost, s->stream));
    }
    r->basis.resize(s->m);
    HIP_TRY(hipMemcpyAsync(r->basis.data(), s->basis, sizeof(int32_t) * s->m,
                           hipMemcpyDeviceToHost, s->stream));
    const int64_t nlog = std::min(s->npivots, s->log_cap);
    r->log.resize(nlog);
    if (nlog > 0)
        HIP_TRY(hipMemcpyAsync(r->log.data(), s->log, sizeof(dlp_pivot) * nlog,
                               hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (s->g.cd.on) CALL_TRY(cond_expand_z(s, z));   // the objective row in variable order
    for (int ph = 0; ph < DLP_NUM_PHASES; ++ph) r->timings[ph] = s->timings[ph];
    const std::vector<double>& rh = rhs_all ? *rhs_all : rhs;
    const int64_t rows_elig = rhs_all ? (int64_t)rhs_all->size() : s->g.rows_elig;
    const int64_t row_first = rhs_all ? 0 : s->row_first;
    if (s->general) return general_result(s, z, rh, r, row_first, rows_elig);
    r->objective = z[s->N];
    r->x.assign(s->n, 0.0);
    for (int64_t il = 0; il < rows_elig; ++il) {
        const int32_t v = r->basis[row_first + il];
        if (v < s->n) r->x[v] = rh[il];
    }
    r->y.resize(s->m);
    for (int64_t i = 0; i < s->m; ++i) r->y[i] = z[s->n + i];
    return DLP_OK;
}

// One result for a row-block solve whose P rank sessions live in this process:
// rank 0's objective row, basis and log (replicated on every rank) and every
// rank's eligible RHS rows, concatenated in global row order.
int merge_result(dlp_session* const* ss, int P, dlp_result* r) {
    for (int k = 0; k < P; ++k) CALL_TRY(flush_pending(ss[k]));   // the RHS must be current
    std::vector<std::pair<int64_t, int>> order;
    for (int k = 0; k < P; ++k) order.push_back({ss[k]->row_first, k});
    std::sort(order.begin(), order.end());
    std::vector<double> all;
    int64_t next = 0;
    for (const auto& o : order) {
        dlp_session* sk = ss[o.second];
        if (sk->row_first != next) {
            set_error("rank sessions do not tile the rows");
            return DLP_ERR_ARG;
        }
        std::vector<double> loc;
        CALL_TRY(local_rhs(sk, loc));
        all.insert(all.end(), loc.begin(), loc.end());
        next += sk->rows;
    }
    return extract_result(ss[order[0].second], r, &all);
}

// dlp_solve on n_gpus devices of this process: one RCCL communicator over
// devices [device, device + P) (ncclCommInitAll, so a failed start cannot
// leave a rank waiting), one host thread per device creating, running and
// reading its rank ("single process, one host thread per
// device").  The ranks advance in lockstep through the collectives.
// One attempt; *used_peer says whether the ranks ran on the peer exchange, *xwhy why the auto
// exchange did not (set-up).
int solve_in_process_once(const dlp_problem* prob, const dlp_options& o, int P, dlp_result** out,
                          bool* used_peer, std::string* xwhy_out) {
    *used_peer = false;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (o.device < 0 || o.device + P > ndev) {
        set_error("n_gpus = " + std::to_string(P) + " from device " + std::to_string(o.device) +
                  " exceeds the " + std::to_string(ndev) + " visible devices");
        return DLP_ERR_NODEVICE;
    }
    std::vector<int> devs(P);
    for (int r = 0; r < P; ++r) devs[r] = o.device + r;
    std::vector<ncclComm_t> comms(P, nullptr);
    NCCL_TRY(ncclCommInitAll(comms.data(), P, devs.data()));
    std::vector<dlp_session*> ss(P, nullptr);
    std::vector<int> rc(P, DLP_OK);
    std::vector<std::string> err(P);
    // the first rank to fail; the others' waits see it and abort their communicators
    // (wait_stream), so no thread stays blocked behind a collective that cannot complete
    std::atomic<int> failed{-1};
    auto on_ranks = [&](auto&& fn) {
        std::vector<std::thread> th;
        for (int r = 0; r < P; ++r)
            th.emplace_back([&, r] {
                rc[r] = fn(r);
                if (rc[r] < 0) {
                    err[r] = dlp_last_error();
                    int none = -1;
                    failed.compare_exchange_strong(none, r);
                }
            });
        for (auto& t : th) t.join();
        const int f = failed.load();
        if (f >= 0) {
            set_error("rank " + std::to_string(f) + ": " + err[f]);
            return rc[f];
        }
        return DLP_OK;
    };
    int res = on_ranks([&](int r) {
        dlp_options orr = o;
        orr.device = devs[r];
        orr.n_gpus = 0;
        auto* s = new (std::nothrow) dlp_session();
        if (!s) return DLP_ERR_OOM;
        int k = DLP_OK;
        try {
            k = session_init(prob, &orr, r, P, nullptr, s, comms[r]);
        } catch (const std::exception& e) {
            set_error(std::string("session_init: ") + e.what());
            k = DLP_ERR_OOM;
        }
        if (k != DLP_OK) {
            if (s->comm == comms[r]) s->comm = nullptr;   // freed below with the others
            free_session(s);
            return k;
        }
        comms[r] = nullptr;   // the session owns it now
        s->group_failed = &failed;
        ss[r] = s;
        return DLP_OK;
    });
    // owner-rooted peer exchange: every rank's block addressed directly (peer access between
    // the devices, no IPC inside one process); auto (DLP_XCHG_DEFAULT) falls back to RCCL when
    // the devices cannot connect; then each rank's auto lookahead follows its exchange
    std::string xwhy;
    if (res == DLP_OK && (o.exchange == DLP_XCHG_PEER || o.exchange == DLP_XCHG_DEFAULT)) {
        res = dlp_sessions_connect(ss.data(), P);
        // only "these devices cannot connect" falls back; a HIP error, OOM or a failure after
        // some ranks installed their peer tables is returned
        if (res == DLP_ERR_UNSUPPORTED && o.exchange == DLP_XCHG_DEFAULT) {
            xwhy = dlp_last_error();
            res = DLP_OK;
            for (dlp_session* s : ss) s->xmode = dlp_session::X_RCCL;
        }
    }
    if (res == DLP_OK) {
        *used_peer = ss[0]->xmode == dlp_session::X_PEER;
        *xwhy_out = xwhy;
    }
    if (res == DLP_OK)
        res = on_ranks([&](int r) {
            ss[r]->xreason = xwhy;
            HIP_TRY(hipSetDevice(ss[r]->device));
            return la_policy(ss[r]);
        });
    if (res == DLP_OK) {
        res = on_ranks([&](int r) {
            if (const char* e = std::getenv("DLP_TEST_FAIL_RANK"))   // tests: fail this rank's 2nd poll
                if (std::atoi(e) == r) ss[r]->fault_after_polls = 1;
            if (const char* e = std::getenv("DLP_TEST_FAIL_PEER_RANK"))   // the same, on the peer exchange only
                if (std::atoi(e) == r && ss[r]->xmode == dlp_session::X_PEER) ss[r]->fault_after_polls = 1;
            int64_t done = 0;
            return dlp_session_run(ss[r], o.max_pivots, &done);
        });
    }
    if (res == DLP_OK) {
        auto* r = new (std::nothrow) dlp_result();
        if (!r) {
            res = DLP_ERR_OOM;
        } else {
            res = merge_result(ss.data(), P, r);
            r->exchange = *used_peer ? DLP_XCHG_PEER : DLP_XCHG_RCCL;
            r->exchange_reason = xwhy;
            if (res == DLP_OK)
                *out = r;
            else
                delete r;
        }
    }
    // No rank's exchange block may be freed while another rank's kernels can still push into
    // it: after a failure every rank's device waits are ended (abort words), then every stream
    // drains, and only then is anything freed.
    if (res != DLP_OK)
        for (auto* s : ss)
            if (s && s->xabort) __atomic_store_n(s->xabort, 1u, __ATOMIC_SEQ_CST);
    for (auto* s : ss)
        if (s) {
            (void)hipSetDevice(s->device);
            if (s->stream) (void)hipStreamSynchronize(s->stream);
            if (s->pstream) (void)hipStreamSynchronize(s->pstream);
        }
    for (auto* s : ss)
        if (s) free_session(s);
    for (auto c : comms)
        if (c) (void)ncclCommDestroy(c);
    return res;
}

// dlp_solve(n_gpus = P).  With the auto exchange, a solve whose run fails on the peer exchange
// (a device wait that never completes, a fault in a cross-device store) is rerun from the start
// over RCCL on fresh sessions, as bench.py's measure_with_fallback does: the peer
// path's cross-device stores have run only on one-GPU boxes so far.  The result records the
// exchange that produced it and why (dlp_result_exchange).  Only an exchange failure is rerun
// (DLP_ERR_RCCL: a peer wait that timed out or was aborted, kStatusXFail, or the window limit);
// OOM, state, HIP and argument errors are deterministic or fatal and are returned unchanged
// (ADVICE r05).
int solve_in_process(const dlp_problem* prob, const dlp_options& o, int P, dlp_result** out) {
    bool peer = false;
    std::string why;
    const int rc = solve_in_process_once(prob, o, P, out, &peer, &why);
    if (rc != DLP_ERR_RCCL || !peer || o.exchange != DLP_XCHG_DEFAULT)
        return rc;
    const std::string first = dlp_last_error();
    dlp_options o2 = o;
    o2.exchange = DLP_XCHG_RCCL;
    const int rc2 = solve_in_process_once(prob, o2, P, out, &peer, &why);
    if (rc2 != DLP_OK) {
        set_error("peer exchange run failed (" + first + "), and the RCCL rerun: " + dlp_last_error());
        return rc2;
    }
    (*out)->exchange_reason = "peer exchange failed during the run: " + first;
    return DLP_OK;
}

// ---- peer exchange set-up ------------------------------------
// Every rank's ratio workgroups (its candidates when the ratio launch selects) from the same row
// partition every rank computes (dlp_rank_rows; a general LP with artificials carries its Phase II
// objective row on the last rank); returns the slots per sender, identical on every rank.
int xslots(const dlp_session* s, dlp::XPeers* x) {
    const bool carry = s->general && s->prob_dims.sf.nart > 0;
    int nslot = 1;
    for (int r = 0; r < s->nranks && r < dlp::kMaxRanks; ++r) {
        int64_t first = 0, count = 0;
        (void)dlp_rank_rows(s->m, r, s->nranks, &first, &count);
        if (carry && r == s->nranks - 1) count += 1;
        const int nrat = (int)((count + 1 + s->g.rthreads - 1) / s->g.rthreads);
        x->nrat[r] = nrat;
        nslot = std::max(nslot, nrat);
    }
    return nslot;
}

// This rank's exchange block (uncached device memory, zeroed: flags start below every seq)
// and the pinned abort word its waits read.
int ensure_xblock(dlp_session* s) {
    if (s->xblk) return DLP_OK;
    if (!s->exchange) {
        set_error("the peer exchange needs a row-block rank session (nranks > 1 or an RCCL id)");
        return DLP_ERR_STATE;
    }
    if (s->nranks > dlp::kMaxRanks) {
        set_error("the peer exchange supports at most 64 ranks");
        return DLP_ERR_UNSUPPORTED;
    }
    HIP_TRY(hipSetDevice(s->device));
    const size_t bytes = dlp::xblock_layout(s->nranks, s->ld, xslots(s, &s->xpeers_host), &s->xpeers_host);
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess) {
        s->xblk_uncached = true;
    } else {
        (void)hipGetLastError();
        HIP_TRY(hipMalloc(&p, bytes));   // system-scope accesses keep it coherent either way
    }
    s->xblk = (uint64_t*)p;
    HIP_TRY(hipMemset(s->xblk, 0, bytes));
    if (!s->xabort) {
        HIP_TRY(hipHostMalloc((void**)&s->xabort, 64, hipHostMallocCoherent | hipHostMallocMapped));
        *s->xabort = 0;
    }
    if (!s->xpeers) HIP_TRY(hipMalloc(&s->xpeers, sizeof(dlp::XPeers)));
    return DLP_OK;
}

// Device-side bound of one peer-exchange wait (100 MHz constant clock): the host's window limit
// plus 5 s, so that the host (which reports why) acts first; 0 = wait on the abort word only.
uint64_t xwait_ticks(double stall_limit_s) {
    return stall_limit_s > 0 ? (uint64_t)((stall_limit_s + 5.0) * 1e8) : 0;
}

// Install the peer table (bases[r] = rank r's block as this device addresses it).  devs[r]: the
// device ordinal (in this process) of rank r, -1 where unknown (dlp_session_connect_ipc's bare
// handles): ranks on this session's device share its CUs (coloc_n / coloc_i, chain_cus_policy).
int install_peers(dlp_session* s, const std::vector<uint64_t*>& bases, const std::vector<int>& devs) {
    s->coloc_n = 0;
    s->coloc_i = 0;
    for (int r = 0; r < s->nranks; ++r)
        if (r == s->rank || (r < (int)devs.size() && devs[r] == s->device)) {
            ++s->coloc_n;
            if (r < s->rank) ++s->coloc_i;
        }
    dlp::XPeers& x = s->xpeers_host;
    (void)dlp::xblock_layout(s->nranks, s->ld, xslots(s, &x), &x);
    for (int r = 0; r < dlp::kMaxRanks; ++r) x.base[r] = r < (int)bases.size() ? bases[r] : nullptr;
    x.me = s->rank;
    x.wait_ticks = xwait_ticks(s->stall_limit_s);
    void* dabort = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dabort, s->xabort, 0));
    x.abort_word = (const uint32_t*)dabort;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipMemcpy(s->xpeers, &x, sizeof(x), hipMemcpyHostToDevice));
    s->xmode = dlp_session::X_PEER;
    if (s->gexec) { (void)hipGraphExecDestroy(s->gexec); s->gexec = nullptr; }
    if (s->graph) { (void)hipGraphDestroy(s->graph); s->graph = nullptr; }
    return DLP_OK;
}

int connect_ipc(dlp_session* s, const uint8_t* handles) {
    CALL_TRY(ensure_xblock(s));
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    std::vector<uint64_t*> bases(s->nranks, nullptr);
    for (int r = 0; r < s->nranks; ++r) {
        if (r == s->rank) {
            bases[r] = s->xblk;
            continue;
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)r * sizeof(hipIpcMemHandle_t), sizeof(h));
        void* p = nullptr;
        HIP_TRY(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        s->ipc_open.push_back(p);
        bases[r] = (uint64_t*)p;
    }
    CALL_TRY(install_peers(s, bases, {}));
    return la_policy(s);
}

// ---- choosing the exchange over the communicator --------------------
// Every rank's record, all-gathered: its exchange block's IPC handle, whether it could make
// one, the PCI bus id of its device (mapped to this process's ordinals, so peer access is
// checked for the devices really involved) and the reason when not.
struct XRec {
    uint8_t handle[64];
    int32_t ok;
    int32_t pad;
    char bus[32];
    char why[152];
};
static_assert(sizeof(XRec) == 256, "XRec is 256 bytes");

// All-gather `bytes` per rank over the session's communicator (a blocking collective with
// the window wait's failure containment).
int comm_allgather(dlp_session* s, const void* mine, void* all, size_t bytes) {
    uint8_t* dbuf = nullptr;
    HIP_TRY(hipMalloc(&dbuf, bytes * (s->nranks + 1)));
    int rc = DLP_OK;
    if (hipMemcpy(dbuf + bytes * s->nranks, mine, bytes, hipMemcpyHostToDevice) != hipSuccess) {
        set_error("hipMemcpy (exchange set-up)");
        rc = DLP_ERR_HIP;
    }
    if (rc == DLP_OK) {
        const ncclResult_t nr = ncclAllGather(dbuf + bytes * s->nranks, dbuf, bytes, ncclUint8, s->comm, s->stream);
        if (nr != ncclSuccess) {
            set_error(std::string("ncclAllGather (exchange set-up): ") + ncclGetErrorString(nr));
            rc = DLP_ERR_RCCL;
        }
    }
    if (rc == DLP_OK) rc = wait_stream(s);
    if (rc == DLP_OK && hipMemcpy(all, dbuf, bytes * s->nranks, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("hipMemcpy (exchange set-up)");
        rc = DLP_ERR_HIP;
    }
    (void)hipFree(dbuf);
    return rc;
}

// This rank's half of a peer connect from every rank's record: each other rank's device (by its
// PCI bus id, mapped to this process's ordinals), peer access to it, its block opened.  On a
// failure out->ok = 0 with the reason in out->why and nothing left open.
void open_peer_blocks(dlp_session* s, XRec* all, XRec* out, std::vector<void*>* opened,
                      std::vector<uint64_t*>* bases, std::vector<int>* devs) {
    bases->assign(s->nranks, nullptr);
    devs->assign(s->nranks, -1);
    (*devs)[s->rank] = s->device;
    for (int r = 0; r < s->nranks && out->ok; ++r) {
        if (r == s->rank) {
            (*bases)[r] = s->xblk;
            continue;
        }
        int dev = -1, can = 0;
        all[r].bus[sizeof(all[r].bus) - 1] = 0;
        if (hipDeviceGetByPCIBusId(&dev, all[r].bus) != hipSuccess || dev < 0) {
            (void)hipGetLastError();
            std::snprintf(out->why, sizeof(out->why), "rank %d's device %s is not visible to this process",
                          r, all[r].bus);
            out->ok = 0;
            break;
        }
        (*devs)[r] = dev;
        if (dev != s->device && (hipDeviceCanAccessPeer(&can, s->device, dev) != hipSuccess || !can)) {
            (void)hipGetLastError();
            std::snprintf(out->why, sizeof(out->why), "device %d cannot access device %d (rank %d)", s->device,
                          dev, r);
            out->ok = 0;
            break;
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, all[r].handle, sizeof(h));
        void* p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            std::snprintf(out->why, sizeof(out->why), "hipIpcOpenMemHandle of rank %d's block: %s", r,
                          hipGetErrorString(e));
            out->ok = 0;
            break;
        }
        opened->push_back(p);
        (*bases)[r] = (uint64_t*)p;
    }
    if (!out->ok) {
        for (void* p : *opened) (void)hipIpcCloseMemHandle(p);
        opened->clear();
    }
}

// This rank's record: its exchange block's IPC handle and its device's PCI bus id (ok = 0 with the
// reason when either cannot be had).  DLP_TEST_PEER_FAIL=<rank> (tests only) makes that rank fail.
void make_xrec(dlp_session* s, XRec* me) {
    *me = XRec{};
    me->ok = 1;
    auto fail = [&](const std::string& w) {
        if (!me->ok) return;
        me->ok = 0;
        std::snprintf(me->why, sizeof(me->why), "%s", w.c_str());
    };
    if (const char* e = std::getenv("DLP_TEST_PEER_FAIL"))
        if (std::atoi(e) == s->rank) fail("injected (DLP_TEST_PEER_FAIL)");
    if (me->ok && ensure_xblock(s) != DLP_OK) fail(std::string("exchange block: ") + dlp_last_error());
    if (me->ok) {
        hipIpcMemHandle_t h;
        if (hipIpcGetMemHandle(&h, s->xblk) != hipSuccess) {
            (void)hipGetLastError();
            fail("hipIpcGetMemHandle of the exchange block failed");
        } else {
            std::memcpy(me->handle, &h, sizeof(h));
        }
    }
    if (hipDeviceGetPCIBusId(me->bus, (int)sizeof(me->bus), s->device) != hipSuccess) {
        (void)hipGetLastError();
        fail("hipDeviceGetPCIBusId failed");
    }
}

// Owner-rooted peer exchange over the communicator, agreed by every rank: each rank makes its
// block and IPC handle, the records are all-gathered, each rank checks peer access to every
// other rank's device and opens their blocks, and a second all-gather agrees on the outcome.
// DLP_ERR_UNSUPPORTED (on every rank alike, *why set, nothing installed) when any rank could
// not; other errors are failures of the communicator itself.  DLP_TEST_PEER_FAIL=<rank>
// (tests only) makes that rank report a failure.
int peer_connect_collective(dlp_session* s, std::string* why) {
    XRec me;
    make_xrec(s, &me);
    std::vector<XRec> all(s->nranks);
    CALL_TRY(comm_allgather(s, &me, all.data(), sizeof(XRec)));
    for (int r = 0; r < s->nranks; ++r)
        if (!all[r].ok) {
            *why = "rank " + std::to_string(r) + ": " + std::string(all[r].why, strnlen(all[r].why, sizeof(all[r].why)));
            return DLP_ERR_UNSUPPORTED;
        }
    // peer access to every other rank's device, then its block
    XRec me2{};
    me2.ok = 1;
    std::vector<void*> opened;
    std::vector<uint64_t*> bases;
    std::vector<int> devs;
    open_peer_blocks(s, all.data(), &me2, &opened, &bases, &devs);
    std::vector<XRec> all2(s->nranks);
    const int rc = comm_allgather(s, &me2, all2.data(), sizeof(XRec));
    int bad = -1;
    for (int r = 0; r < s->nranks && rc == DLP_OK && bad < 0; ++r)
        if (!all2[r].ok) bad = r;
    if (rc != DLP_OK || bad >= 0) {
        for (void* p : opened) (void)hipIpcCloseMemHandle(p);   // (nothing is open when me2.ok == 0)
        if (rc != DLP_OK) return rc;
        *why = "rank " + std::to_string(bad) + ": " + std::string(all2[bad].why, strnlen(all2[bad].why, sizeof(all2[bad].why)));
        return DLP_ERR_UNSUPPORTED;
    }
    s->ipc_open.insert(s->ipc_open.end(), opened.begin(), opened.end());
    return install_peers(s, bases, devs);
}

// A communicator session's exchange: `mode` DLP_XCHG_RCCL, DLP_XCHG_PEER (an error when the
// ranks cannot connect) or DLP_XCHG_DEFAULT (peer where every rank pair connects, else RCCL
// with the reason kept for dlp_session_exchange_reason); then the auto lookahead follows.
int settle_exchange(dlp_session* s, int mode) {
    if (mode == DLP_XCHG_PEER || mode == DLP_XCHG_DEFAULT) {
        std::string why;
        const int rc = peer_connect_collective(s, &why);
        if (rc == DLP_ERR_UNSUPPORTED) {
            if (mode == DLP_XCHG_PEER) {
                set_error("peer exchange unavailable: " + why);
                return rc;
            }
            s->xreason = why;
            s->xmode = dlp_session::X_RCCL;
        } else if (rc != DLP_OK) {
            return rc;
        }
    } else {
        s->xmode = dlp_session::X_RCCL;
    }
    return la_policy(s);
}

// Phase-interleaved multi-rank run (dlp_sessions_run): every rank's phase p before any
// rank's phase p + 1, for every pivot, from one host thread.
int sessions_phase(dlp_session* const* ss, int P, int phase, int64_t slot, bool last, int kind,
                   int64_t row) {
    for (int r = 0; r < P; ++r) {
        HIP_TRY(hipSetDevice(ss[r]->device));
        if (kind == 0)
            CALL_TRY(pivot_phase(ss[r], phase, slot, last));
        else if (kind == 1)
            CALL_TRY(forced_phase(ss[r], phase, row));
        else
            CALL_TRY(carry_phase(ss[r], phase));
    }
    return DLP_OK;
}

}  // namespace

// =========================================================================
extern "C" {

void dlp_options_default(dlp_options* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->device = 0;
    o->pricing = DLP_PRICING_DANTZIG_BLAND;
    o->tol_dj = 1e-9;
    o->tol_piv = 1e-9;
    o->max_pivots = 1000000;
    o->log_pivots = 1;
    o->check_interval = 64;
    o->timing = 0;
    o->nontemporal = -1;   // auto
    o->rows_per_block = 0;
    o->use_graph = 1;
    o->update_variant = -1;   // auto
    o->ld_align = 0;          // auto
    o->tol_feas = 1e-9;
    o->defer = 0;   // auto
    o->lookahead = -1;   // auto
}

const char* dlp_status_string(int st) {
    switch (st) {
        case DLP_OK: return "optimal";
        case DLP_INFEASIBLE: return "infeasible";
        case DLP_UNBOUNDED: return "unbounded";
        case DLP_PIVOT_LIMIT: return "pivot limit";
        case DLP_RUNNING: return "running";
        case DLP_ERR_ARG: return "invalid argument";
        case DLP_ERR_OOM: return "out of device memory";
        case DLP_ERR_HIP: return "HIP error";
        case DLP_ERR_RCCL: return "exchange (RCCL / peer) error";
        case DLP_ERR_NODEVICE: return "no HIP device";
        case DLP_ERR_STATE: return "invalid state";
        case DLP_ERR_UNSUPPORTED: return "unsupported";
        default: return "unknown status";
    }
}

const char* dlp_last_error(void) { return dlp::g_err.c_str(); }

int dlp_device_count(int* count) {
    if (!count) return DLP_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return DLP_OK;
}

int dlp_rank_rows(int64_t m, int rank, int nranks, int64_t* first, int64_t* count) {
    if (m < 0 || nranks <= 0 || rank < 0 || rank >= nranks || !first || !count) {
        set_error("dlp_rank_rows: bad arguments");
        return DLP_ERR_ARG;
    }
    const int64_t a = (m * rank) / nranks, b = (m * (rank + 1)) / nranks;
    *first = a;
    *count = b - a;
    return DLP_OK;
}

int dlp_candidate_select(const dlp_candidate* cands, int n, int* winner) {
    if (!cands || n <= 0 || !winner) return DLP_ERR_ARG;
    int w = -1;
    dlp::Cand best{};
    best.valid = 0;
    for (int r = 0; r < n; ++r) {
        dlp::Cand c;
        std::memcpy(&c, &cands[r], sizeof(c));
        if (dlp::cand_better(c, best)) { best = c; w = r; }
    }
    *winner = w;
    return DLP_OK;
}

int64_t dlp_tableau_ld(int64_t m, int64_t n) { return round16(n + m + 1); }

int dlp_update_variants(void) { return dlp::update_variants(); }

int dlp_problem_create_dense(int64_t m, int64_t n, const double* A, const double* b,
                             const double* c, dlp_problem** out) {
    if (!out || m <= 0 || n <= 0 || !A || !b || !c || n + m + 1 > INT32_MAX) {
        set_error("dlp_problem_create_dense: bad arguments");
        return DLP_ERR_ARG;
    }
    for (int64_t i = 0; i < m; ++i)
        if (!(b[i] >= 0.0)) {
            set_error("b must be >= 0 (slack starting basis; Phase I is not implemented)");
            return DLP_ERR_UNSUPPORTED;
        }
    auto* p = new (std::nothrow) dlp_problem();
    if (!p) return DLP_ERR_OOM;
    p->kind = dlp::PROB_DENSE;
    p->m = m;
    p->n = n;
    p->A.assign(A, A + m * n);
    p->b.assign(b, b + m);
    p->c.assign(c, c + n);
    *out = p;
    return DLP_OK;
}

int dlp_problem_create_random(int kind, int64_t m, int64_t n, uint64_t seed, dlp_problem** out) {
    if (!out || m <= 0 || n <= 0 || (kind != DLP_GEN_DENSE && kind != DLP_GEN_DEGENERATE) ||
        n + m + 1 > INT32_MAX) {
        set_error("dlp_problem_create_random: bad arguments");
        return DLP_ERR_ARG;
    }
    auto* p = new (std::nothrow) dlp_problem();
    if (!p) return DLP_ERR_OOM;
    p->kind = dlp::PROB_RANDOM;
    p->m = m;
    p->n = n;
    p->gen_kind = kind;
    p->seed = seed;
    *out = p;
    return DLP_OK;
}

int dlp_problem_create_adalloc(int num_advertisers, int num_impressions, int num_slots,
                               double bid_sparsity, double scaling_factor, dlp_problem** out) {
    if (!out || num_slots != 1) {
        set_error("dlp_problem_create_adalloc: num_slots must be 1 (as every reference scenario)");
        return DLP_ERR_ARG;
    }
    auto* p = new (std::nothrow) dlp_problem();
    if (!p) return DLP_ERR_OOM;
    int rc = dlp::build_adalloc(num_advertisers, num_impressions, bid_sparsity, scaling_factor,
                                &p->ad);
    if (rc != DLP_OK) {
        delete p;
        set_error("dlp_problem_create_adalloc: bad arguments");
        return rc;
    }
    p->kind = dlp::PROB_ADALLOC;
    p->m = (int64_t)num_advertisers + num_impressions;
    p->n = (int64_t)p->ad.adv.size();
    *out = p;
    return DLP_OK;
}

int dlp_problem_create_general(int64_t m, int64_t n, const double* A, const double* row_lo,
                               const double* row_hi, const double* col_lo, const double* col_hi,
                               const double* c, double c0, int sense, dlp_problem** out) {
    if (!out || m < 0 || n <= 0 || (m > 0 && (!A || !row_lo || !row_hi)) || !col_lo || !col_hi ||
        !c || (sense != DLP_MINIMIZE && sense != DLP_MAXIMIZE) || std::isnan(c0)) {
        set_error("dlp_problem_create_general: bad arguments");
        return DLP_ERR_ARG;
    }
    for (int64_t j = 0; j < n; ++j)
        if (std::isnan(c[j]) || std::isinf(c[j])) {
            set_error("dlp_problem_create_general: c must be finite");
            return DLP_ERR_ARG;
        }
    auto* p = new (std::nothrow) dlp_problem();
    if (!p) return DLP_ERR_OOM;
    try {
        dlp::General& g = p->gen;
        g.m = m;
        g.n = n;
        if (m > 0) {
            g.A.assign(A, A + m * n);
            g.row_lo.assign(row_lo, row_lo + m);
            g.row_hi.assign(row_hi, row_hi + m);
        }
        g.col_lo.assign(col_lo, col_lo + n);
        g.col_hi.assign(col_hi, col_hi + n);
        g.c.assign(c, c + n);
        g.c0 = c0;
        g.sense = sense;
        const int rc = dlp::build_stdform(g, &p->sf);
        if (rc != DLP_OK) {
            delete p;
            return rc;
        }
    } catch (const std::bad_alloc&) {
        delete p;
        set_error("dlp_problem_create_general: out of host memory");
        return DLP_ERR_OOM;
    }
    p->kind = dlp::PROB_GENERAL;
    p->m = m;
    p->n = n;
    *out = p;
    return DLP_OK;
}

int dlp_problem_create_mps(const char* path, dlp_problem** out) {
    if (!path || !out) {
        set_error("dlp_problem_create_mps: bad arguments");
        return DLP_ERR_ARG;
    }
    dlp::General g;
    try {
        CALL_TRY(dlp::parse_mps(path, &g));
    } catch (const std::bad_alloc&) {
        set_error("dlp_problem_create_mps: out of host memory");
        return DLP_ERR_OOM;
    }
    return dlp_problem_create_general(g.m, g.n, g.A.data(), g.row_lo.data(), g.row_hi.data(),
                                      g.col_lo.data(), g.col_hi.data(), g.c.data(), g.c0, g.sense,
                                      out);
}

int dlp_problem_get_general(const dlp_problem* p, double* A, double* row_lo, double* row_hi,
                            double* col_lo, double* col_hi, double* c, double* c0, int* sense) {
    if (!p) return DLP_ERR_ARG;
    if (p->kind == dlp::PROB_RANDOM) {
        set_error("random problems are generated on the device; use dlp_session_tableau");
        return DLP_ERR_UNSUPPORTED;
    }
    const int64_t m = p->m, n = p->n;
    if (p->kind == dlp::PROB_GENERAL) {
        const dlp::General& g = p->gen;
        if (A && m > 0) std::memcpy(A, g.A.data(), sizeof(double) * m * n);
        if (row_lo && m > 0) std::memcpy(row_lo, g.row_lo.data(), sizeof(double) * m);
        if (row_hi && m > 0) std::memcpy(row_hi, g.row_hi.data(), sizeof(double) * m);
        if (col_lo) std::memcpy(col_lo, g.col_lo.data(), sizeof(double) * n);
        if (col_hi) std::memcpy(col_hi, g.col_hi.data(), sizeof(double) * n);
        if (c) std::memcpy(c, g.c.data(), sizeof(double) * n);
        if (c0) *c0 = g.c0;
        if (sense) *sense = g.sense;
        return DLP_OK;
    }
    // dense / ad-allocation: max c^T x, A x <= b, x >= 0
    std::vector<double> b(m);
    CALL_TRY(dlp_problem_get_dense(p, A, b.data(), c));
    for (int64_t i = 0; i < m; ++i) {
        if (row_lo) row_lo[i] = -HUGE_VAL;
        if (row_hi) row_hi[i] = b[i];
    }
    for (int64_t j = 0; j < n; ++j) {
        if (col_lo) col_lo[j] = 0.0;
        if (col_hi) col_hi[j] = HUGE_VAL;
    }
    if (c0) *c0 = 0.0;
    if (sense) *sense = DLP_MAXIMIZE;
    return DLP_OK;
}

int dlp_problem_std_dims(const dlp_problem* p, int64_t* m_std, int64_t* ncols, int64_t* nprice,
                         int64_t* nart) {
    if (!p) return DLP_ERR_ARG;
    if (p->kind == dlp::PROB_GENERAL) {
        if (m_std) *m_std = p->sf.m;
        if (ncols) *ncols = p->sf.ncols();
        if (nprice) *nprice = p->sf.nprice();
        if (nart) *nart = p->sf.nart;
    } else {
        if (m_std) *m_std = p->m;
        if (ncols) *ncols = p->m + p->n;
        if (nprice) *nprice = p->m + p->n;
        if (nart) *nart = 0;
    }
    return DLP_OK;
}

int dlp_problem_dims(const dlp_problem* p, int64_t* m, int64_t* n) {
    if (!p) return DLP_ERR_ARG;
    if (m) *m = p->m;
    if (n) *n = p->n;
    return DLP_OK;
}

int dlp_problem_get_dense(const dlp_problem* p, double* A, double* b, double* c) {
    if (!p) return DLP_ERR_ARG;
    if (p->kind == dlp::PROB_GENERAL) {
        set_error("general LPs have row / column bounds: use dlp_problem_get_general");
        return DLP_ERR_UNSUPPORTED;
    }
    if (p->kind == dlp::PROB_RANDOM) {
        set_error("random problems are generated on the device; use dlp_session_tableau");
        return DLP_ERR_UNSUPPORTED;
    }
    std::vector<double> T;
    const int64_t ld = round16(p->n + p->m + 1);
    host_tableau(p, 0, p->m, ld, T);
    for (int64_t i = 0; i < p->m; ++i) {
        if (A) std::memcpy(A + i * p->n, T.data() + i * ld, sizeof(double) * p->n);
        if (b) b[i] = T[i * ld + p->n + p->m];
    }
    if (c)
        for (int64_t j = 0; j < p->n; ++j) c[j] = -T[p->m * ld + j];
    return DLP_OK;
}

int dlp_problem_adalloc_bids(const dlp_problem* p, int64_t* nnz, int32_t* adv, int32_t* imp,
                             double* bid) {
    if (!p || !nnz || p->kind != dlp::PROB_ADALLOC) return DLP_ERR_ARG;
    *nnz = (int64_t)p->ad.adv.size();
    if (adv) std::memcpy(adv, p->ad.adv.data(), sizeof(int32_t) * p->ad.adv.size());
    if (imp) std::memcpy(imp, p->ad.imp.data(), sizeof(int32_t) * p->ad.imp.size());
    if (bid) std::memcpy(bid, p->ad.bid.data(), sizeof(double) * p->ad.bid.size());
    return DLP_OK;
}

void dlp_problem_free(dlp_problem* p) { delete p; }

int dlp_session_create_rank(const dlp_problem* prob, const dlp_options* opt, int rank,
                            int nranks, const void* uid, dlp_session** out) {
    if (!prob || !out || nranks <= 0 || rank < 0 || rank >= nranks) {
        set_error("dlp_session_create_rank: bad arguments");
        return DLP_ERR_ARG;
    }
    CALL_TRY(validate_options(opt));
    auto* s = new (std::nothrow) dlp_session();
    if (!s) return DLP_ERR_OOM;
    int rc = DLP_OK;
    try {
        rc = session_init(prob, opt, rank, nranks, uid, s);
    } catch (const std::exception& e) {
        set_error(std::string("session_init: ") + e.what());
        rc = DLP_ERR_OOM;
    }
    if (rc == DLP_OK && uid) rc = settle_exchange(s, opt->exchange);   // collective over the new communicator
    if (rc != DLP_OK) {
        free_session(s);
        return rc;
    }
    *out = s;
    return DLP_OK;
}

int dlp_session_create(const dlp_problem* prob, const dlp_options* opt, dlp_session** out) {
    return dlp_session_create_rank(prob, opt, 0, 1, nullptr, out);
}

int dlp_comm_unique_id(void* out128) {
    if (!out128) return DLP_ERR_ARG;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(out128, &id, sizeof(id));
    return DLP_OK;
}

int dlp_session_run(dlp_session* s, int64_t max_pivots, int64_t* pivots_done) {
    if (!s || max_pivots < 0) return DLP_ERR_ARG;
    if (s->exchange && s->xmode == dlp_session::X_HOST) {
        set_error("session has no communicator: drive it with dlp_session_step_*, or connect the "
                  "ranks (dlp_sessions_connect / dlp_session_connect_ipc)");
        return DLP_ERR_STATE;
    }
    HIP_TRY(hipSetDevice(s->device));
    const int64_t start = s->npivots;
    int64_t budget = std::min<int64_t>(max_pivots, s->opt.max_pivots - s->launched);
    const bool graph = s->opt.use_graph && !s->exchange && s->ev_per_pivot == 0 && !s->la;
    while (s->status == DLP_RUNNING && budget > 0) {
        if (s->drive_next < s->drive.size() || s->carry_pending) {   // Phase I -> II switch
            while (s->drive_next < s->drive.size() && budget > 0) {
                CALL_TRY(enqueue_forced(s, s->drive[s->drive_next++]));
                s->launched += 1;
                budget -= 1;
            }
            if (s->drive_next == s->drive.size() && s->carry_pending) {
                CALL_TRY(enqueue_carry(s));
                CALL_TRY(finish_phase1(s));
            } else {
                CALL_TRY(poll(s));
            }
            continue;
        }
        // a small-LP window is one launch that stops by itself at the optimum: poll less
        const int64_t chunk = std::min<int64_t>(
            budget, s->cluster ? std::max<int64_t>(s->opt.check_interval, 1024) : s->opt.check_interval);
        if (s->cluster) {
            CALL_TRY(enqueue_cluster(s, chunk));
        } else if (graph && chunk == s->opt.check_interval) {
            CALL_TRY(run_window_graph(s, chunk));
        } else {
            for (int64_t k = 0; k < chunk; ++k) CALL_TRY(enqueue_pivot(s, k, k == chunk - 1));
            s->ev_pending = s->ev_per_pivot ? chunk : 0;
        }
        s->launched += chunk;
        budget -= chunk;
        CALL_TRY(poll(s));
    }
    if (pivots_done) *pivots_done = s->npivots - start;
    if (s->status != DLP_RUNNING) return s->status;
    if (s->launched >= s->opt.max_pivots) return DLP_PIVOT_LIMIT;
    return DLP_RUNNING;
}

// Caller-driven steps.  A general LP's Phase I -> II switch is carried by the
// same three-step exchange: forced drive-out pivots, then one carry step
// (its candidate is an empty slot, its "pivot row" the carried objective row).
// Deferred sessions under the step API: the same kernels as enqueue_pivot_defer,
// with the two exchanges done by the caller between the calls.
int step_candidate_defer(dlp_session* s) {
    const dlp_options& o = s->opt;
    s->step_kind = dlp_session::STEP_PIVOT;
    HIP_TRY(dlp::launch_ratio_defer(s->g, s->d, s->basis, s->pp, s->st, s->partials,
                                    s->ratio_blocks_max, s->cand_send, s->exchange ? 2 : 1, o.tol_dj,
                                    o.tol_piv, o.pricing, s->log, s->log_cap, s->stream));
    return DLP_OK;
}

int step_select_defer(dlp_session* s) {
    const dlp_options& o = s->opt;
    if (s->exchange)
        HIP_TRY(dlp::launch_select(s->g, s->cand_recv, s->nranks, s->basis, s->st, o.pricing,
                                   s->log, s->log_cap, s->stream, false, true));
    HIP_TRY(dlp::launch_prow_defer(s->g, s->d, s->st, s->prow_send, s->pp, o.tol_dj, s->log,
                                   s->log_cap, s->exchange ? 2 : 1, s->stream));
    return DLP_OK;
}

int step_update_defer(dlp_session* s) {
    const dlp_options& o = s->opt;
    if (s->exchange)
        HIP_TRY(dlp::launch_commit_defer(s->g, s->d, s->st, s->prow_recv, s->pp, o.tol_dj, s->log,
                                         s->log_cap, s->stream));
    s->since_flush += 1;
    s->launched += 1;
    if (s->since_flush >= s->d.K) CALL_TRY(enqueue_flush(s));
    return DLP_OK;
}

// Before anything reads the tableau: apply the pending steps of a deferred block
// (the step API leaves a partial block pending when the caller stops).
int flush_pending(dlp_session* s) {
    if (s->la) {
        if (s->since_flush > 0) CALL_TRY(la_block_end(s, true, nullptr));
        return la_drain(s);
    }
    if (s->d.K > 1 && s->since_flush > 0) CALL_TRY(enqueue_flush(s));
    return DLP_OK;
}

int dlp_session_step_candidate(dlp_session* s) {
    if (!s) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    CALL_TRY(la_disable(s));   // the step API drives single-buffer blocks
    s->step_void = false;
    // the Phase I -> II switch (drive-out pivots, carried row) runs on the eager
    // kernels in every session, as in dlp_session_run: apply a pending deferred
    // block first, since a forced pivot reads its row from the tableau
    if (s->drive_next < s->drive.size() || s->carry_pending) CALL_TRY(flush_pending(s));
    if (s->drive_next < s->drive.size()) {
        s->step_kind = dlp_session::STEP_FORCED;
        return enqueue_forced_candidate(s, s->drive[s->drive_next++]);
    }
    if (s->carry_pending) {
        s->step_kind = dlp_session::STEP_CARRY;
        HIP_TRY(hipMemsetAsync(s->cand_send, 0, sizeof(dlp::Cand), s->stream));
        return DLP_OK;
    }
    if (s->d.K > 1) return step_candidate_defer(s);
    s->step_kind = dlp_session::STEP_PIVOT;
    return enqueue_candidate(s);
}

int dlp_session_step_select(dlp_session* s) {
    if (!s) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    if (s->step_void) return DLP_OK;
    switch (s->step_kind) {
        case dlp_session::STEP_FORCED: return enqueue_forced_select(s);
        case dlp_session::STEP_CARRY: return enqueue_carry_out(s);
        default: break;
    }
    if (s->d.K > 1) return step_select_defer(s);
    CALL_TRY(enqueue_select(s));
    return enqueue_prow(s);
}

int dlp_session_step_update(dlp_session* s) {
    if (!s) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    if (s->step_void) return DLP_OK;
    if (s->step_kind == dlp_session::STEP_CARRY) {
        CALL_TRY(enqueue_carry_in(s));
        return finish_phase1(s);
    }
    if (s->d.K > 1 && s->step_kind == dlp_session::STEP_PIVOT) return step_update_defer(s);
    CALL_TRY(enqueue_update(s));
    s->launched += 1;
    return DLP_OK;
}

int dlp_session_buffer(dlp_session* s, int which, void** dev_ptr, size_t* bytes) {
    if (!s || !dev_ptr || !bytes) return DLP_ERR_ARG;
    switch (which) {
        case DLP_BUF_CAND_SEND: *dev_ptr = s->cand_send; *bytes = sizeof(dlp::Cand); break;
        case DLP_BUF_CAND_RECV: *dev_ptr = s->cand_recv; *bytes = sizeof(dlp::Cand) * s->nranks; break;
        case DLP_BUF_PROW_SEND: *dev_ptr = s->prow_send; *bytes = sizeof(int64_t) * s->ld; break;
        case DLP_BUF_PROW_RECV: *dev_ptr = s->prow_recv; *bytes = sizeof(int64_t) * s->ld; break;
        default: return DLP_ERR_ARG;
    }
    return DLP_OK;
}

int dlp_session_read_buffer(dlp_session* s, int which, void* host, size_t bytes) {
    void* dev = nullptr;
    size_t cap = 0;
    CALL_TRY(dlp_session_buffer(s, which, &dev, &cap));
    if (!host || bytes > cap) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return DLP_OK;
}

int dlp_session_write_buffer(dlp_session* s, int which, const void* host, size_t bytes) {
    void* dev = nullptr;
    size_t cap = 0;
    CALL_TRY(dlp_session_buffer(s, which, &dev, &cap));
    if (!host || bytes > cap) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return DLP_OK;
}

int dlp_session_sync(dlp_session* s) {
    if (!s) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    return poll(s);
}

int dlp_session_status(dlp_session* s, int* status, int64_t* npivots) {
    if (!s) return DLP_ERR_ARG;
    CALL_TRY(dlp_session_sync(s));
    if (status) *status = s->status;
    if (npivots) *npivots = s->npivots;
    return DLP_OK;
}

int dlp_session_timings(dlp_session* s, double* ms_out, int64_t* nsamples) {
    if (!s || !ms_out) return DLP_ERR_ARG;
    for (int ph = 0; ph < DLP_NUM_PHASES; ++ph) ms_out[ph] = s->timings[ph];
    if (nsamples) *nsamples = s->nsamples;
    return DLP_OK;
}

int dlp_session_set_tuning(dlp_session* s, int update_variant, int rows_per_block,
                           int nontemporal) {
    if (!s || update_variant >= dlp::update_variants() || rows_per_block < 0) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (update_variant < 0) update_variant = s->streaming ? 22 : 26;   // auto, as session_init
    if (nontemporal < 0) nontemporal = s->streaming ? 1 : 0;
    if (s->d.K > 1) {   // deferred: rows_per_block sets the pass band; pricing tiles stay 512
        if (dlp::update_tile(update_variant) != dlp::kDeferTile) {
            set_error("a deferred session (defer > 1) needs a 512-column update variant");
            return DLP_ERR_ARG;
        }
        s->defer_rb_req = rows_per_block > 0 ? rows_per_block : 0;
        s->defer_rb = s->defer_rb_req > 0 ? fit_defer_rb(s, s->defer_rb_req) : auto_defer_rb(s);
    }
    s->opt.update_variant = update_variant;
    s->opt.nontemporal = nontemporal;
    const int tile = dlp::update_tile(update_variant);
    s->g.ntiles = (int)((s->width + tile - 1) / tile);
    s->g.rows_per_block = rows_per_block > 0 ? rows_per_block : auto_rows_per_block(s);
    s->g.rows_per_block = std::min(s->g.rows_per_block, dlp::kMaxBandLdsHost);
    if (s->gexec) { (void)hipGraphExecDestroy(s->gexec); s->gexec = nullptr; }
    if (s->graph) { (void)hipGraphDestroy(s->graph); s->graph = nullptr; }
    // pricing partials depend only on the current objective row: rebuild at the new tiling
    HIP_TRY(dlp::launch_price_init(s->g, s->pp, s->opt.tol_dj, update_variant, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return DLP_OK;
}

int dlp_session_get_tuning(dlp_session* s, int* update_variant, int* rows_per_block,
                           int* nontemporal) {
    if (!s) return DLP_ERR_ARG;
    if (update_variant) *update_variant = s->opt.update_variant;
    if (rows_per_block) *rows_per_block = s->d.K > 1 ? s->defer_rb : s->g.rows_per_block;
    if (nontemporal) *nontemporal = s->opt.nontemporal;
    return DLP_OK;
}

int dlp_session_chain_cus(dlp_session* s, int* cus) {
    if (!s || !cus) return DLP_ERR_ARG;
    *cus = s->la ? s->chain_cus : 0;
    return DLP_OK;
}

int dlp_session_small_lp(dlp_session* s, int* small_lp) {
    if (!s || !small_lp) return DLP_ERR_ARG;
    *small_lp = s->cluster ? 1 : 0;
    return DLP_OK;
}

int dlp_session_set_defer_tuning(dlp_session* s, int occupancy, int form) {
    if (!s || occupancy < 0 || occupancy > 32 || form < -1 || form > 23) return DLP_ERR_ARG;
    if ((form == 0 || form == 4 || form == 6 || form == 7 || form == 10 || form == 11 || form == 14 ||
         form == 15 || form == 16 || form == 17 || form == 20) &&
        s->d.K > 32) {
        set_error("the 2-doubles-per-lane pass holds at most 32 steps");
        return DLP_ERR_ARG;
    }
    s->defer_occ = occupancy;
    if (form >= 0) s->form_auto = false;
    if (form >= 0 && s->la && !dlp::lookahead_form(form)) CALL_TRY(la_disable(s));
    if (form >= 0) {
        s->d.form = form;
        s->dslot[0].form = s->dslot[1].form = form;
        // the band follows the form (auto), or is clamped to what the form's LDS holds
        if (s->d.K > 1)
            s->defer_rb = s->defer_rb_req > 0 ? fit_defer_rb(s, s->defer_rb_req) : auto_defer_rb(s);
    }
    if (s->gexec) { (void)hipGraphExecDestroy(s->gexec); s->gexec = nullptr; }
    if (s->graph) { (void)hipGraphDestroy(s->graph); s->graph = nullptr; }
    return DLP_OK;
}

int dlp_sessions_connect(dlp_session* const* ranks, int nranks) {
    if (!ranks || nranks <= 0 || nranks > dlp::kMaxRanks) return DLP_ERR_ARG;
    std::vector<dlp_session*> by(nranks, nullptr);
    for (int k = 0; k < nranks; ++k) {
        dlp_session* s = ranks[k];
        if (!s || s->nranks != nranks || s->rank < 0 || s->rank >= nranks || by[s->rank]) {
            set_error("dlp_sessions_connect: every rank session of the solve, once each");
            return DLP_ERR_ARG;
        }
        by[s->rank] = s;
    }
    if (const char* e = std::getenv("DLP_TEST_PEER_FAIL")) {   // tests only
        set_error("rank " + std::string(e) + ": injected (DLP_TEST_PEER_FAIL)");
        return DLP_ERR_UNSUPPORTED;
    }
    for (dlp_session* s : by) CALL_TRY(ensure_xblock(s));
    // direct peer access between the devices involved (xGMI)
    for (dlp_session* a : by)
        for (dlp_session* b : by) {
            if (a->device == b->device) continue;
            int ok = 0;
            HIP_TRY(hipDeviceCanAccessPeer(&ok, a->device, b->device));
            if (!ok) {
                set_error("device " + std::to_string(a->device) + " cannot access device " +
                          std::to_string(b->device));
                return DLP_ERR_UNSUPPORTED;
            }
            HIP_TRY(hipSetDevice(a->device));
            const hipError_t e = hipDeviceEnablePeerAccess(b->device, 0);
            (void)hipGetLastError();
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                set_error("hipDeviceEnablePeerAccess(" + std::to_string(a->device) + " -> " +
                          std::to_string(b->device) + "): " + hipGetErrorString(e));
                return DLP_ERR_UNSUPPORTED;
            }
        }
    std::vector<uint64_t*> bases(nranks);
    for (int r = 0; r < nranks; ++r) bases[r] = by[r]->xblk;
    std::vector<int> devs(nranks);
    for (int r = 0; r < nranks; ++r) devs[r] = by[r]->device;
    for (dlp_session* s : by) {
        HIP_TRY(hipSetDevice(s->device));
        HIP_TRY(hipStreamSynchronize(s->stream));
        CALL_TRY(install_peers(s, bases, devs));
        CALL_TRY(la_policy(s));
    }
    return DLP_OK;
}

int dlp_session_exchange_handle(dlp_session* s, void* out64) {
    if (!s || !out64) return DLP_ERR_ARG;
    CALL_TRY(ensure_xblock(s));
    hipIpcMemHandle_t h;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipIpcGetMemHandle(&h, s->xblk));
    std::memcpy(out64, &h, sizeof(h));
    return DLP_OK;
}

int dlp_session_exchange_record(dlp_session* s, void* out256) {
    if (!s || !out256) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    XRec me;
    make_xrec(s, &me);
    if (!me.ok) {
        set_error(std::string("dlp_session_exchange_record: ") + std::string(me.why, strnlen(me.why, sizeof(me.why))));
        return DLP_ERR_UNSUPPORTED;
    }
    static_assert(sizeof(XRec) == DLP_XREC_BYTES, "XRec is the exchange record");
    std::memcpy(out256, &me, sizeof(me));
    return DLP_OK;
}

int dlp_session_connect_records(dlp_session* s, const void* records) {
    if (!s || !records) return DLP_ERR_ARG;
    if (!s->ipc_open.empty() || s->xmode == dlp_session::X_PEER) {
        set_error("dlp_session_connect_records: already connected");
        return DLP_ERR_STATE;
    }
    CALL_TRY(ensure_xblock(s));
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    std::vector<XRec> all(s->nranks);
    std::memcpy(all.data(), records, sizeof(XRec) * s->nranks);
    for (int r = 0; r < s->nranks; ++r)
        if (!all[r].ok) {
            set_error("dlp_session_connect_records: rank " + std::to_string(r) + " has no record");
            return DLP_ERR_ARG;
        }
    XRec out{};
    out.ok = 1;
    std::vector<void*> opened;
    std::vector<uint64_t*> bases;
    std::vector<int> devs;
    open_peer_blocks(s, all.data(), &out, &opened, &bases, &devs);
    if (!out.ok) {
        set_error(std::string("peer exchange unavailable: ") + std::string(out.why, strnlen(out.why, sizeof(out.why))));
        return DLP_ERR_UNSUPPORTED;
    }
    s->ipc_open.insert(s->ipc_open.end(), opened.begin(), opened.end());
    CALL_TRY(install_peers(s, bases, devs));
    return la_policy(s);
}

int dlp_session_colocated(dlp_session* s, int* n, int* index) {
    if (!s || !n || !index) return DLP_ERR_ARG;
    *n = s->coloc_n;
    *index = s->coloc_i;
    return DLP_OK;
}

int dlp_session_connect_ipc(dlp_session* s, const void* handles) {
    if (!s || !handles) return DLP_ERR_ARG;
    if (!s->ipc_open.empty() || s->xmode == dlp_session::X_PEER) {
        set_error("dlp_session_connect_ipc: already connected");
        return DLP_ERR_STATE;
    }
    return connect_ipc(s, (const uint8_t*)handles);
}

int dlp_session_set_exchange(dlp_session* s, int mode) {
    if (!s || (mode != DLP_XCHG_RCCL && mode != DLP_XCHG_PEER)) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (mode == DLP_XCHG_RCCL) {
        if (!s->comm) {
            set_error("the session has no RCCL communicator");
            return DLP_ERR_STATE;
        }
        s->xmode = dlp_session::X_RCCL;
        return la_policy(s);
    }
    if (s->xpeers_host.nranks == s->nranks && s->xpeers_host.base[s->rank] == s->xblk && s->xblk) {
        s->xmode = dlp_session::X_PEER;   // connected before
        return la_policy(s);
    }
    if (!s->comm) {
        set_error("dlp_session_set_exchange(PEER) without a communicator: use dlp_sessions_connect "
                  "or dlp_session_connect_ipc");
        return DLP_ERR_STATE;
    }
    return settle_exchange(s, DLP_XCHG_PEER);   // every rank's IPC handle over the communicator
}

int dlp_session_exchange_reason(dlp_session* s, char* buf, size_t cap) {
    if (!s || !buf || cap == 0) return DLP_ERR_ARG;
    std::snprintf(buf, cap, "%s", s->xreason.c_str());
    return DLP_OK;
}

int dlp_session_get_exchange(dlp_session* s, int* mode) {
    if (!s || !mode) return DLP_ERR_ARG;
    *mode = s->xmode;
    return DLP_OK;
}

int dlp_sessions_run(dlp_session* const* ranks, int nranks, int64_t max_pivots, int64_t* pivots_done) {
    if (!ranks || nranks <= 0 || max_pivots < 0) return DLP_ERR_ARG;
    std::vector<dlp_session*> ss(ranks, ranks + nranks);
    for (dlp_session* s : ss)
        if (!s || s->nranks != nranks || s->cluster ||
            (nranks > 1 && s->xmode != dlp_session::X_PEER)) {
            set_error("dlp_sessions_run: the rank sessions of one solve, connected by dlp_sessions_connect");
            return DLP_ERR_STATE;
        }
    dlp_session* s0 = ss[0];
    const int64_t start = s0->npivots;
    int64_t budget = std::min<int64_t>(max_pivots, s0->opt.max_pivots - s0->launched);
    // ranks that share a device keep every wait in a launch of its own (no xfuse): their
    // streams may share a hardware queue, where a launch that waits must come after the
    // launches of the other ranks it waits for (the phase interleaving below)
    bool shared = false;
    for (int a = 0; a < nranks; ++a)
        for (int b = a + 1; b < nranks; ++b) shared = shared || ss[a]->device == ss[b]->device;
    struct FuseGuard {
        std::vector<dlp_session*>& v;
        std::vector<bool> keep;
        FuseGuard(std::vector<dlp_session*>& v_, bool off) : v(v_) {
            for (dlp_session* s : v) {
                keep.push_back(s->xfuse);
                if (off) s->xfuse = false;
            }
        }
        ~FuseGuard() {
            for (size_t k = 0; k < v.size(); ++k) v[k]->xfuse = keep[k];
        }
    } fuse_guard(ss, shared);
    auto poll_all = [&]() -> int {
        for (dlp_session* s : ss) {
            HIP_TRY(hipSetDevice(s->device));
            CALL_TRY(poll(s));
        }
        for (dlp_session* s : ss)
            if (s->status != s0->status || s->npivots != s0->npivots) {
                set_error("dlp_sessions_run: ranks diverged");
                return DLP_ERR_STATE;
            }
        return DLP_OK;
    };
    while (s0->status == DLP_RUNNING && budget > 0) {
        if (s0->drive_next < s0->drive.size() || s0->carry_pending) {   // Phase I -> II switch
            while (s0->drive_next < s0->drive.size() && budget > 0) {
                const int64_t row = s0->drive[s0->drive_next];
                for (int ph = 0; ph < 3; ++ph) CALL_TRY(sessions_phase(ss.data(), nranks, ph, 0, true, 1, row));
                for (dlp_session* s : ss) {
                    s->drive_next += 1;
                    s->launched += 1;
                }
                budget -= 1;
            }
            if (s0->drive_next == s0->drive.size() && s0->carry_pending) {
                for (int ph = 0; ph < 3; ++ph) CALL_TRY(sessions_phase(ss.data(), nranks, ph, 0, true, 2, 0));
                for (dlp_session* s : ss) {
                    HIP_TRY(hipSetDevice(s->device));
                    CALL_TRY(finish_phase1(s));
                }
            } else {
                CALL_TRY(poll_all());
            }
            continue;
        }
        const int64_t chunk = std::min<int64_t>(budget, s0->opt.check_interval);
        for (int64_t k = 0; k < chunk; ++k)
            for (int ph = 0; ph < 3; ++ph)
                CALL_TRY(sessions_phase(ss.data(), nranks, ph, k, k == chunk - 1, 0, 0));
        for (dlp_session* s : ss) {
            s->ev_pending = s->ev_per_pivot ? chunk : 0;
            s->launched += chunk;
        }
        budget -= chunk;
        CALL_TRY(poll_all());
    }
    if (pivots_done) *pivots_done = s0->npivots - start;
    if (s0->status != DLP_RUNNING) return s0->status;
    if (s0->launched >= s0->opt.max_pivots) return DLP_PIVOT_LIMIT;
    return DLP_RUNNING;
}

int dlp_session_set_exchange_timeout(dlp_session* s, double seconds) {
    if (!s || !(seconds >= 0.0)) return DLP_ERR_ARG;
    s->stall_limit_s = seconds;
    if (s->xpeers) {   // the device waits' own bound follows (between runs: the stream is idle)
        s->xpeers_host.wait_ticks = xwait_ticks(seconds);
        HIP_TRY(hipSetDevice(s->device));
        HIP_TRY(hipStreamSynchronize(s->stream));
        HIP_TRY(hipMemcpy(s->xpeers, &s->xpeers_host, sizeof(s->xpeers_host), hipMemcpyHostToDevice));
    }
    return DLP_OK;
}

int dlp_session_abort(dlp_session* s) {
    if (!s) return DLP_ERR_ARG;
    s->abort_req.store(1);
    return DLP_OK;
}

int dlp_session_inject_fault(dlp_session* s, int64_t after_polls) {
    if (!s || after_polls < 0) return DLP_ERR_ARG;
    s->fault_after_polls = after_polls;
    s->npolls = 0;
    return DLP_OK;
}

int dlp_session_get_lookahead(dlp_session* s, int* on) {
    if (!s || !on) return DLP_ERR_ARG;
    *on = s->la ? 1 : 0;
    return DLP_OK;
}

int dlp_session_set_fused_pivot(dlp_session* s, int on) {
    if (!s || on < 0 || on > 1) return DLP_ERR_ARG;   // (a condensed session keeps two launches)
    s->fuse_pivot = on != 0;
    if (s->gexec) { (void)hipGraphExecDestroy(s->gexec); s->gexec = nullptr; }
    if (s->graph) { (void)hipGraphDestroy(s->graph); s->graph = nullptr; }
    return DLP_OK;
}

int dlp_session_get_defer_tuning(dlp_session* s, int* occupancy, int* form, int* K) {
    if (!s) return DLP_ERR_ARG;
    if (occupancy) *occupancy = s->defer_occ;
    if (form) *form = s->d.K > 1 ? s->d.form : -1;
    if (K) *K = s->d.K;
    return DLP_OK;
}

int dlp_session_reset_timings(dlp_session* s) {
    if (!s) return DLP_ERR_ARG;
    for (double& t : s->timings) t = 0.0;
    s->nsamples = 0;
    s->upd_launches = 0;
    return DLP_OK;
}

int dlp_session_update_stats(dlp_session* s, int64_t* launches, double* ms, int* defer) {
    if (!s) return DLP_ERR_ARG;
    if (launches) *launches = s->upd_launches;
    if (ms) *ms = s->timings[DLP_PHASE_UPDATE];
    if (defer) *defer = s->d.K;
    return DLP_OK;
}

// the row stride of dlp_session_tableau / read_rows: the stored one, or for a condensed tableau the
// full layout's roundup(N + 1, 16)
static int64_t logical_ld(const dlp_session* s) { return s->g.cd.on ? s->ld_full : s->ld; }

int dlp_session_info(dlp_session* s, int64_t* rows_local, int64_t* row_first, int64_t* ld,
                     int64_t* ncols) {
    if (!s) return DLP_ERR_ARG;
    if (rows_local) *rows_local = s->rows;
    if (row_first) *row_first = s->row_first;
    if (ld) *ld = logical_ld(s);
    if (ncols) *ncols = s->N;
    return DLP_OK;
}

int dlp_session_storage(dlp_session* s, int64_t* ld, int64_t* ncols, int* condensed) {
    if (!s) return DLP_ERR_ARG;
    if (ld) *ld = s->ld;
    if (ncols) *ncols = s->g.ncols;
    if (condensed) *condensed = s->g.cd.on;
    return DLP_OK;
}

int dlp_session_tableau(dlp_session* s, double* host) {
    if (!s || !host) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    CALL_TRY(flush_pending(s));
    if (s->g.cd.on) return cond_read_rows(s, 0, s->rows + 1, host, logical_ld(s));
    HIP_TRY(hipMemcpyAsync(host, s->T, sizeof(double) * (s->rows + 1) * s->ld,
                           hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return DLP_OK;
}

int dlp_session_read_rows(dlp_session* s, int64_t first, int64_t count, double* host) {
    if (!s || !host || first < 0 || count < 0 || first + count > s->rows + 1) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    CALL_TRY(flush_pending(s));
    if (s->g.cd.on) return cond_read_rows(s, first, count, host, logical_ld(s));
    HIP_TRY(hipMemcpyAsync(host, s->T + first * s->ld, sizeof(double) * count * s->ld,
                           hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return DLP_OK;
}

int dlp_session_result(dlp_session* s, dlp_result** out) {
    if (!s || !out) return DLP_ERR_ARG;
    HIP_TRY(hipSetDevice(s->device));
    CALL_TRY(flush_pending(s));
    auto* r = new (std::nothrow) dlp_result();
    if (!r) return DLP_ERR_OOM;
    int rc = extract_result(s, r);
    if (rc != DLP_OK) {
        delete r;
        return rc;
    }
    *out = r;
    return DLP_OK;
}

void dlp_session_free(dlp_session* s) { free_session(s); }

int dlp_sessions_result(dlp_session* const* ranks, int nranks, dlp_result** out) {
    if (!ranks || nranks <= 0 || !out) return DLP_ERR_ARG;
    for (int k = 0; k < nranks; ++k)
        if (!ranks[k] || ranks[k]->nranks != nranks) {
            set_error("dlp_sessions_result: every rank session of the solve, once each");
            return DLP_ERR_ARG;
        }
    auto* r = new (std::nothrow) dlp_result();
    if (!r) return DLP_ERR_OOM;
    const int rc = merge_result(ranks, nranks, r);
    if (rc != DLP_OK) {
        delete r;
        return rc;
    }
    *out = r;
    return DLP_OK;
}

int dlp_solve(const dlp_problem* prob, const dlp_options* opt, dlp_result** out) {
    dlp_options o;
    if (opt)
        o = *opt;
    else
        dlp_options_default(&o);
    if (!prob || !out) return DLP_ERR_ARG;
    if (o.n_gpus < 0) {
        set_error("n_gpus must be >= 0");
        return DLP_ERR_ARG;
    }
    if (o.n_gpus >= 1) {
        CALL_TRY(validate_options(&o));
        return solve_in_process(prob, o, o.n_gpus, out);
    }
    dlp_session* s = nullptr;
    CALL_TRY(dlp_session_create(prob, &o, &s));
    int64_t done = 0;
    int rc = dlp_session_run(s, o.max_pivots, &done);
    if (rc < 0) {
        dlp_session_free(s);
        return rc;
    }
    rc = dlp_session_result(s, out);
    dlp_session_free(s);
    return rc;
}

int dlp_result_status(const dlp_result* r) { return r ? r->status : DLP_ERR_ARG; }
double dlp_result_objective(const dlp_result* r) { return r ? r->objective : NAN; }
int64_t dlp_result_num_pivots(const dlp_result* r) { return r ? r->npivots : -1; }

int dlp_result_x(const dlp_result* r, double* x, int64_t n) {
    if (!r || !x || n != r->n) return DLP_ERR_ARG;
    std::memcpy(x, r->x.data(), sizeof(double) * n);
    return DLP_OK;
}
int dlp_result_y(const dlp_result* r, double* y, int64_t m) {
    if (!r || !y || m != r->m) return DLP_ERR_ARG;
    std::memcpy(y, r->y.data(), sizeof(double) * m);
    return DLP_OK;
}
int dlp_result_basis(const dlp_result* r, int32_t* basis, int64_t m) {
    if (!r || !basis || m != (int64_t)r->basis.size()) return DLP_ERR_ARG;
    std::memcpy(basis, r->basis.data(), sizeof(int32_t) * m);
    return DLP_OK;
}
int dlp_result_info(const dlp_result* r, int64_t* m_basis, int64_t* phase1_pivots) {
    if (!r) return DLP_ERR_ARG;
    if (m_basis) *m_basis = (int64_t)r->basis.size();
    if (phase1_pivots) *phase1_pivots = r->phase1_pivots;
    return DLP_OK;
}
int dlp_result_pivot_log(const dlp_result* r, dlp_pivot* log, int64_t cap, int64_t* count) {
    if (!r) return DLP_ERR_ARG;
    const int64_t n = (int64_t)r->log.size();
    if (count) *count = n;
    if (log && cap > 0) std::memcpy(log, r->log.data(), sizeof(dlp_pivot) * std::min(cap, n));
    return DLP_OK;
}
int dlp_result_timings(const dlp_result* r, double* ms_out) {
    if (!r || !ms_out) return DLP_ERR_ARG;
    for (int ph = 0; ph < DLP_NUM_PHASES; ++ph) ms_out[ph] = r->timings[ph];
    return DLP_OK;
}
int dlp_release_cached_memory(int device, int64_t* bytes) {
    streams_drain(device);
    const size_t n = pool_drain(device < 0 ? kAllDevices : device) + dlp::batched_release(device);
    if (bytes) *bytes = (int64_t)n;
    return DLP_OK;
}
int dlp_result_exchange(const dlp_result* r, int* mode, char* reason, int64_t cap) {
    if (!r) return DLP_ERR_ARG;
    if (mode) *mode = r->exchange;
    if (reason && cap > 0) std::snprintf(reason, (size_t)cap, "%s", r->exchange_reason.c_str());
    return DLP_OK;
}
void dlp_result_free(dlp_result* r) { delete r; }

}  // extern "C"
