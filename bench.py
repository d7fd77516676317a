#!/usr/bin/env python3
"""Benchmark: simplex pivots/s + achieved HBM GB/s of the tableau update on a
dense fp64 tableau (BASELINE.json metric), 1/2/4/8 MI355X.

    python bench.py [--gpus N] [--steps S] [--warmup W] [--workload c3|c2]
                    [--step-unit block|pivot]

What is timed: pivots of ONE LP whose tableau is resident in HBM, row-block
partitioned over the N ranks (one process per GPU, exchange inside libdlp).  For
N > 1 run it either under torch.distributed.run (WORLD_SIZE set) or plainly as
`python3 bench.py --gpus N`: then bench.py starts its own N rank processes
(launch_ranks) and relays rank 0's line.  The LP is fixed as N
grows, so scaling is strong.  Default workload C3: m = n = 32768 (N = 65536,
17.2 GB tableau), generated on the device (synthetic, seed 3 = config id).

A "step" is one pass of the hot path over the tableau.  The update is the
deferred rank-K form: K pivots are selected (pricing, ratio
test, pivot-row exchange) on replayed views of the resident tableau, then ONE
HBM pass applies all K to every element, bit-identical to K rank-1 updates.
So with --step-unit block (default) a step = K pivots + their tableau pass
(K = 64 at C3), and S steps time S*K pivots, every one of them fully applied
(a window never ends with pivots pending).  With --step-unit pivot a step is
one pivot, and the window's last pass covers only its last partial block
(DESIGN.md §6 explains the difference).  `value` is pivots/s either way.

Rank 0 prints ONE JSON line.  roofline prices the tableau pass: algorithmic
bytes per launch = 16 * rows_local * (N + 1) (one read + one write of every
constraint element) over its mean launch time from HIP events
on the session stream.  `traffic` is the committed rocprofv3 PMC summary of the
same kernel at the same geometry (profiles/, tools/pmc_summary.py), or null
when none matches.  cpu_baseline (rank 0, N = 1 only) is the in-repo CPU
oracle (same pivot rule, test infrastructure) on a bounded sample of the same
LP: all host threads available to this process, then 1 thread.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: (m, n, seed, description)
    "c3": (32768, 32768, 3, "C3 dense LP 32768 x 32768 (+32768 slack): fp64 tableau 32769 x 65537, "
                            "row-block over the GPUs"),
    "c2": (4096, 4096, 2, "C2 dense LP 4096 x 4096 (+4096 slack): fp64 tableau 4097 x 8193"),
    # the per-rank floor of the 8-GPU C3 split, on ONE GPU: a rank of C3 at P = 8 holds 4,096 rows
    # of the condensed tableau's 32,769 columns (the n = 32,768 nonbasic columns + RHS, DESIGN.md
    # §16); a 4096 x 32768 LP has exactly that stored tableau.  Run as a 1-rank exchange session
    # (RCCL id, nranks = 1), so the chain carries the select / commit kernels and the exchange
    # stores a rank of the split runs; only the xGMI latency is missing.  (Round 5's c3rP LPs,
    # 4096 x 61440 etc., matched the full tableau's 65,537 columns.)
    "c3r8": (4096, 32768, 38, "C3 rank geometry at P = 8: dense LP 4096 x 32768, condensed fp64 tableau "
                              "4097 x 32769 = one rank of the 8-GPU C3 split, 1-rank exchange"),
    "c3r4": (8192, 32768, 34, "C3 rank geometry at P = 4: dense LP 8192 x 32768, condensed fp64 tableau "
                              "8193 x 32769 = one rank of the 4-GPU C3 split, 1-rank exchange"),
    "c3r2": (16384, 32768, 32, "C3 rank geometry at P = 2: dense LP 16384 x 32768, condensed fp64 tableau "
                               "16385 x 32769 = one rank of the 2-GPU C3 split, 1-rank exchange"),
}
RANK_WORKLOADS = ("c3r2", "c3r4", "c3r8")
# C5 (BASELINE.json configs[4]): 4,096 independent 64 x 128 LPs, one workgroup per LP
C5 = {"nlp": 4096, "m": 64, "n": 128, "seed": 5000}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP64_PEAK_TFS = 77.3   # measured v_fma_f64 peak on MI355X (tools/passlab.hip valu probe)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--step-unit", default="block", choices=("block", "pivot"),
                    help="block: a step is K pivots + one rank-K tableau pass; pivot: one pivot")
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS) + ["c5"],
                    help="c5: the batched small-LP workload (a step = one solve of the whole batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU baseline: time budget of each oracle window (all CPUs, OMP share, 1)")
    ap.add_argument("--no-eager-window", action="store_true",
                    help="skip the eager rank-1 (defer = 1) roofline window on the same LP")
    ap.add_argument("--eager-pivots", type=int, default=3)
    ap.add_argument("--no-pivot-window", action="store_true",
                    help="skip the extra --step-unit pivot window reported beside the main figure")
    ap.add_argument("--exchange", default="auto", choices=("auto", "rccl", "peer"),
                    help="N > 1 (and c3r8): the main window's row-block exchange: owner-rooted peer stores "
                         "into the ranks' exchange blocks, or RCCL collectives; auto = peer where every "
                         "rank pair connects, else RCCL (the reason is reported)")
    ap.add_argument("--alt-pivots", type=int, default=256,
                    help="N > 1: pivots of the second window, run with the other exchange (0 = none)")
    ap.add_argument("--rows-per-block", type=int, default=0)
    ap.add_argument("--nontemporal", type=int, default=-1, help="-1 = auto")
    ap.add_argument("--variant", type=int, default=-1, help="update-kernel variant, -1 = auto")
    ap.add_argument("--ld-align", type=int, default=0, help="row alignment (doubles), 0 = auto")
    ap.add_argument("--timing", type=int, default=1,
                    help="1 = HIP events around the update/pass launches only, 2 = every phase")
    ap.add_argument("--defer", type=int, default=0,
                    help="pivots per tableau pass (1 = eager rank-1 per pivot, 0 = auto)")
    ap.add_argument("--occupancy", type=int, default=-1, help="pass workgroups/CU cap (-1 = default)")
    ap.add_argument("--form", type=int, default=-1, help="pass kernel form (-1 = default)")
    ap.add_argument("--lookahead", type=int, default=-1,
                    help="select block b+1 during the pass of block b: 1 on, 0 off, -1 auto")
    ap.add_argument("--pmc-dir", default=None,
                    help="rocprofv3 --pmc output dir (FETCH_SIZE / WRITE_SIZE) to fill roofline.traffic")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="--gpus N > 1 without a launcher: seconds the N rank processes may take in all "
                         "before every one is killed and bench.py exits 124")
    ap.add_argument("--launch-grace", type=float, default=30.0,
                    help="--gpus N > 1 without a launcher: seconds the other ranks get to end on their own "
                         "after one rank fails")
    ap.add_argument("--stub-worker", default=None, choices=("ok", "fail1", "hang1"),
                    help=argparse.SUPPRESS)   # tests/test_bench_launcher.py: a rank that does no GPU work
    return ap.parse_args()


# ---------------------------------------------------------------------------------------------
# rank launcher: `python3 bench.py --gpus N` with no WORLD_SIZE in the environment starts its
# own N rank processes (one per GPU), so the driver's scaling run works whether or not it goes
# through torch.distributed.run.  The parent never touches the GPU (no torch.cuda, no libdlp):
# it only spawns children (never an exec), relays rank 0's JSON line and reports failures.
# ---------------------------------------------------------------------------------------------

def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _die_with_parent():
    """preexec_fn of a rank child: SIGKILL when the launcher dies (Linux PR_SET_PDEATHSIG), so a
    killed launcher never leaves ranks on the GPUs.  Runs between fork and exec in the child; the
    launcher has made no GPU call."""
    try:
        import ctypes
        import signal
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGKILL))
    except Exception:  # noqa: BLE001 - best effort: without it the launcher's own kill still runs
        pass


def launch_ranks(n, argv, timeout_s, grace_s=30.0, out=None, err=None):
    """Start N rank processes of this script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT (127.0.0.1, a free port), wait for all of them, and return the exit code:
    0 when every rank exited 0 and rank 0 printed a JSON line (relayed once to `out`), else the
    first failing rank's code, 124 when the ranks outlived `timeout_s`, 1 when rank 0 printed no
    line.  When one rank fails the others get `grace_s` to end on their own (an exchange timeout
    ends a healthy rank in bounded time), then are terminated and killed by PID."""
    import subprocess
    import threading
    out = out or sys.stdout
    err = err or sys.stderr
    port = _free_port()
    script = os.path.abspath(__file__)
    procs, lines, lock = [], [], threading.Lock()

    def pump(r, stream):
        for raw in stream:
            s = raw.rstrip("\n")
            parsed = None
            if r == 0 and s.startswith("{"):
                try:
                    parsed = json.loads(s)
                except ValueError:
                    parsed = None
            with lock:
                if isinstance(parsed, dict) and "metric" in parsed:
                    lines.append(s)
                else:
                    print(f"[rank {r}] {s}", file=err, flush=True)

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", NODE_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   DLP_BENCH_LAUNCHER="1")
        p = subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env, stdout=subprocess.PIPE,
                             stderr=None, text=True, preexec_fn=_die_with_parent)
        procs.append(p)
    pumps = [threading.Thread(target=pump, args=(r, p.stdout), daemon=True) for r, p in enumerate(procs)]
    for t in pumps:
        t.start()

    def stop_all(why):
        print(f"bench launcher: {why}; stopping ranks "
              f"{[r for r, p in enumerate(procs) if p.poll() is None]}", file=err, flush=True)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.monotonic() + 10.0
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    import signal

    def on_signal(signum, _frame):
        stop_all(f"launcher got signal {signum}")
        raise SystemExit(128 + signum)
    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        deadline = time.monotonic() + timeout_s
        first_fail, code = None, 0
        while True:
            codes = [p.poll() for p in procs]
            if all(c is not None for c in codes):
                break
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad and first_fail is None:
                first_fail = time.monotonic()
                code = bad[0][1]
                print(f"bench launcher: rank {bad[0][0]} exited with {bad[0][1]}", file=err, flush=True)
            if first_fail is not None and time.monotonic() - first_fail > grace_s:
                stop_all(f"{grace_s:g} s after the first rank failure")
                break
            if time.monotonic() > deadline:
                stop_all(f"ranks still running after {timeout_s:g} s (--launch-timeout)")
                code = code or 124
                break
            time.sleep(0.1)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    for t in pumps:
        t.join(timeout=5.0)
    codes = [p.returncode for p in procs]
    if code == 0:
        code = next((c for c in codes if c != 0), 0)
        if code < 0:   # killed by a signal
            code = 128 - code
    if code == 0 and not lines:
        print("bench launcher: rank 0 printed no JSON line", file=err, flush=True)
        code = 1
    if code == 0:
        print(lines[-1], file=out, flush=True)
    else:
        print(f"bench launcher: exit codes by rank {codes}", file=err, flush=True)
    return code


def stub_worker(args):
    """--stub-worker (tests only): a rank that checks its launcher environment, joins a gloo
    group over MASTER_ADDR:MASTER_PORT and all-gathers its rank, with no GPU work.  fail1: rank 1
    exits 3 before the rendezvous; hang1: rank 1 sleeps."""
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert int(os.environ["LOCAL_RANK"]) == rank and world == args.gpus
    if rank == 1 and args.stub_worker == "fail1":
        raise SystemExit(3)
    if rank == 1 and args.stub_worker == "hang1":
        time.sleep(3600)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.zeros(world, dtype=torch.int64)
    t[rank] = rank + 1000 * os.getpid()
    dist.all_reduce(t)
    if rank == 0:
        print("stub rank 0 starting", flush=True)   # non-JSON output is relayed to stderr
        print(json.dumps({"metric": "stub", "value": world, "ranks": [int(v) % 1000 for v in t],
                          "pids": [int(v) // 1000 for v in t],
                          "master": [os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"]]}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def pmc_traffic(pmc_dir: str, kernel_substr: str):
    """Per-launch HBM bytes of the update kernel from rocprofv3 counter CSVs:
    (2 x FETCH_SIZE + WRITE_SIZE) KiB -> bytes (gfx950 FETCH_SIZE reads 1/2 of a
    wide coalesced stream: MI355X_MICROARCH.md §HBM)."""
    import csv
    import glob
    fetch, write = [], []
    for path in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel_substr not in row.get("Kernel_Name", ""):
                    continue
                name, val = row.get("Counter_Name"), float(row.get("Counter_Value", 0))
                if name == "FETCH_SIZE":
                    fetch.append(val)
                elif name == "WRITE_SIZE":
                    write.append(val)
    if not fetch or not write:
        return None
    return (2.0 * sum(fetch) / len(fetch) + sum(write) / len(write)) * 1024.0


def committed_traffic(key: dict):
    """The committed PMC summary (profiles/r*/*_pmc_traffic.json, written by
    tools/pmc_summary.py) whose recorded geometry equals this run's `key`
    (workload, kernel kind, K, form, band rows, nt, ld); (None, None) when none
    matches, so a summary of another kernel or geometry is never reported."""
    import glob
    hits = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "r*", "*_pmc_traffic.json")):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        geo = d.get("geometry")
        if isinstance(geo, dict) and all(geo.get(k) == v for k, v in key.items()) \
                and d.get("traffic_bytes_per_launch"):
            hits.append((os.path.relpath(path, ROOT), d["traffic_bytes_per_launch"]))
    if not hits:
        return None, None

    def order(h):   # the latest run: profiles/rRRxx in the order the runs were named (r05z < r05aa)
        import re
        m = re.search(r"profiles/r(\d+)([a-z]*)", h[0].replace(os.sep, "/"))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (0, 0, "")
    src, val = max(hits, key=order)
    return val, src


def cpu_info():
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return model, os.cpu_count() or 1, avail


def cpu_baseline(m, n, seed, budget_s, K=1):
    """The in-repo C++ oracle (same pivot rule, OpenMP over rows; test
    infrastructure: the CPU comparator only) on the same LP, SURVEY.md §8(d):
    every CPU this process may use (sched_getaffinity, passed to the oracle
    explicitly, not inherited from OMP_NUM_THREADS), then the same LP continued
    on OMP_NUM_THREADS threads (the box's per-GPU CPU share, when set) and on 1
    thread.  `value` is the faster multi-thread run (threads_for_value says
    which); every run is reported.  With K > 1, `like_for_like` times the GPU's own
    deferred rank-K algorithm on the host (oracle/oracle_defer.inc) on those threads."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py  # test infrastructure: the CPU comparator only
    model, nproc, avail = cpu_info()
    omp = os.environ.get("OMP_NUM_THREADS")
    share = int(omp) if (omp and omp.isdigit() and 0 < int(omp) < avail) else None
    plan = [(avail, 100000, budget_s)] + ([(share, 100000, budget_s)] if share else []) + \
           [(1, 100000, budget_s)]
    runs, gen = oracle_py.bench_windows(m, n, seed, plan, gen_threads=avail)
    for (secs, k), (thr, _, _) in zip(runs, plan):
        if not (secs and k):
            raise RuntimeError(f"CPU baseline sample too small: {k} pivots in {secs} s on {thr} threads "
                               f"(the LP ended inside the sample)")
    rate = {thr: k / secs for (secs, k), (thr, _, _) in zip(runs, plan)}
    where = (f"{model}; os.cpu_count() = {nproc}, {avail} usable by this process"
             + (f", OMP_NUM_THREADS = {omp}" if omp else ""))
    # value: the faster of the all-CPU and per-GPU-share runs (on a box whose cgroup grants this
    # process a CPU share below its affinity mask, 256 threads run slower than 16); both kept
    best = max((t for t in rate if t > 1), key=lambda t: rate[t], default=1)
    out = {"value": rate[best], "unit": "pivots/s", "cores": best, "kind": "port",
           "threads_for_value": best, "all_cpus": {"value": rate[avail], "unit": "pivots/s", "cores": avail},
           "cpu_model": model, "nproc": nproc, "cpus_usable": avail,
           "sample": (f"in-repo C++ oracle (same pivot rule, eager rank-1, OpenMP over rows) on the same "
                      f"LP {m}x{n} seed {seed}: 1 warm-up pivot, then consecutive windows of <= {budget_s:g} s "
                      f"each: " + ", ".join(f"{k} pivots in {secs:.2f} s on {thr} threads"
                                            for (secs, k), (thr, _, _) in zip(runs, plan))
                      + f" ({where}); host tableau generation {gen:.1f} s not timed"),
           "single_thread": {"value": rate[1], "unit": "pivots/s", "cores": 1,
                             "pivots": runs[-1][1], "seconds": runs[-1][0]}}
    if share:
        out["omp_share"] = {"value": rate[share], "unit": "pivots/s", "cores": share,
                            "pivots": runs[1][1], "seconds": runs[1][0]}
    if K > 1:
        # like-for-like: the GPU's own algorithm on the host — the oracle's
        # deferred rank-K restatement (oracle/oracle_defer.inc: replayed selections, then one
        # pass per block, bit-identical to eager), same LP, same K, whole blocks only, on the
        # thread count that gave `value`
        druns, dgen = oracle_py.bench_windows_defer(m, n, seed, K, [(best, 10 ** 6, budget_s)],
                                                    gen_threads=avail)
        dsecs, dk = druns[0]
        if not (dsecs and dk):
            raise RuntimeError(f"deferred CPU baseline: {dk} pivots in {dsecs} s (the LP ended inside the sample)")
        out["like_for_like"] = {
            "value": dk / dsecs, "unit": "pivots/s", "cores": best, "kind": "port",
            "algorithm": f"deferred rank-{K} (the GPU's): replayed selections + one pass per {K}-pivot block",
            "sample": (f"in-repo C++ oracle, oracle/oracle_defer.inc (AVX2 + FMA, OpenMP over row bands), same "
                       f"LP {m}x{n} seed {seed}: 1 warm-up block, then {dk} pivots = {dk // K} whole blocks "
                       f"in {dsecs:.2f} s on {best} threads ({where}); generation {dgen:.1f} s not timed")}
    return out


def log_parity(workload, log):
    """Self-check of the run: the pivot log against the committed digests of the oracle's run
    of the same LP (tests/golden/digests.json, tests/golden/make_digests.py: sha256 of log
    prefixes), at every committed prefix the run reached.  With N > 1 this is the row-block
    exchange's parity evidence at the bench size (the log is replicated on every rank)."""
    import hashlib
    path = os.path.join(ROOT, "tests", "golden", "digests.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    g = d.get("c3_k64" if workload == "c3" else workload)
    if not g or "log_prefix_sha256" not in g:
        return None
    prefixes = dict(g["log_prefix_sha256"])
    if workload == "c3":   # the whole-tableau stops carry log digests too (1876: the N > 1 second window)
        for k, st in d.get("c3_tableau", {}).get("stops", {}).items():
            prefixes.setdefault(k, st["log_sha256"])
    got = {}
    for k, h in prefixes.items():
        if int(k) <= len(log):
            got[k] = hashlib.sha256(log[:int(k)].tobytes()).hexdigest() == h
    if g.get("pivots") == len(log):
        got[str(len(log))] = hashlib.sha256(log.tobytes()).hexdigest() == g["log_sha256"]
    return {"source": "tests/golden/digests.json (oracle, same LP)", "prefixes_checked": sorted(got, key=int),
            "bit_identical": all(got.values()) if got else None}


def agree_any(flag, dist, torch, device):
    """True on every rank when `flag` is true on any rank (MAX all-reduce); the flag itself at N = 1."""
    if dist is None:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item()) != 0


def guarded_run(sess, pivots, timed, barrier_sync, any_rank, errors):
    """sess.run on every rank.  A failure (an exchange error or timeout: `errors`) is held until
    every rank has passed the same barriers, then agreed, so all ranks take the same next step
    and every collective stays matched."""
    err, st, done, el = None, None, 0, 0.0
    if timed:
        barrier_sync()
        t0 = time.perf_counter()
    try:
        st, done = sess.run(pivots)
    except errors as e:
        err = e
    if timed:
        barrier_sync()
        el = time.perf_counter() - t0
    return st, done, el, err, any_rank(err is not None)


def measure(sess, warm, timed, barrier_sync, any_rank, errors):
    """Warm-up window, then the timed window: (status, pivots done, seconds, error, failed on any rank)."""
    st, done, _, err, bad = guarded_run(sess, warm, False, barrier_sync, any_rank, errors)
    if bad:
        return st, done, 0.0, err, True
    if done != warm:
        raise SystemExit(f"warm-up ended early: status {st} after {done} pivots")
    sess.reset_timings()
    return guarded_run(sess, timed, True, barrier_sync, any_rank, errors)


def measure_with_fallback(sess, warm, timed, barrier_sync, any_rank, errors, reopen=None):
    """measure(); when it failed on any rank and `reopen` is given (N > 1, auto exchange, the peer
    exchange chosen), every rank closes its session and measures again on reopen()'s (RCCL).
    The owner-rooted exchange has never run across xGMI on this pool's one-GPU boxes.
    Returns (session, status, done, seconds, fallback reason or None, the new exchange name)."""
    st, done, el, err, bad = measure(sess, warm, timed, barrier_sync, any_rank, errors)
    why, name = None, None
    if bad and reopen is not None:
        why = f"peer exchange failed during the run: {err if err else 'on another rank'}"
        # a connected rank's exchange block receives its peers' stores: end every rank's device
        # waits (abort word), drain this rank's streams, and only after every rank has done so
        # (barrier) free anything (include/dlp.h, "Freeing connected ranks")
        sess.abort()
        barrier_sync()
        sess.close()
        sess, name = reopen()
        st, done, el, err, bad = measure(sess, warm, timed, barrier_sync, any_rank, errors)
    if bad:
        raise SystemExit(f"run failed: {err if err else 'on another rank'}")
    return sess, st, done, el, why, name


def alt_exchange_window(sess, dist, barrier_sync, args, L, torch):
    """Switch every rank to the other exchange and time args.alt_pivots pivots.  The switch
    to PEER all-gathers the exchange blocks' IPC handles over the session's communicator;
    every rank's outcome is agreed (MIN all-reduce) before anything is timed, and the window
    runs with a 60 s stall limit, so a broken path ends as an error field, never a hang."""
    mode, name = (L.XCHG_PEER, "peer") if sess.get_exchange() == L.XCHG_RCCL else (L.XCHG_RCCL, "rccl")
    out = {"exchange": name, "pivots": args.alt_pivots}
    ok = 1
    try:
        sess.set_exchange(mode)
        sess.set_exchange_timeout(60.0)
    except L.DLPError as e:
        ok, out["error"] = 0, str(e)
    t = torch.tensor([ok], dtype=torch.int32, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if int(t.item()) == 0:
        out.setdefault("error", "another rank failed to switch")
        return out
    barrier_sync()
    t0 = time.perf_counter()
    done = 0
    try:
        st, done = sess.run(args.alt_pivots)
    except L.DLPError as e:
        out["error"] = str(e)
    barrier_sync()   # every rank, failed or not, so the collectives below stay matched
    el = torch.tensor([time.perf_counter() - t0, 1.0 if "error" in out else 0.0], dtype=torch.float64,
                      device="cuda")
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if el[1].item() > 0:
        out.setdefault("error", "failed on another rank")
        return out
    out.update({"done": done, "seconds": float(el[0].item())})
    if done == args.alt_pivots:
        out["pivots_per_s"] = done / out["seconds"]
    return out


def c5_cpu_baseline(budget_s):
    """The oracle (same rule, 1 thread) on consecutive LPs of the C5 batch until budget_s of
    solve time (generation not timed): LPs/s on one core."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py  # test infrastructure: the CPU comparator only
    model, nproc, avail = cpu_info()
    secs, k, piv = 0.0, 0, 0
    while secs < budget_s and k < C5["nlp"]:
        A, b, c = oracle_py.gen_dense(C5["m"], C5["n"], C5["seed"] + k)
        t0 = time.perf_counter()
        r = oracle_py.solve_dense(A, b, c, nthreads=1, log_cap=0)
        secs += time.perf_counter() - t0
        piv += r.num_pivots
        k += 1
    return {"value": k / secs, "unit": "LPs/s", "cores": 1, "kind": "port", "cpu_model": model,
            "sample": f"in-repo C++ oracle (same rule, 1 thread) on LPs 0..{k - 1} of the batch: {k} LPs, "
                      f"{piv} pivots in {secs:.2f} s of solve time (generation not timed)"}


def c5_hardware_bound():
    """The committed SQ-counter summary of the batched kernel (profiles/r*/c5_hardware_bound.json,
    the latest): VALU-issue and LDS busy fractions, wave states; None when absent."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "c5_hardware_bound.json")))
    if not paths:
        return None
    try:
        with open(paths[-1]) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    keep = ("valu_issue_util", "lds_util", "wave_parked_frac", "wave_issue_stalled_frac", "effective_clock_ghz")
    out = {k: d[k] for k in keep if k in d}
    out["source"] = os.path.relpath(paths[-1], ROOT)
    return out


def c5_main(args):
    """--workload c5: the whole batch solved S times after W warm-ups.  A step = one
    dlp_batched_solve of the batch (tableaus generated on the device, then ONE solve kernel);
    `value` = LPs / s of solve-kernel time (HIP events around the kernel: inputs resident in
    HBM), the wall rate (allocation + generation + read-back included) beside it.  roofline:
    C5 is bound by per-pivot serial latency x residency, not by HBM or the FMA pipe
    (DESIGN.md §6): peak = resident LPs (occupancy query) / the single-LP pivot latency
    (256 LPs, one per CU), achieved = the batch's pivots / kernel time."""
    import torch
    import numpy as np
    import distributedlpsolver_amd as dlp
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    # strong split: rank r takes LPs [r nlp / P, (r + 1) nlp / P) of the batch (seeds seed + k)
    first, last = rank * C5["nlp"] // world, (rank + 1) * C5["nlp"] // world
    nlp, m, n = last - first, C5["m"], C5["n"]
    seed = C5["seed"] + first

    def solve():
        return dlp.batched_solve(nlp, m, n, seed, device=local, log_cap=0)

    def sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        solve()
    sync()
    t0 = time.perf_counter()
    kms, piv, allopt = [], [], True
    for _ in range(args.steps):
        br = solve()
        kms.append(br.kernel_ms)
        piv.append(int(br.num_pivots.sum()))
        allopt = allopt and bool((br.status == 0).all())
    sync()
    wall = time.perf_counter() - t0
    kern = sum(kms) * 1e-3
    if dist is not None:
        t = torch.tensor([wall, kern], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, kern = float(t[0].item()), float(t[1].item())
        # the whole batch's outcome, not rank 0's slice: every rank optimal, pivots summed
        a = torch.tensor([1 if allopt else 0], dtype=torch.int64, device="cuda")
        dist.all_reduce(a, op=dist.ReduceOp.MIN)
        allopt = bool(a.item())
        pv = torch.tensor(piv, dtype=torch.int64, device="cuda")
        dist.all_reduce(pv, op=dist.ReduceOp.SUM)
        piv = [int(v) for v in pv.tolist()]
    occ = dlp.batched_occupancy(m, n, local)
    cus = torch.cuda.get_device_properties(local).multi_processor_count
    # single-LP serial latency: 256 LPs of the batch, one per CU
    one = dlp.batched_solve(min(256, nlp), m, n, seed, device=local, log_cap=0)
    t1 = one.kernel_ms * 1e-3 / max(int(one.num_pivots.max()), 1)
    resident = min(nlp, occ["lps_per_cu"] * cus)
    peak = resident / t1   # pivots/s with every resident LP at the single-LP latency
    achieved = piv[-1] * args.steps / kern     # pivots of the whole batch (all ranks) per second
    pivots_lp = piv[-1] / C5["nlp"]
    if rank == 0:
        total = C5["nlp"] * args.steps
        bytes_solve = 16.0 * C5["nlp"] * (m + 1) * (m + n + 1)   # one read + one write of every tableau
        line = {
            "metric": "batched simplex: LPs/s (C5, 4096 independent 64x128 fp64 LPs, one workgroup per LP)",
            "value": total / kern, "unit": "LPs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * kern / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (device-generated splitmix64 dense LPs, seeds 5000..9095)",
            "config": {"workload": f"C5: {C5['nlp']} x ({m} x {n}) dense LPs, seed {C5['seed']} + k",
                       "parallelism": f"batch split over {world} GPU(s)",
                       "step": "one dlp_batched_solve of the whole batch",
                       "residency": ("register-resident: one lane per column slot, the slot's 65 rows in "
                                     "VGPRs (BASELINE.json says 'tableau held in LDS'; the LDS-resident kernel "
                                     "is DLP_BATCH_LDS=1, bit-identical, slower: DESIGN.md §6)")
                       if occ["register_kernel"] else "LDS-resident (one workgroup's LDS holds the tableau)"},
            "all_optimal": allopt, "pivots_per_solve": piv[-1], "pivots_per_lp": pivots_lp,
            "wall_lps_per_s": total / wall,
            "occupancy": dict(occ, cus=cus, resident_lps=resident),
            "roofline": {"bound": "latency", "unit": "pivots/s", "achieved": achieved, "peak": peak,
                         "frac": achieved / peak,
                         "model": ("peak = resident LPs (VGPR/LDS occupancy) / single-LP pivot latency; "
                                   "single-LP latency from 256 LPs one per CU"),
                         "single_lp_us_per_pivot": t1 * 1e6,
                         "batch_us_per_pivot_per_lp": resident / achieved * 1e6,
                         "hbm_frac": bytes_solve / (kern / args.steps) / 1e9 / HBM_PEAK_GBS,
                         # hardware-anchored: the VALU-issue and LDS busy fractions of the
                         # same kernel from rocprofv3 SQ counters (committed, profiles/r06o/)
                         "hardware": c5_hardware_bound(),
                         "fp64_frac": (2.0 * piv[-1] * (m + 1) * (m + n + 1) / (kern / args.steps) / 1e12
                                       / FP64_PEAK_TFS)},
            "cpu_baseline": None if (world > 1 or args.no_cpu_baseline) else c5_cpu_baseline(args.cpu_seconds),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here (before anything touches a GPU) and relay rank 0
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout, args.launch_grace))
    if args.stub_worker:
        return stub_worker(args)
    if args.workload == "c5":
        return c5_main(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import distributedlpsolver_amd as dlp
    from distributedlpsolver_amd import _lib as L

    m, n, seed, desc = WORKLOADS[args.workload]
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        obj = [dlp.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        rccl_id = obj[0]
    else:
        dist = None
        # c3r2/4/8: a 1-rank communicator, so the rank's exchange kernels run (candidate and row
        # pushes, the waits)
        rccl_id = dlp.comm_unique_id() if args.workload in RANK_WORKLOADS else None
    xsess = world > 1 or rccl_id is not None
    xopt = {"auto": getattr(L, "XCHG_DEFAULT", 0), "rccl": L.XCHG_RCCL, "peer": L.XCHG_PEER}[args.exchange]

    def barrier_sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    prob = dlp.Problem.random(m, n, seed)

    def open_session(x, rid):
        # K is fixed by the session (auto: 64 on a streaming tableau); the pivot budget
        # leaves room for the widest window and the extra pivot window
        return dlp.Session(prob, rank=rank, nranks=world, rccl_id=rid, device=local,
                           check_interval=64 * max(args.steps, args.warmup, 1), timing=args.timing,
                           nontemporal=args.nontemporal, update_variant=args.variant,
                           ld_align=args.ld_align, rows_per_block=args.rows_per_block,
                           max_pivots=64 * (args.warmup + args.steps) + args.steps + args.alt_pivots + 2,
                           log_pivots=1, defer=args.defer, lookahead=args.lookahead,
                           exchange=x if xsess else 0)

    def any_rank(flag):
        return agree_any(flag, dist, torch, "cuda")

    def configure(sess):
        if args.occupancy >= 0 or args.form >= 0:
            if sess.update_stats()[2] > 1:
                sess.set_defer_tuning(args.occupancy if args.occupancy >= 0 else 0, args.form)
        if xsess:
            # a dead rank ends the run in bounded time (its peers' waits abort), never a hang
            sess.set_exchange_timeout(60.0)

    XNAMES = {L.XCHG_RCCL: "rccl", L.XCHG_PEER: "peer"}
    sess = open_session(xopt, rccl_id)
    configure(sess)
    K = sess.update_stats()[2]
    per_step = K if args.step_unit == "block" else 1
    warm, timed = args.warmup * per_step, args.steps * per_step
    xmode = XNAMES.get(sess.get_exchange(), "none") if xsess else None
    xreason = sess.exchange_reason() if xsess and hasattr(sess, "exchange_reason") else None

    def reopen_rccl():
        obj = [dlp.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        s2 = open_session(L.XCHG_RCCL, obj[0])
        configure(s2)
        return s2, XNAMES.get(s2.get_exchange(), "none")

    fallback_ok = world > 1 and xmode == "peer" and args.exchange == "auto"
    sess, st, done, elapsed, run_fallback, xmode2 = measure_with_fallback(
        sess, warm, timed, barrier_sync, any_rank, dlp.DLPError, reopen_rccl if fallback_ok else None)
    if run_fallback:
        xmode, xreason = xmode2, run_fallback
    if done != timed:
        raise SystemExit(f"timed window ended early: status {st} after {done} pivots")
    lookahead_on = sess.lookahead()
    chain_cus = sess.chain_cus() if hasattr(sess, "chain_cus") else None
    # CUs the pass runs on (all of the device's unless the lookahead split gave the chain some of them;
    # co-located rank processes' slices are not subtracted here)
    dev_cus = torch.cuda.get_device_properties(local).multi_processor_count
    pass_cus = dev_cus - chain_cus if (lookahead_on and chain_cus) else dev_cus

    tm, nsamp = sess.timings()
    launches, upd_total_ms, _ = sess.update_stats()
    variant, rb_used, nt_used = sess.get_tuning()
    form = sess.defer_form() if K > 1 else None
    # the tableau as stored: the condensed tableau keeps the n nonbasic columns
    # + the RHS (the m basic columns are unit vectors the rule never changes)
    condensed = bool(getattr(sess, "condensed", False))
    ld_used = sess.storage_ld if condensed else sess.ld
    rows_local, N1 = sess.rows, (sess.storage_ncols if condensed else sess.ncols) + 1
    upd_ms = upd_total_ms / max(launches, 1)   # per update-kernel launch (rank-1, or rank-K pass)
    # algorithmic bytes of one launch: one read + one write of every resident element
    # (the deferred pass skips the objective row, kept current by the pivot-row kernel)
    bytes_launch = 16.0 * (rows_local + (1 if K == 1 else 0)) * N1
    achieved = bytes_launch / (upd_ms * 1e-3) / 1e9 if upd_ms > 0 else None   # timing 0: untimed
    obj_after = None

    # the same LP continues: a --step-unit pivot window of args.steps pivots beside the main
    # figure (its last pass covers a partial block), timed the same way
    pw = None
    if not args.no_pivot_window and args.step_unit == "block" and K > 1:
        barrier_sync()
        t1 = time.perf_counter()
        st, done = sess.run(args.steps)
        barrier_sync()
        pw_el = time.perf_counter() - t1
        if done == args.steps:
            pw = {"pivots": args.steps, "seconds": pw_el, "passes": -(-args.steps // K)}

    if dist is not None:
        import torch as _t
        t = _t.tensor([elapsed, pw["seconds"] if pw else 0.0], dtype=_t.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        if pw:
            pw["seconds"] = float(t[1].item())
    if pw:
        pw["pivots_per_s"] = pw["pivots"] / pw["seconds"]

    res = sess.result()
    obj_after = res.objective
    parity = log_parity(args.workload, res.pivot_log) if rank == 0 else None

    # N > 1: the same LP continues for args.alt_pivots pivots through the OTHER exchange
    # (RCCL collectives <-> owner-rooted peer stores), timed the same way, so that one
    # scaling run measures both; a failure to switch or to run is reported, not fatal
    alt = None
    if dist is not None and args.alt_pivots > 0 and K > 1 and run_fallback is None:
        alt = alt_exchange_window(sess, dist, barrier_sync, args, L, torch)
        if alt.get("pivots_per_s") and rank == 0:
            alt["pivot_log_vs_oracle"] = log_parity(args.workload, sess.result().pivot_log)
    sess.close()

    # the north star's own figure: the EAGER rank-1 update (defer = 1) on the same tableau,
    # a short window of single-pivot launches timed by HIP events on the session stream
    eager = None
    if world == 1 and not args.no_eager_window and K > 1:
        with dlp.Session(prob, device=local, check_interval=args.eager_pivots, timing=1, defer=1,
                         max_pivots=args.eager_pivots + 1, log_pivots=1) as es:
            es.run(1)   # warm-up pivot
            es.reset_timings()
            t2 = time.perf_counter()
            st, done = es.run(args.eager_pivots)
            torch.cuda.synchronize()
            e_el = time.perf_counter() - t2
            e_launch, e_ms, _ = es.update_stats()
            e_var, e_rb, e_nt = es.get_tuning()
            e_rows, e_N1 = es.rows, es.ncols + 1   # (the eager session stores the full tableau)
        e_ms1 = e_ms / max(e_launch, 1)
        e_bytes = 16.0 * (e_rows + 1) * e_N1
        e_ach = e_bytes / (e_ms1 * 1e-3) / 1e9 if e_ms1 > 0 else None
        eager = {"kernel": f"rank-1 update variant {e_var} (rows/band {e_rb}, nt {e_nt})",
                 "pivots": done, "launches": e_launch, "launch_ms": e_ms1,
                 "algorithmic_bytes_per_launch": e_bytes, "achieved": e_ach, "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "frac": e_ach / HBM_PEAK_GBS if e_ach else None,
                 "pivots_per_s": done / e_el if e_el > 0 else None}

    if rank == 0:
        kind = "update" if K == 1 else "pass"
        ksub = "update_" if K == 1 else "pass"
        geo = {"workload": args.workload, "kernel": kind, "K": K, "form": form,
               "rows_per_block": rb_used, "nontemporal": nt_used, "ld": ld_used,
               "rows_local": rows_local}
        if condensed:
            geo["condensed"] = True
        if args.pmc_dir:
            traffic, traffic_src = pmc_traffic(args.pmc_dir, ksub), f"live: {args.pmc_dir}"
        elif world == 1:
            traffic, traffic_src = committed_traffic(geo)
        else:
            traffic, traffic_src = None, None
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(m, n, seed, args.cpu_seconds, K)
        value = timed / elapsed
        line = {
            "metric": ("simplex pivots/s + achieved HBM GB/s (dense fp64 tableau; roofline of the "
                       + (f"rank-{K} tableau pass" if K > 1 else "rank-1 update") + ")"),
            "value": value,
            "unit": "pivots/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device-generated splitmix64 dense LP, seed = config id)",
            "config": {"workload": desc, "m": m, "n": n, "N": m + n, "ld": ld_used, "seed": seed,
                       "rows_per_rank": rows_local, "parallelism": f"rowblock{world}",
                       "pricing": "dantzig->bland on degeneracy", "pivots_per_tableau_pass": K,
                       "tableau": (f"condensed: {N1 - 1} nonbasic columns + RHS stored per row (the {m} basic "
                                   f"columns are unit vectors, DESIGN.md §16)" if condensed else
                                   f"full: {N1} columns per row"),
                       "step": (f"{per_step} pivots + their rank-{K} tableau pass" if per_step > 1
                                else "one pivot"),
                       "lookahead": lookahead_on},
            "pivots_timed": timed,
            "pivots_per_step": per_step,
            "K": K,
            "passes_in_window": launches,
            "achieved_hbm_gbs": achieved,
            "phases_ms_per_pivot": ({"ratio": tm[0] / max(nsamp, 1), "exchange": tm[1] / max(nsamp, 1),
                                     "prow": tm[2] / max(nsamp, 1), "update": tm[3] / max(nsamp, 1)}
                                    if args.timing >= 2 else None),
            "update_launches": launches,
            "pivot_step_window": pw,
            "exchange": xmode,
            "exchange_requested": args.exchange if xsess else None,
            "exchange_fallback_reason": xreason or None,
            # the rank's block, split (c3r8: the per-rank floor of the 8-GPU split): without
            # lookahead a block is its selection chain, then its pass, so the chain per pivot is
            # (block - pass) / K; under lookahead they overlap and only the block is measured
            "block": {"ms": 1e3 * elapsed / args.steps * (K / per_step), "pass_ms": upd_ms,
                      "chain_us_per_pivot": ((1e3 * elapsed / args.steps * (K / per_step) - upd_ms) / K * 1e3
                                             if (K > 1 and not lookahead_on and upd_ms > 0) else None),
                      "lookahead": lookahead_on, "rows_local": rows_local,
                      # lookahead: CUs of the chain's stream, the pass on the rest (0 = unmasked)
                      "chain_cus": chain_cus},
            "alt_exchange_window": alt,
            "objective_after_run": obj_after,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved else None,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "bytes_model": ("16 * rows_local * (stored columns): one read + one write of every "
                                         "stored element" + ("; condensed tableau, n + 1 columns" if condensed else
                                                             "")),
                         "kernel": (f"rank-1 update variant {variant} (rows/band {rb_used}, "
                                    f"nt {nt_used}, ld {ld_used})" if K == 1 else
                                    f"rank-{K} tableau pass, form {form} (rows/band {rb_used}, "
                                    f"nt {nt_used}, ld {ld_used}): {K} pivots per launch"),
                         "launch_ms": upd_ms,
                         # the pass is also an fp64 FMA stream (K fmas per element): its share of
                         # the measured vector fp64 peak (77.3 TF/s, profiles/r02j/lab8a.txt)
                         "fp64_tflops": (2.0 * K * rows_local * (N1 - 1) / (upd_ms * 1e-3) / 1e12
                                         if upd_ms > 0 else None),
                         "fp64_frac": (2.0 * K * rows_local * (N1 - 1) / (upd_ms * 1e-3) / 1e12 / FP64_PEAK_TFS
                                       if upd_ms > 0 else None),
                         # under lookahead's CU split the pass holds only its own CUs: its fp64 peak is their
                         # share (8 FLOP per algorithmic byte at K = 64 is above that share's ridge)
                         "pass_cus": pass_cus,
                         "fp64_frac_of_pass_cus": (2.0 * K * rows_local * (N1 - 1) / (upd_ms * 1e-3) / 1e12
                                                   / (FP64_PEAK_TFS * pass_cus / dev_cus)
                                                   if upd_ms > 0 and pass_cus else None)},
            "rank1_update_roofline": eager,
            "pivot_log_vs_oracle": parity,
            "cpu_baseline": cpu,
            "geometry": geo,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    finally:
        # pooled streams (CU-masked ones included), buffers and batch contexts released before the
        # runtime's own teardown (a rocprofv3-traced run crashed at exit without it, profiles/r06i/)
        if "distributedlpsolver_amd" in sys.modules and os.environ.get("DLP_BENCH_LAUNCHER") != "parent":
            try:
                sys.modules["distributedlpsolver_amd"].release_cached_memory(-1)
            except Exception:  # noqa: BLE001 - best effort at exit
                pass
