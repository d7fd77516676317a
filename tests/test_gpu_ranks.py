"""GPU: the per-process rank path of a scaling run, with a second rank.

`bench.py --gpus N` runs one process per GPU; each is a rank session of a streaming LP
with the shipped defaults: K = 64, lookahead auto (on once the peer exchange is
connected), the chain / pass CU split (128 chain CUs at 4,096 local rows), the form-21
pass with band publication, and the two-launch peer pivot (workgroup 0 of the ratio
launch and every pivot-row workgroup of a non-owner wait on ANOTHER PROCESS's stores).
Here two such processes share one MI355X: bench.py's c3r4 LP (8192 x 57344, seed 34) is
split into 2 x 4,096 rows, so each rank holds 4,096 x 65,537 — exactly one rank of C3's
8-GPU split.  The exchange blocks are opened through IPC handles gathered over gloo
(RCCL cannot join two ranks on one device; the RCCL fallback is covered by injection,
tests/test_gpu_peer.py, tests/test_bench_fallback.py).

Every process checks its own output against the oracle's committed stops
(tests/golden/make_digests.py rank_split): the pivot log, basis and objective
(replicated on every rank), its row block's whole-tableau digest and the objective row.
Reference analog of the split: R/global_problem.cpp:270-274."""
import hashlib
import os
import socket

import numpy as np
import pytest

from conftest import load_golden

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _block_sha(s, width, chunk=512):
    """sha256 of this rank's constraint rows, first `width` doubles each, in row order
    (the stream make_digests.tableau_sha hashes for the oracle's row block)."""
    h = hashlib.sha256()
    for first in range(0, s.rows, chunk):
        cnt = min(chunk, s.rows - first)
        h.update(np.ascontiguousarray(s.read_rows(first, cnt)[:, :width]).tobytes())
    return h.hexdigest()


def _want_block(want, world, rank):
    """The oracle's digest of this rank's row block at one stop (entries with several splits keep
    them under "blocks", keyed by the rank count)."""
    return want["blocks"][str(world)][rank] if "blocks" in want else want["block_sha256"][rank]


def _rank_worker(rank, world, port, g, windows, env, q):
    """One process = one rank session, driven exactly as bench.py drives it (dlp_session_run
    windows on its own stream), checked against the oracle's stops after each window."""
    import torch.distributed as dist
    os.environ.update(env)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank, "checks": {}}
    s = None
    try:
        la = int(env.get("LOOKAHEAD", "-1"))
        s = dlp.Session(dlp.Problem.random(g["m"], g["n"], g["seed"]), rank=rank, nranks=world,
                        defer=0, lookahead=la, check_interval=64 * 20, log_pivots=1,
                        max_pivots=sum(windows) + 2)
        # the records carry each rank's device (PCI bus id), so the library sees that the ranks
        # share this GPU and gives each chain a CU slice of its own (chain_cus_policy)
        hs = [None] * world
        dist.all_gather_object(hs, s.exchange_record())
        s.connect_records(hs)
        s.set_exchange_timeout(60.0)
        out["config"] = {"exchange": s.get_exchange(), "lookahead": s.lookahead(),
                         "chain_cus": s.chain_cus(), "colocated": s.colocated(),
                         "defer_tuning": s.get_defer_tuning(),
                         "rows": s.rows, "row_first": s.row_first, "ld": s.ld}
        dist.barrier()
        total = 0
        for w in windows:
            st, done = s.run(w)
            total += done
            out.setdefault("runs", []).append((st, done))
            want = g["stops"].get(str(total))
            if want is None:
                continue
            res = s.result()
            got = {"log": _sha(res.pivot_log) == want["log_sha256"],
                   "basis": _sha(res.basis) == want["basis_sha256"],
                   "objective": float(res.objective).hex() == want["objective_hex"],
                   "block": _block_sha(s, g["width"]) == _want_block(want, world, rank),
                   "objective_row": _sha(s.read_rows(s.rows, 1)[0, :g["width"]]) == want["objective_row_sha256"]}
            out["checks"][str(total)] = got
        # no rank frees its exchange block while a peer's kernels may still store into it
        dist.barrier()
        s.close()
        s = None
    except Exception as e:   # reported to the parent, which fails the test
        out["error"] = repr(e)
    finally:
        q.put(out)
        if s is not None:
            s.abort()
        dist.destroy_process_group()


def _run_two(windows, env, timeout=240, key="rank_split", world=None):
    import torch.multiprocessing as mp
    g = load_golden("digests.json")[key]
    world = world or g["P"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, g, windows, env, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = sorted((q.get(timeout=timeout) for _ in procs), key=lambda o: o["rank"])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    for o in out:
        assert "error" not in o, o
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return g, out


@pytest.mark.parametrize("case", ["default", "chain_cus_0", "no_lookahead", "ratio64"])
def test_two_process_rank_path(case):
    """default: the shipped auto policy (K = 64, lookahead on with the peer exchange, the 128
    chain CUs of a 4,096-row rank split into two disjoint 64-CU slices because both processes
    share this GPU, form 21 + band publication, two-launch peer pivot), 136 pivots (two full
    blocks + 8) then a 64-pivot window that ends inside a block (200), then 64 more (264);
    chain_cus_0: DLP_CHAIN_CUS=0 (chain and pass unmasked); no_lookahead: lookahead = 0
    (the form-23 LDS-ring pass in place); ratio64: 64-lane ratio workgroups (65 candidate slots
    per rank in the peer exchange instead of 17)."""
    env = {"chain_cus_0": {"DLP_CHAIN_CUS": "0"}, "no_lookahead": {"LOOKAHEAD": "0"},
           "ratio64": {"DLP_RATIO_THREADS": "64"}}.get(case, {})
    windows = [136, 64, 64] if case == "default" else [136]
    g, out = _run_two(windows, env)
    for o in out:
        cfg = o["config"]
        assert cfg["exchange"] == L.XCHG_PEER and cfg["colocated"] == (2, o["rank"])
        assert cfg["rows"] == g["m"] // g["P"] and cfg["row_first"] == o["rank"] * g["m"] // g["P"]
        assert cfg["defer_tuning"][2] == 64
        if case == "no_lookahead":
            assert not cfg["lookahead"] and cfg["defer_tuning"][1] == 23
        else:
            assert cfg["lookahead"] and cfg["defer_tuning"][1] == 21
            assert cfg["chain_cus"] == (0 if case == "chain_cus_0" else 64)
        assert [d for _, d in o["runs"]] == windows
        assert set(o["checks"]) == {str(k) for k in np.cumsum(windows)}
        for k, got in o["checks"].items():
            assert all(got.values()), (o["rank"], k, got)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_c3_rank_processes(world):
    """The rank geometries of the N = 2, 4 and 8 scaling runs, each rank its own process on this
    one GPU: C3 itself (32,768 x 32,768 seed 3, bench.py's default LP) split into 2 x 16,384 rows
    (the auto policy: 64 chain CUs, 256-lane ratio workgroups, the form-23 pass on the other CUs),
    4 x 8,192 (128-lane ratio workgroups, form 23, the register pivot-row kernel of a chain on CUs
    of its own) or 8 x 4,096 (the same with the form-21 pass), with lookahead and the two-launch
    peer pivot; 136 pivots (two full blocks + 8; N = 2: then 64 more, ending inside a block)
    against the oracle's stops (tests/golden/make_digests.py rank_split_c3); world 3 is a ragged
    split (10,922 / 10,923 / 10,923 rows).
    All processes share this one GPU, under the default environment: the library learns that from
    the exchange records (each rank's PCI bus id) and gives each rank's chain a disjoint CU slice
    of its budget (2 x 32 of 64 at P = 2, 4 x 32 of 128 at P = 4), or no masks where a slice would
    be under 32 CUs (P = 3: 64 / 3, P = 8: 128 / 8).  With one shared mask the spinning chain
    workgroups of the waiting ranks filled those CUs and starved the owner's (3+ processes,
    profiles/r05w/); on N GPUs each rank is alone on its device and keeps the whole budget."""
    windows = [136, 64] if world == 2 else [136]
    g, out = _run_two(windows, {}, timeout=420, key="rank_split_c3", world=world)
    want_cus = {2: 32, 3: 0, 4: 32, 8: 0}[world]
    for o in out:
        cfg = o["config"]
        first, last = o["rank"] * g["m"] // world, (o["rank"] + 1) * g["m"] // world
        assert cfg["exchange"] == L.XCHG_PEER and cfg["lookahead"]
        assert cfg["colocated"] == (world, o["rank"])
        assert cfg["rows"] == last - first and cfg["row_first"] == first
        assert cfg["chain_cus"] == want_cus
        assert cfg["defer_tuning"][1:] == (23 if (want_cus > 0 and cfg["rows"] > 4096) else 21, 64)
        assert [d for _, d in o["runs"]] == windows
        assert set(o["checks"]) == {str(k) for k in np.cumsum(windows)}
        for k, got in o["checks"].items():
            assert all(got.values()), (o["rank"], k, got)


def _split_sha(s, width, cut, chunk=512):
    """Digests of rows [0, cut) and [cut, rows) of a one-session tableau: the two rank blocks of
    the rank_split stops."""
    out = []
    for a, b in ((0, cut), (cut, s.rows)):
        h = hashlib.sha256()
        for first in range(a, b, chunk):
            cnt = min(chunk, b - first)
            h.update(np.ascontiguousarray(s.read_rows(first, cnt)[:, :width]).tobytes())
        out.append(h.hexdigest())
    return out


def test_rccl_rank_session_lookahead_on_cu_split():
    """an RCCL-exchange rank session keeps lookahead when the chain has CUs of its
    own (the collectives never share a CU with the pass): the rank_split LP as one 1-rank RCCL
    session (8,192 rows: 96 chain CUs, form 23 on the rest), 136 + 64 pivots against the
    oracle's stops (both row blocks, objective row, log, basis)."""
    g = load_golden("digests.json")["rank_split"]
    with dlp.Session(dlp.Problem.random(g["m"], g["n"], g["seed"]), rank=0, nranks=1,
                     rccl_id=dlp.comm_unique_id(), exchange=L.XCHG_RCCL, defer=0, check_interval=64 * 20,
                     max_pivots=300) as s:
        assert s.get_exchange() == L.XCHG_RCCL
        assert s.lookahead() and s.chain_cus() == 96 and s.get_defer_tuning()[1:] == (23, 64)
        total = 0
        for w in (136, 64):
            st, done = s.run(w)
            total += done
            want = g["stops"][str(total)]
            res = s.result()
            assert _sha(res.pivot_log) == want["log_sha256"]
            assert _sha(res.basis) == want["basis_sha256"]
            assert float(res.objective).hex() == want["objective_hex"]
            assert _split_sha(s, g["width"], g["m"] // 2) == want["block_sha256"]
            assert _sha(s.read_rows(s.rows, 1)[0, :g["width"]]) == want["objective_row_sha256"]


def _stall_worker(rank, world, port, g, q):
    """Rank 0 runs two windows; rank 1 runs only the first and then stops taking part (it stays
    alive, so its exchange block stays mapped).  Rank 0's device waits in the second window end at
    its exchange timeout + 5 s through the abort word; the run returns DLP_ERR_RCCL."""
    import time as _t
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank}
    s = None
    try:
        s = dlp.Session(dlp.Problem.random(g["m"], g["n"], g["seed"]), rank=rank, nranks=world, defer=0,
                        check_interval=64, max_pivots=400)
        hs = [None] * world
        dist.all_gather_object(hs, s.exchange_handle())
        s.connect_ipc(hs)
        s.set_exchange_timeout(3.0)
        dist.barrier()
        out["first"] = s.run(136)
        if rank == 0:
            t0 = _t.time()
            try:
                s.run(64)
                out["second"] = "completed"
            except L.DLPError as e:
                out["second"] = (e.status, str(e))
            out["seconds"] = _t.time() - t0
        s.abort()                 # every rank: no device wait outlives the test
        import torch
        torch.cuda.synchronize()
        dist.barrier()            # both streams drained before either block is freed
        s.close()
        s = None
    except Exception as e:   # reported to the parent
        out["error"] = repr(e)
    finally:
        q.put(out)
        dist.destroy_process_group()


def test_two_process_rank_stall_is_bounded():
    """Failure containment across processes at the shipped geometry: a rank
    that stops taking part mid-solve ends its peer's run with DLP_ERR_RCCL in bounded time, not a
    hang; both processes then abort, drain and free their blocks cleanly."""
    import torch.multiprocessing as mp
    g = load_golden("digests.json")["rank_split"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stall_worker, args=(r, 2, port, g, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted((q.get(timeout=240) for _ in procs), key=lambda o: o["rank"])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    for o in out:
        assert "error" not in o, o
        assert o["first"] == (L.RUNNING, 136) or o["first"][1] == 136, o
    st, msg = out[0]["second"]
    assert st == L.ERR_RCCL, out[0]
    assert out[0]["seconds"] < 60, out[0]
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
