#!/usr/bin/env python3
"""Benchmark: simplex pivots/s + achieved HBM GB/s of the rank-1 update on a
dense fp64 tableau (BASELINE.json metric), 1/2/4/8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2]

A "step" is one simplex pivot (pricing + ratio test + pivot-row exchange +
rank-1 elimination) of ONE LP whose tableau is resident in HBM, row-block
partitioned over the N ranks (launched by torch.distributed.run for N > 1,
one process per GPU, exchange over RCCL inside libdlp).  The LP is fixed as N
grows, so scaling is strong.  Default workload C3: m = n = 32768 (N = 65536,
17.2 GB tableau), generated on the device (synthetic, seed 3 = config id).

Rank 0 prints ONE JSON line.  The roofline object prices the update kernel:
algorithmic bytes per launch = 16 (m_local + 1)(N + 1) (one read + one write of
every resident tableau element) over its mean launch time from
HIP events on the session stream.  cpu_baseline (rank 0, N = 1 only) is the
in-repo CPU oracle (same pivot rule) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: (m, n, seed, description)
    "c3": (32768, 32768, 3, "C3 dense LP 32768 x 32768 (+32768 slack): fp64 tableau 32769 x 65537, "
                            "row-block over the GPUs"),
    "c2": (4096, 4096, 2, "C2 dense LP 4096 x 4096 (+4096 slack): fp64 tableau 4097 x 8193"),
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults are whole deferred blocks (K = 32 at C3): a window that ends mid-block pays a
    # full tableau pass for its last few pivots (run() leaves the tableau current), so a
    # 200-pivot window measures 7 passes for 6.25 blocks of work
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-pivots", type=int, default=60)
    ap.add_argument("--cpu-threads", type=int, default=16)
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
    ap.add_argument("--pmc-dir", default=None,
                    help="rocprofv3 --pmc output dir (FETCH_SIZE / WRITE_SIZE) to fill roofline.traffic")
    return ap.parse_args()


def pmc_traffic(pmc_dir: str, kernel_substr: str = "update_"):
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


def committed_traffic(workload: str, kernel: str):
    """Latest committed PMC summary for this workload and kernel
    (profiles/*/<workload>_<kernel>_pmc_traffic.json, kernel = update | pass), produced by
    tools/gpu_profile.sh + tools/pmc_summary.py on the same kernel; None when absent."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"{workload}_{kernel}_pmc_traffic.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        d = json.load(f)
    return d.get("traffic_bytes_per_launch"), os.path.relpath(paths[-1], ROOT)


def cpu_baseline(m, n, seed, k, threads):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py  # test infrastructure: the CPU comparator only
    secs, done, gen = oracle_py.bench_pivots(m, n, seed, 1, k, threads)
    return {"value": done / secs, "unit": "pivots/s", "cores": threads, "kind": "port",
            "sample": f"in-repo C++ oracle (same pivot rule, OpenMP over rows), same LP "
                      f"{m}x{n} seed {seed}: 1 warm-up + {done} timed pivots in {secs:.2f} s "
                      f"(host tableau generation {gen:.1f} s not timed)"}


def defer_of(sess) -> int:
    return sess.update_stats()[2]


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import distributedlpsolver_amd as dlp

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
        rccl_id = None

    def barrier_sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    sess = dlp.Session(dlp.Problem.random(m, n, seed), rank=rank, nranks=world, rccl_id=rccl_id,
                       device=local, check_interval=max(args.steps, args.warmup, 1),
                       timing=args.timing, nontemporal=args.nontemporal,
                       update_variant=args.variant, ld_align=args.ld_align,
                       rows_per_block=args.rows_per_block, max_pivots=args.warmup + args.steps + 1,
                       log_pivots=1, defer=args.defer)
    if args.occupancy >= 0 or args.form >= 0:
        if defer_of(sess) > 1:
            sess.set_defer_tuning(args.occupancy if args.occupancy >= 0 else 0, args.form)
    st, done = sess.run(args.warmup)
    if done != args.warmup:
        raise SystemExit(f"warm-up ended early: status {st} after {done} pivots")
    sess.reset_timings()

    barrier_sync()
    t0 = time.perf_counter()
    st, done = sess.run(args.steps)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if done != args.steps:
        raise SystemExit(f"timed window ended early: status {st} after {done} pivots")

    tm, nsamp = sess.timings()
    launches, upd_total_ms, defer = sess.update_stats()
    variant, rb_used, nt_used = sess.get_tuning()
    ld_used = sess.ld
    rows_local, N1 = sess.rows, sess.ncols + 1
    upd_ms = upd_total_ms / max(launches, 1)   # per update-kernel launch (rank-1, or rank-k pass)
    # algorithmic bytes of one launch: one read + one write of every resident element
    # (the deferred pass skips the objective row, kept current by the pivot-row kernel)
    bytes_launch = 16.0 * (rows_local + (1 if defer == 1 else 0)) * N1
    achieved = bytes_launch / (upd_ms * 1e-3) / 1e9 if upd_ms > 0 else None   # timing 0: untimed

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    res = sess.result()
    sess.close()

    if rank == 0:
        ksub = "update_" if defer == 1 else "pass"
        if args.pmc_dir:
            traffic, traffic_src = pmc_traffic(args.pmc_dir, ksub), f"live: {args.pmc_dir}"
        else:
            traffic, traffic_src = (committed_traffic(args.workload, "update" if defer == 1 else "pass")
                                    if world == 1 else (None, None))
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(m, n, seed, args.cpu_pivots, args.cpu_threads)
        value = args.steps / elapsed
        line = {
            "metric": "simplex pivots/s (dense fp64 tableau, rank-1 update HBM roofline)",
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
            "config": {"workload": desc, "m": m, "n": n, "N": m + n, "ld": ld_used, "seed": seed, "rows_per_rank": rows_local,
                       "parallelism": f"rowblock{world}", "pricing": "dantzig->bland on degeneracy",
                       "pivots_per_tableau_pass": defer},
            "achieved_hbm_gbs": achieved,
            "phases_ms_per_pivot": ({"ratio": tm[0] / max(nsamp, 1), "exchange": tm[1] / max(nsamp, 1),
                                     "prow": tm[2] / max(nsamp, 1), "update": tm[3] / max(nsamp, 1)}
                                    if args.timing >= 2 else None),
            "update_launches": launches,
            "objective_after_window": res.objective,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved else None,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "kernel": (f"rank-1 update variant {variant} (rows/band {rb_used}, "
                                    f"nt {nt_used}, ld {ld_used})" if defer == 1 else
                                    f"rank-{defer} tableau pass pass_s_kernel (rows/band {rb_used}, "
                                    f"nt {nt_used}, ld {ld_used}): {defer} pivots per launch"),
                         "launch_ms": upd_ms},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
