"""CPU checks of bench.py's host-side pieces (no GPU): the CPU-baseline leg
(the oracle on a bounded sample, all usable threads then 1 thread) and the
committed-PMC lookup, so that a bench run on the box cannot die in them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_cpu_baseline_small():
    cb = bench.cpu_baseline(1500, 1500, 3, 0.2)
    assert cb["unit"] == "pivots/s" and cb["kind"] == "port"
    assert cb["value"] > 0 and cb["single_thread"]["value"] > 0
    assert cb["cores"] >= 1 and cb["single_thread"]["cores"] == 1
    assert cb["cpu_model"] and cb["nproc"] >= 1 and cb["cpus_usable"] >= 1


def test_cpu_baseline_like_for_like():
    """The deferred rank-K leg (the GPU's algorithm on the host): whole blocks, labelled."""
    cb = bench.cpu_baseline(1500, 1500, 3, 0.2, K=16)
    lf = cb["like_for_like"]
    assert lf["unit"] == "pivots/s" and lf["value"] > 0 and lf["cores"] == cb["cores"]
    assert "deferred rank-16" in lf["algorithm"]


def test_committed_traffic_unknown_geometry():
    val, src = bench.committed_traffic({"workload": "none", "kernel": "pass", "K": -1})
    assert val is None and src is None


def test_committed_traffic_for_the_default_bench_geometry():
    """The default bench (C3, K = 32, form 4) finds its committed PMC summary, and
    profiles/ travels to the GPU box (bench.py reads it there)."""
    geo = {"workload": "c3", "kernel": "pass", "K": 32, "form": 4, "rows_per_block": 256,
           "nontemporal": 1, "ld": 66048, "rows_local": 32768}
    val, src = bench.committed_traffic(geo)
    assert val and 3.0e10 < val < 4.5e10 and src.startswith("profiles/")
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        pats = [line.strip() for line in f if line.strip()]
    assert not any(p.strip("./").startswith("profiles") for p in pats)
