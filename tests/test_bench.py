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


def test_committed_traffic_unknown_geometry():
    val, src = bench.committed_traffic({"workload": "none", "kernel": "pass", "K": -1})
    assert val is None and src is None
