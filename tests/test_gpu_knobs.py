"""Every A/B tuning knob of INTEGRATION.md §4 gives the same bits as the default path.

The knobs are read once per process, so each setting runs in a child process (`_knob_run.py`
below, through the C ABI) and prints digests of what it computed: the pivot log, the objective,
the basis and — for the deferred sessions — the whole tableau.  The default run of the same
workload is the reference (it is itself checked against the oracle by the parity tests:
`test_gpu_large.py`, `test_gpu_lookahead.py`, `test_gpu_cluster.py`, `test_c5_full_batch`)."""
import functools
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

SCRIPT = r"""
import hashlib, json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import distributedlpsolver_amd as dlp

def h(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

kind = sys.argv[2]
out = {}
if kind == "defer":   # one rank of C3 at P = 8 (2.15 GB) or P = 4 (4.3 GB): K = 64, lookahead or not
    la = int(sys.argv[3])
    m, n, seed = (4096, 61440, 38) if len(sys.argv) < 5 else (8192, 57344, 34)
    with dlp.Session(dlp.Problem.random(m, n, seed), check_interval=64, lookahead=la,
                     max_pivots=200) as s:
        out["lookahead"], out["form"], out["chain_cus"] = s.lookahead(), s.defer_form(), s.chain_cus()
        out["condensed"] = s.condensed
        st, done = s.run(136)   # two full blocks and a partial one
        r = s.result()
        out.update(done=done, log=h(r.pivot_log), obj=float(r.objective).hex(), basis=h(r.basis),
                   tableau=h(s.tableau()))
elif kind == "batched":
    r = dlp.batched_solve(512, 64, 128, 5000, want_basis=True, log_cap=256)
    out.update(obj=h(r.objective), st=h(r.status), np=h(r.num_pivots), basis=h(r.basis), logs=h(r.logs))
elif kind == "cluster":
    p = dlp.Problem.random(300, 500, 11)
    with dlp.Session(p, small_lp=1) as s:
        out["small_lp"] = s.small_lp()
        s.run(10 ** 6)
        r = s.result()
    out.update(log=h(r.pivot_log), obj=float(r.objective).hex(), x=h(r.x), y=h(r.y))
print(json.dumps(out))
"""


def _run(kind, args=(), env=None):
    e = dict(os.environ)
    for k in ("DLP_LEAN_LCH", "DLP_Q_DEPTH", "DLP_BATCH_LDS", "DLP_CLUSTER_WG", "DLP_BAND_PUB", "DLP_CHAIN_CUS",
              "DLP_FAT_PROW", "DLP_TEST_MASK_FAIL", "DLP_CONDENSED", "DLP_Q_U", "DLP_RATIO_ROWS", "DLP_CHAIN_RING",
              "DLP_RATIO_THREADS", "DLP_PASS_LDS", "DLP_PROW_GROUP", "DLP_RATIO_RP"):
        e.pop(k, None)
    e.update(env or {})
    p = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, kind, *map(str, args)], env=e,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@functools.lru_cache(maxsize=None)
def _ref(kind, *args):
    return _run(kind, args)


@pytest.mark.parametrize("env", [{"DLP_LEAN_LCH": "4"}, {"DLP_LEAN_LCH": "8"}, {"DLP_BAND_PUB": "0"},
                                 {"DLP_CHAIN_CUS": "0"}, {"DLP_CHAIN_CUS": "32"}, {"DLP_CHAIN_CUS": "200"},
                                 {"DLP_FAT_PROW": "0"}, {"DLP_RATIO_THREADS": "64"},
                                 {"DLP_RATIO_THREADS": "128"}, {"DLP_RATIO_THREADS": "256"},
                                 {"DLP_CHAIN_RING": "16"}, {"DLP_CHAIN_RING": "16", "DLP_FAT_PROW": "0"},
                                 {"DLP_PROW_GROUP": "4"}, {"DLP_PROW_GROUP": "4", "DLP_RATIO_ROWS": "16"},
                                 {"DLP_RATIO_ROWS": "64", "DLP_RATIO_RP": "12"}])
def test_lookahead_chain_knobs(env):
    ref = _ref("defer", 1)
    # 4,096 rows, condensed, alone on the device: the chain on 96 CUs, the pass on the other 160 (chain_cus_policy)
    assert ref["lookahead"] and ref["form"] == 21 and ref["done"] == 136 and ref["chain_cus"] == 96
    got = _run("defer", [1], env)
    if "DLP_CHAIN_CUS" in env:
        assert got.pop("chain_cus") == int(env["DLP_CHAIN_CUS"])
        ref = {k: v for k, v in ref.items() if k != "chain_cus"}
    assert got == ref


@pytest.mark.parametrize("la", [0, 1])
def test_full_tableau_knob(la):
    """DLP_CONDENSED=0: the full tableau (every basic column stored) instead of the condensed one
     — the same pivot log, objective, basis and whole tableau (read back in the full
    layout), with lookahead (the restart replays in the LEAN chain kernels) and without."""
    ref = _ref("defer", la)
    assert ref["condensed"]
    got = _run("defer", [la], {"DLP_CONDENSED": "0"})
    assert got.pop("condensed") is False
    # (the chain's CU budget follows the layout: 96 condensed, 128 full at 4,096 rows; the bits do not)
    got.pop("chain_cus")
    assert got == {k: v for k, v in ref.items() if k not in ("condensed", "chain_cus")}


def test_cu_split_with_the_form23_pass():
    """8,192 rows (one rank of C3 at P = 4): the chain on 96 CUs and the LDS-ring pass (form 23)
    on the rest, against both streams unmasked with the form-21 pass: the same bits."""
    ref = _run("defer", [1, "p4"])
    assert ref["lookahead"] and ref["form"] == 23 and ref["chain_cus"] == 96
    got = _run("defer", [1, "p4"], {"DLP_CHAIN_CUS": "0"})
    assert got.pop("form") == 21 and got.pop("chain_cus") == 0
    assert got == {k: v for k, v in ref.items() if k not in ("form", "chain_cus")}


def test_cu_split_falls_back_to_unmasked_streams():
    """Where CU-masked queues cannot be created the lookahead runs on unmasked streams (form 21), the
    same bits."""
    ref = _run("defer", [1, "p4"])
    got = _run("defer", [1, "p4"], {"DLP_TEST_MASK_FAIL": "1"})
    assert got.pop("chain_cus") == 0 and got.pop("form") == 21 and got["lookahead"]
    assert got == {k: v for k, v in ref.items() if k not in ("form", "chain_cus")}


@pytest.mark.parametrize("n", ["64", "128", "256"])
def test_ratio_threads_without_lookahead(n):
    """Smaller deferred ratio workgroups (more of them, one lane per row) on the non-lookahead path."""
    assert _run("defer", [0], {"DLP_RATIO_THREADS": n}) == _ref("defer", 0)


@pytest.mark.parametrize("depth", ["2", "3", "6", "8"])
def test_form23_ring_depth(depth):
    ref = _ref("defer", 0)
    assert not ref["lookahead"] and ref["form"] == 23 and ref["chain_cus"] == 0
    assert _run("defer", [0], {"DLP_Q_DEPTH": depth}) == ref


@pytest.mark.parametrize("env", [{"DLP_Q_U": "2"}, {"DLP_Q_U": "4"}, {"DLP_Q_U": "4", "DLP_Q_DEPTH": "3"}])
def test_form23_rows_per_group(env):
    """The LDS-ring pass with 2 or 4 rows per group (2 / 3 groups in flight): the same bits, alone (no
    lookahead) and on the lookahead's CU split at 8,192 rows."""
    assert _run("defer", [0], env) == _ref("defer", 0)
    ref = _ref("defer", 1, "p4")
    assert ref["form"] == 23 and ref["chain_cus"] == 96
    assert _run("defer", [1, "p4"], env) == ref


@pytest.mark.parametrize("rows", ["0", "16", "32", "64"])
def test_ratio_ring_rows(rows):
    """The selection kernel of a chain on CUs of its own: the LEAN ring (0) or the grouped ring with 16 /
    32 / 64 rows per wave (ratio_ring_kernel, 512 / 256 / 128 lanes per 128-row workgroup): the same
    bits (4,096 rows: the chain on 96 CUs)."""
    ref = _ref("defer", 1)
    assert ref["chain_cus"] == 96
    assert _run("defer", [1], {"DLP_RATIO_ROWS": rows}) == ref


@pytest.mark.parametrize("env", [{"DLP_PASS_LDS": "57344"}, {"DLP_PASS_LDS": "57344", "DLP_Q_DEPTH": "6"}])
def test_pass_lds_cap(env):
    """Pass workgroups held to 2 per CU by their LDS (the chain beside them keeps the rest): same bits,
    without lookahead (form 23) and with it (form 21 beside the chain)."""
    assert _run("defer", [0], env) == _ref("defer", 0)
    assert _run("defer", [1], env) == _ref("defer", 1)


def test_batched_lds_kernel_knob():
    assert _run("batched", env={"DLP_BATCH_LDS": "1"}) == _ref("batched")


@pytest.mark.parametrize("wg", ["16", "64"])   # slices of 51 / 13 columns fit the LDS
def test_cluster_workgroup_knob(wg):
    ref = _ref("cluster")
    assert ref["small_lp"]
    assert _run("cluster", env={"DLP_CLUSTER_WG": wg}) == ref

