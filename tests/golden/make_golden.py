"""Regenerate the committed golden fixtures (run in the BUILD container only).

    python tests/golden/make_golden.py

Sources of truth:
  * scipy 1.15.3 HiGHS (``linprog(method='highs')``) for objective / x / y of
    every fixture LP — an independent solver, never shipped to the GPU box;
  * the reference itself, built from its own sources by ``make -C oracle ref``
    (oracle/_ref/dlp_ref, hard-coded to its default 1000x1000x0.1 scenario,
    R/main.cpp:19-38): its stdout degrees pin the ad-allocation generator
    restatement and its per-iteration MW "Dual Value" (an upper bound on OPT)
    is recorded beside the exact OPT;
  * known-answer LPs restated from scipy's own test-suite
    (scipy/optimize/tests/test_linprog.py: Beale cycling example :1043-1064,
    Klee-Minty :1031-1041).
The oracle (tests/oracle_py.py) is used only to materialise the generated
instances (its generator spec is what the fixtures pin) and to record its
own pivot-sequence digests as regression goldens.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import subprocess
import sys

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as O  # noqa: E402


def highs(A, b, c):
    r = linprog(-np.asarray(c), A_ub=A, b_ub=b, bounds=(0, None), method="highs")
    assert r.status == 0, r.message
    return dict(objective=float(-r.fun), x=[float(v) for v in r.x],
                y=[float(-v) for v in r.ineqlin.marginals])


def log_digest(log) -> str:
    return hashlib.sha256(np.ascontiguousarray(log).tobytes()).hexdigest()


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1)
    print("wrote", name)


def kats():
    beale = dict(name="beale_cycling",
                 source="scipy/optimize/tests/test_linprog.py:1043-1064 (min form; c negated here)",
                 A=[[0.5, -5.5, -2.5, 9.0], [0.5, -1.5, -0.5, 1.0], [1.0, 0.0, 0.0, 0.0]],
                 b=[0.0, 0.0, 1.0], c=[10.0, -57.0, -9.0, -24.0],
                 expected_x=[1.0, 0.0, 1.0, 0.0], expected_objective=1.0)
    klee = dict(name="klee_minty_3",
                source="scipy/optimize/tests/test_linprog.py:1031-1041",
                A=[[1.0, 0.0, 0.0], [20.0, 1.0, 0.0], [200.0, 20.0, 1.0]],
                b=[1.0, 100.0, 10000.0], c=[100.0, 10.0, 1.0],
                expected_x=[0.0, 0.0, 10000.0], expected_objective=10000.0)
    # Unbounded: max x1 s.t. -x1 + x2 <= 1 (x1 unbounded above).
    unb = dict(name="unbounded_2", source="build KAT", A=[[-1.0, 1.0]], b=[1.0], c=[1.0, 0.0],
               expected_status=2)
    # Optimal at the start (c <= 0): zero pivots.
    opt0 = dict(name="optimal_at_start", source="build KAT", A=[[1.0, 2.0], [3.0, 1.0]],
                b=[4.0, 5.0], c=[-1.0, -2.0], expected_status=0, expected_objective=0.0,
                expected_pivots=0)
    out = []
    for k in (beale, klee, unb, opt0):
        for pricing in (0, 1):
            s = O.solve_dense(np.array(k["A"]), np.array(k["b"]), np.array(k["c"]), pricing=pricing)
            k[f"oracle_pivots_pricing{pricing}"] = int(s.num_pivots)
            k[f"oracle_log_pricing{pricing}"] = [[int(e["q"]), int(e["p"]), int(e["leaving"]),
                                                  float(e["ratio"]), float(e["objective"])]
                                                 for e in s.pivot_log]
        if "expected_status" not in k or k["expected_status"] == 0:
            if k["name"] != "optimal_at_start":
                k["highs"] = highs(np.array(k["A"]), np.array(k["b"]), np.array(k["c"]))
        out.append(k)
    dump("kat.json", out)


def generated():
    cases = [
        dict(name="c1_dense_200x400_s1", m=200, n=400, seed=1, degenerate=False),
        dict(name="c1_dense_200x400_s2", m=200, n=400, seed=2, degenerate=False),
        dict(name="dense_64x64_s7", m=64, n=64, seed=7, degenerate=False),
        dict(name="c4_degen_64x64_s5", m=64, n=64, seed=5, degenerate=True),
        dict(name="c4_degen_128x128_s3", m=128, n=128, seed=3, degenerate=True),
        dict(name="c4_degen_256x512_s4", m=256, n=512, seed=4, degenerate=True),
    ]
    out = []
    for cs in cases:
        A, b, c = O.gen_dense(cs["m"], cs["n"], cs["seed"], cs["degenerate"])
        cs["gen_head"] = dict(A00_07=[float(v) for v in A[0, :8]], b0_3=[float(v) for v in b[:4]],
                              c0_3=[float(v) for v in c[:4]],
                              b_sum=float(np.sum(b)), A_sum=float(np.sum(A)))
        cs["highs"] = highs(A, b, c)
        s = O.solve_dense(A, b, c)
        cs["oracle"] = dict(status=int(s.status), objective=float(s.objective),
                            pivots=int(s.num_pivots), log_sha256=log_digest(s.pivot_log),
                            degenerate_pivots=int((s.pivot_log["ratio"] == 0).sum()))
        out.append(cs)
    dump("generated.json", out)


def adalloc():
    out = []
    for (A, I) in [(2, 10), (100, 100), (200, 200), (1000, 1000)]:
        sp = 0.5 if (A, I) == (2, 10) else 0.1
        g = O.gen_adalloc(A, I, sp, 0.25)
        M, b, c = O.adalloc_lp(A, I, sp, 0.25)
        h = highs(M, b, c)
        rec = dict(A=A, I=I, sparsity=sp, scaling=0.25, nnz=int(len(c)),
                   draws_per_advertiser=sorted(set(int(d) for d in g["draws"])),
                   budget=float(g["budgets"][0]), max_bid=g["max_bid"],
                   bids_sha256=hashlib.sha256(g["bid"].tobytes()).hexdigest(),
                   highs_objective=h["objective"])
        if A * I <= 40000:
            rec["highs_x"] = h["x"]
        out.append(rec)
    dump("adalloc.json", out)


def reference_run():
    ref = os.path.join(ROOT, "oracle", "_ref", "dlp_ref")
    if not os.path.exists(ref):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "ref"])
    txt = subprocess.run([ref], capture_output=True, text=True, cwd="/tmp", check=True).stdout
    adv = [int(v) for v in re.findall(r"Advertiser \d+ degree is (\d+)", txt)]
    imp = [int(v) for v in re.findall(r"Impression \d+ degree is (\d+)", txt)]
    dual = [float(v) for v in re.findall(r"Dual Value = (\S+)", txt)]
    dump("ref_adalloc_1000.json", dict(
        source="oracle/_ref/dlp_ref = reference built by `make -C oracle ref` "
               "(R/main.cpp:19-38 default scenario: A=I=1000, sparsity 0.1, scaling 0.25, "
               "300 MW iterations, binary search mode)",
        advertiser_degrees=adv, impression_degrees=imp, dual_values=dual))


def reference_mw_sort():
    """The reference's MW loop in sort mode (R/main.cpp:36 use_binary_search=false), run through
    our driver oracle/ref_mw_main.cpp over the reference's own solver sources."""
    ref = os.path.join(ROOT, "oracle", "_ref", "dlp_ref_mw")
    if not os.path.exists(ref):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "ref"])
    out = {}
    for (A, I, sp, T) in [(1000, 1000, 0.1, 300), (100, 100, 0.1, 100)]:
        txt = subprocess.run([ref, str(A), str(I), str(sp), str(T), "sort"], capture_output=True,
                             text=True, cwd="/tmp", check=True).stdout
        w = re.findall(r"min weight = (\S+), max weight = (\S+)", txt)
        out[f"{A}x{I}"] = dict(
            A=A, I=I, sparsity=sp, iterations=T,
            dual_values=[float(v) for v in re.findall(r"Dual Value = (\S+)", txt)],
            max_infeasibility=[float(v) for v in re.findall(r"max infeasiblity was (\S+)", txt)],
            min_weight=[float(a) for a, _ in w], max_weight=[float(b) for _, b in w])
    dump("ref_mw_sort.json", dict(
        source="oracle/_ref/dlp_ref_mw = reference solver sources + oracle/ref_mw_main.cpp driver, "
               "sort mode (RunMultiplicativeWeights(T, 1e-18, false)), long double, stdout at 6 digits",
        runs=out))


if __name__ == "__main__":
    kats()
    generated()
    adalloc()
    reference_run()
    reference_mw_sort()
