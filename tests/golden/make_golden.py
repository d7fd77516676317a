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
from general_lp import mk, random_general  # noqa: E402


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


def reference_mw_binary():
    """The reference's MW loop in binary (threshold-search) mode, the mode R/main.cpp:36 runs
    (RunMultiplicativeWeights(T, 1e-18, true, 1 - epsilon * 0.001, 3)), through the same driver."""
    ref = os.path.join(ROOT, "oracle", "_ref", "dlp_ref_mw")
    if not os.path.exists(ref):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "ref"])
    out = {}
    for (A, I, sp, T) in [(1000, 1000, 0.1, 300), (100, 100, 0.1, 100)]:
        txt = subprocess.run([ref, str(A), str(I), str(sp), str(T), "binary"], capture_output=True,
                             text=True, cwd="/tmp", check=True).stdout
        w = re.findall(r"min weight = (\S+), max weight = (\S+)", txt)
        cr = re.findall(r"CR: \((\S+), (\S+)\)", txt)
        out[f"{A}x{I}"] = dict(
            A=A, I=I, sparsity=sp, iterations=T,
            dual_values=[float(v) for v in re.findall(r"Dual Value = (\S+)", txt)],
            max_infeasibility=[float(v) for v in re.findall(r"max infeasiblity was (\S+)", txt)],
            min_weight=[float(a) for a, _ in w], max_weight=[float(b) for _, b in w],
            critical_interval=[[float(a), float(b)] for a, b in cr],
            ratios_in_range=[int(v) for v in re.findall(r"total ratios in range (\d+)", txt)])
    dump("ref_mw_binary.json", dict(
        source="oracle/_ref/dlp_ref_mw = reference solver sources + oracle/ref_mw_main.cpp driver, "
               "binary mode (RunMultiplicativeWeights(T, 1e-18, true, 1 - 0.01 * 0.001, 3)), "
               "long double, stdout at 6 digits",
        runs=out))


# ---------------------------------------------------------------- general LPs (f4)
INF = float("inf")


def highs_general(lp):
    """HiGHS on a general LP; marginals per user row = d(objective)/d(row bound) (summed over
    the two sides of a ranged row), objective in the user's sense incl. c0."""
    A = np.asarray(lp["A"], float).reshape(lp["m"], lp["n"])
    rl, rh = np.asarray(lp["row_lo"], float), np.asarray(lp["row_hi"], float)
    sgn = 1.0 if lp["sense"] == 1 else -1.0           # linprog minimises
    c = sgn * np.asarray(lp["c"], float)
    eq = [i for i in range(lp["m"]) if np.isfinite(rl[i]) and rl[i] == rh[i]]
    ub = [i for i in range(lp["m"]) if i not in eq and np.isfinite(rh[i])]
    lb = [i for i in range(lp["m"]) if i not in eq and np.isfinite(rl[i])]
    A_ub = np.vstack([A[ub], -A[lb]]) if ub or lb else None
    b_ub = np.concatenate([rh[ub], -rl[lb]]) if ub or lb else None
    bounds = [(None if not np.isfinite(a) else a, None if not np.isfinite(b) else b)
              for a, b in zip(lp["col_lo"], lp["col_hi"])]
    r = linprog(c, A_ub=A_ub, b_ub=b_ub, A_eq=A[eq] if eq else None,
                b_eq=rl[eq] if eq else None, bounds=bounds, method="highs")
    out = dict(status={0: 0, 2: 1, 3: 2}.get(r.status, -1))
    if r.status == 0:
        y = np.zeros(lp["m"])
        if ub or lb:
            mu = r.ineqlin.marginals
            for k, i in enumerate(ub):
                y[i] += mu[k]
            for k, i in enumerate(lb):
                y[i] -= mu[len(ub) + k]
        if eq:
            for k, i in enumerate(eq):
                y[i] += r.eqlin.marginals[k]
        out.update(objective=float(sgn * r.fun + lp["c0"]), x=[float(v) for v in r.x],
                   y=[float(sgn * v) for v in y])
    return out


def ub_eq(name, source, c, A_ub=None, b_ub=None, A_eq=None, b_eq=None, bounds=(0, None), **expect):
    """A scipy linprog-style KAT (min c^T x) as a general LP."""
    n = len(c)
    rows, lo, hi = [], [], []
    if A_ub is not None:
        for a, b in zip(np.atleast_2d(A_ub), b_ub):
            rows.append(a); lo.append(-INF); hi.append(b)
    if A_eq is not None:
        for a, b in zip(np.atleast_2d(A_eq), b_eq):
            rows.append(a); lo.append(b); hi.append(b)
    if isinstance(bounds, tuple) and len(bounds) == 2 and not isinstance(bounds[0], (tuple, list)):
        bounds = [bounds] * n
    cl = [-INF if b[0] is None else b[0] for b in bounds]
    ch = [INF if b[1] is None else b[1] for b in bounds]
    return mk(name, source, np.array(rows, float).reshape(len(rows), n), lo, hi, cl, ch, c, **expect)


def general():
    S = "scipy/optimize/tests/test_linprog.py"
    nt = dict(c=[-1, 8, 4, -6], A_ub=[[-7, -7, 6, 9], [1, -1, -3, 0], [10, -10, -7, 7], [6, -1, 3, 4]],
              b_ub=[-3, 6, -6, 6], A_eq=[[-10, 1, 1, -8]], b_eq=[-4])
    m20 = 20
    t20 = 2 * np.pi * np.arange(1, m20 + 1) / (m20 + 1)
    t50 = 2 * np.pi * np.arange(50) / 51
    r0 = np.cos(t50) - 1; r0[0] = 0.0
    r1 = np.sin(t50); r1[0] = 0.0
    rs = np.random.RandomState(0)
    cr = rs.rand(10); Ar = rs.rand(10, 10); br = rs.rand(10)
    Ar[-1, :] = 2 * Ar[-2, :]; br[-1] *= -1
    A2, b2, c2 = lpgen_2d(20, 20)
    cases = [
        ub_eq("nontrivial", f"{S}:190-201,1089-1094 (all constraint types, negative rhs)",
              **nt, expected_objective=7083 / 1391,
              expected_x=[101 / 1391, 1462 / 1391, 0, 752 / 1391]),
        ub_eq("inequality_2", f"{S}:692-703 (b < 0 rows)", [6, 3], [[0, 3], [-1, -1], [-2, 1]],
              [2, -1, -1], expected_objective=5.0, expected_x=[2 / 3, 1 / 3]),
        ub_eq("bounds_mixed", f"{S}:762-774 (free + negative lower bound)", [1, -4],
              [[-3, 1], [1, 2]], [6, 4], bounds=[(None, None), (-3, None)],
              expected_objective=-80 / 7, expected_x=[-8 / 7, 18 / 7]),
        ub_eq("bounded_above_only_2", f"{S}:744-751", np.ones(3), A_eq=np.eye(3), b_eq=[1, 2, 3],
              bounds=(-INF, 4), expected_objective=6.0, expected_x=[1, 2, 3]),
        ub_eq("bounds_infinity", f"{S}:753-760 (free variables)", np.ones(3), A_eq=np.eye(3),
              b_eq=[1, 2, 3], bounds=(None, None), expected_objective=6.0, expected_x=[1, 2, 3]),
        ub_eq("bounds_equal_but_infeasible", f"{S}:776-783", [-4, 1], [[7, -2], [0, 1], [2, -2]],
              [14, 0, 3], bounds=[(2, 2), (0, None)], expected_status=1),
        ub_eq("bounds_equal_but_infeasible2", f"{S}:785-792", [-4, 1], A_eq=[[7, -2], [0, 1], [2, -2]],
              b_eq=[14, 0, 3], bounds=[(2, 2), (0, None)], expected_status=1),
        ub_eq("zero_row_1", f"{S}:853-859 (zero equality rows: redundant)", [1, 2, 3],
              A_eq=[[0, 0, 0], [1, 1, 1], [0, 0, 0]], b_eq=[0, 3, 0], expected_objective=3.0),
        ub_eq("remove_redundancy_infeasibility", f"{S}:1068-1082", cr, A_eq=Ar, b_eq=br,
              expected_status=1),
        ub_eq("network_flow", f"{S}:1109-1129 (equality network, one redundant row)",
              [2, 4, 9, 11, 4, 3, 8, 7, 0, 15, 16, 18],
              A_eq=[[-1, -1, 1, 0, 1, 0, 0, 0, 0, 1, 0, 0], [1, 0, 0, 1, 0, 1, 0, 0, 0, 0, 0, 0],
                    [0, 0, -1, -1, 0, 0, 0, 0, 0, 0, 0, 0], [0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 0],
                    [0, 0, 0, 0, -1, -1, -1, 0, 1, 0, 0, 0], [0, 0, 0, 0, 0, 0, 0, -1, -1, 0, 0, 1],
                    [0, 0, 0, 0, 0, 0, 0, 0, 0, -1, -1, -1]],
              b_eq=[0, 19, -16, 33, 0, 0, -36], expected_objective=755.0),
        ub_eq("network_flow_limited_capacity", f"{S}:1131-1157 (boxed flows)", [2, 2, 1, 3, 1],
              A_eq=[[-1, -1, 0, 0, 0], [1, 0, -1, -1, 0], [0, 1, 1, 0, -1], [0, 0, 0, 1, 1]],
              b_eq=[-4, 0, 0, 4], bounds=[(0, 4), (0, 2), (0, 2), (0, 3), (0, 5)],
              expected_objective=14.0),
        ub_eq("enzo", f"{S}:1172-1190", [4, 8, 3, 0, 0, 0],
              A_eq=[[2, 5, 3, -1, 0, 0], [3, 2.5, 8, 0, -1, 0], [8, 10, 4, 0, 0, -1]],
              b_eq=[185, 155, 600], expected_objective=317.5,
              expected_x=[66.25, 0, 17.5, 0, 183.75, 0]),
        ub_eq("enzo_b", f"{S}:1192-1207", [2.8, 6.3, 10.8, -2.8, -6.3, -10.8],
              A_eq=[[-1, -1, -1, 0, 0, 0], [0, 0, 0, 1, 1, 1], [1, 0, 0, 1, 0, 0], [0, 1, 0, 0, 1, 0],
                    [0, 0, 1, 0, 0, 1]], b_eq=[-0.5, 0.4, 0.3, 0.3, 0.3], expected_objective=-1.77),
        ub_eq("enzo_c_degeneracy", f"{S}:1209-1218", -np.ones(m20),
              A_eq=np.vstack((np.cos(t20) - 1, np.sin(t20))), b_eq=[0, 0], expected_objective=0.0,
              expected_x=[0.0] * m20),
        ub_eq("enzo_c_unbounded", f"{S}:1220-1235", -np.ones(50), A_eq=np.vstack((r0, r1)),
              b_eq=[0, 0], expected_status=2),
        ub_eq("enzo_c_infeasible", f"{S}:1237-1249", -np.ones(50),
              A_eq=np.vstack((np.cos(t50) - 1, np.sin(t50))), b_eq=[1, 1], expected_status=1),
        ub_eq("basic_artificial_vars", f"{S}:1251-1267 (artificials basic at the Phase I optimum)",
              [-0.1, -0.07, 0.004, 0.004, 0.004, 0.004],
              [[1.0, 0, 0, 0, 0, 0], [-1.0, 0, 0, 0, 0, 0], [0, -1.0, 0, 0, 0, 0], [0, 1.0, 0, 0, 0, 0],
               [1.0, 1.0, 0, 0, 0, 0]], [3.0, 3.0, 3.0, 3.0, 20.0],
              A_eq=[[1.0, 0, -1, 1, -1, 1], [0, -1.0, -1, 1, -1, 1]], b_eq=[0, 0],
              expected_objective=0.0, expected_x=[0.0] * 6),
        ub_eq("lpgen_2d_20x20", f"{S}:147-171,1096-1107 (inequality form)", c2, A2, b2,
              expected_objective=-64.049494229),
        ub_eq("lpgen_2d_20x20_eq", f"{S}:147-171 as equalities (transportation, one redundant row)",
              c2, A_eq=A2, b_eq=b2),
        mk("testprob", "tests/golden/testprob.mps (the MPS format description's example)",
           [[1, 1, 0], [1, 0, 1], [0, -1, 1]], [-INF, 1, 7], [4, INF, 7], [0, -1, 0], [4, 1, INF],
           [1, 2, 3], expected_objective=16.0),
        random_general("random_8x12", 8, 12, 101),
        random_general("random_20x30", 20, 30, 102),
        random_general("random_40x60_max", 40, 60, 103, sense=-1, c0=2.5),
        random_general("random_60x100", 60, 100, 104, frac_eq=0.1),
        random_general("random_30x20_eq", 30, 20, 105, frac_eq=0.1),
    ]
    for cs in cases:
        cs["highs"] = highs_general(cs)
        lp = O.GeneralLP(np.array(cs["A"]).reshape(cs["m"], cs["n"]), cs["row_lo"], cs["row_hi"],
                         cs["col_lo"], cs["col_hi"], cs["c"], cs["c0"], cs["sense"])
        for pricing in (0, 1):
            s = O.solve_general(lp, pricing=pricing)
            cs[f"oracle_pricing{pricing}"] = dict(
                status=int(s.status), objective=float(s.objective), pivots=int(s.num_pivots),
                phase1_pivots=int(s.phase1_pivots), log_sha256=log_digest(s.pivot_log))
        print(cs["name"], cs["highs"]["status"], cs["highs"].get("objective"),
              cs["oracle_pricing0"])
    dump("general.json", cases)


def lpgen_2d(m, n):
    """scipy/optimize/tests/test_linprog.py:147-171 (restated): m*n vars, m+n constraints."""
    rng = np.random.RandomState(0)
    c = - rng.exponential(size=(m, n))
    A = np.zeros((m + n, m * n))
    b = np.zeros(m + n)
    for j in range(m):
        A[j, j * n:(j + 1) * n] = 1
        b[j] = n / m
    for j in range(n):
        A[m + j, j::n] = 1
        b[m + j] = 1
    return A, b, c.ravel()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "general":
    general()
    sys.exit(0)

if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "mw_binary":
    reference_mw_binary()
    sys.exit(0)

if __name__ == "__main__":
    kats()
    generated()
    adalloc()
    reference_run()
    reference_mw_sort()
    reference_mw_binary()
