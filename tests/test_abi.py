"""CPU: the C-ABI library loads, exports every entry point include/dlp.h
declares, and its host-only logic (partition, candidate selection, problem
objects, the embedded glibc rand() of the reference-instance generator) agrees
with the oracle.  No compute call needs a GPU here."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import oracle_py as O
from conftest import ROOT, load_golden

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

HEADER = os.path.join(ROOT, "include", "dlp.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w ]*?\**\s*\b(dlp_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_loads_and_exports_every_declared_symbol():
    names = header_functions()
    assert len(names) >= 40
    lib = L.lib()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    nm = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r" T (dlp_\w+)", nm))
    assert set(names) <= exported


def test_python_binding_covers_header():
    bound = {s[0] for s in L.SIGNATURES}
    assert set(header_functions()) == bound


def test_options_default():
    o = dlp.options()
    assert o.pricing == L.PRICING_DANTZIG_BLAND and o.tol_dj == 1e-9 and o.tol_piv == 1e-9
    assert o.max_pivots == 1_000_000 and o.log_pivots == 1 and o.check_interval == 64
    assert o.nontemporal == -1 and o.use_graph == 1 and o.timing == 0
    assert o.update_variant == -1 and o.ld_align == 0 and o.rows_per_block == 0
    assert L.lib().dlp_update_variants() >= 30


def test_status_strings():
    assert L.lib().dlp_status_string(0) == b"optimal"
    assert L.lib().dlp_status_string(L.UNBOUNDED) == b"unbounded"


@pytest.mark.parametrize("m", [1, 7, 200, 4096, 32768, 32769])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_rank_rows_partition(m, P):
    parts = [dlp.rank_rows(m, r, P) for r in range(P)]
    assert parts[0][0] == 0
    for (f0, c0), (f1, _) in zip(parts, parts[1:]):
        assert f0 + c0 == f1
    assert sum(c for _, c in parts) == m
    assert max(c for _, c in parts) - min(c for _, c in parts) <= 1


def test_rank_rows_rejects_bad_args():
    with pytest.raises(dlp.DLPError):
        dlp.rank_rows(10, 2, 2)


def _oracle_pick(cands):
    best = None
    for i, c in enumerate(cands):
        if not c["valid"]:
            continue
        if best is None or (c["ratio"], c["basis_var"]) < (cands[best]["ratio"], cands[best]["basis_var"]):
            best = i
    return -1 if best is None else best


def test_candidate_select_matches_rule():
    rng = np.random.default_rng(0)
    for trial in range(300):
        n = int(rng.integers(1, 9))
        c = np.zeros(n, dlp.CAND_DTYPE)
        c["valid"] = rng.integers(0, 2, n)
        c["ratio"] = rng.choice([0.0, 0.5, 1.0, 2.0], n)   # many exact ties
        c["basis_var"] = rng.permutation(1000)[:n]
        c["row"] = rng.integers(0, 100, n)
        assert dlp.candidate_select(c) == _oracle_pick(c)


def test_tableau_ld():
    for m, n in [(200, 400), (4096, 4096), (32768, 32768), (3, 2)]:
        assert dlp.tableau_ld(m, n) == O.ld(m, n)
        assert dlp.tableau_ld(m, n) % 16 == 0 and dlp.tableau_ld(m, n) >= n + m + 1


def test_dense_problem_roundtrip_and_validation():
    A, b, c = O.gen_dense(5, 7, 1)
    p = dlp.Problem.dense(A, b, c)
    assert (p.m, p.n) == (5, 7)
    A2, b2, c2 = p.to_dense()
    np.testing.assert_array_equal(A2, A)
    np.testing.assert_array_equal(b2, b)
    np.testing.assert_array_equal(c2, c)
    b[2] = -1.0
    with pytest.raises(dlp.DLPError) as e:
        dlp.Problem.dense(A, b, c)
    assert e.value.status == L.ERR_UNSUPPORTED
    with pytest.raises(ValueError):
        dlp.Problem.dense(A, b[:3], c)


@pytest.mark.parametrize("A,I,sp", [(2, 10, 0.5), (100, 100, 0.1), (1000, 1000, 0.1)])
def test_adalloc_embedded_rand_matches_libc(A, I, sp):
    """libdlp embeds glibc's TYPE_3 rand(); the oracle calls libc rand()."""
    p = dlp.Problem.adalloc(A, I, 1, sp, 0.25)
    adv, imp, bid = p.adalloc_bids()
    g = O.gen_adalloc(A, I, sp, 0.25)
    np.testing.assert_array_equal(adv, g["adv"])
    np.testing.assert_array_equal(imp, g["imp"])
    assert bid.tobytes() == g["bid"].tobytes()
    assert p.m == A + I and p.n == len(bid)
    if A * I <= 10000:
        M, b, c = p.to_dense()
        M2, b2, c2 = O.adalloc_lp(A, I, sp, 0.25)
        np.testing.assert_array_equal(M, M2)
        np.testing.assert_array_equal(b, b2)
        np.testing.assert_array_equal(c, c2)


def test_adalloc_rejects_multislot():
    with pytest.raises(dlp.DLPError):
        dlp.Problem.adalloc(10, 10, 2, 0.1, 0.25)


def test_no_device_fails_loudly():
    """Without a GPU there is no CPU fallback: session creation errors out."""
    if dlp.device_count() > 0:
        pytest.skip("a HIP device is visible")
    p = dlp.Problem.random(10, 10, 1)
    with pytest.raises(dlp.DLPError) as e:
        dlp.solve(p)
    assert e.value.status == L.ERR_NODEVICE
    with pytest.raises(dlp.DLPError):
        dlp.batched_solve(4, 8, 8, 1)


def test_product_never_imports_oracle():
    code = ("import sys, distributedlpsolver_amd, distributedlpsolver_amd.rowblock; "
            "bad=[m for m in sys.modules if 'oracle' in m]; print(bad); assert not bad")
    subprocess.run([sys.executable, "-c", code], cwd=ROOT, check=True)
    # no import / include / dlopen of the oracle anywhere in the product
    bad = re.compile(r"import\s+oracle|oracle_py|liboracle|#include\s+\"oracle|oracle\.h|oracle_\w+\(")
    for dirpath, _, files in os.walk(os.path.join(ROOT, "distributedlpsolver_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                assert not bad.search(open(os.path.join(dirpath, f)).read()), f
    nm = subprocess.run(["nm", "-D", L.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in nm


def test_missing_library_is_loud(tmp_path):
    code = ("import distributedlpsolver_amd._lib as L; L.LIB_PATH='/nonexistent/libdlp.so'; L._lib=None\n"
            "try:\n    L.lib()\nexcept L.NativeLibraryMissing: print('LOUD')\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True)
    assert "LOUD" in out.stdout
