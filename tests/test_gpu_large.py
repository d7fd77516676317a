"""GPU, BASELINE.json full sizes: C2 (4096 x 4096, N = 8192) bit-exact against
the oracle for a window of pivots; C3 (32768 x 32768, N = 65536, 17.2 GB
tableau) against the oracle on sampled rows plus size-independent invariants
(basic columns form an exact identity, objective non-decreasing)."""
import hashlib

import numpy as np
import pytest

import oracle_py as O
from conftest import load_golden, tableau_sha256

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

pytestmark = pytest.mark.gpu


def _basis_identity(rows, row_ids, basis):
    """Rows row_ids of the tableau, exact identity on the basic columns."""
    for r, i in zip(rows, row_ids):
        cols = basis[row_ids]
        expect = (np.asarray(row_ids) == i).astype(np.float64)
        np.testing.assert_array_equal(r[cols], expect)


def test_c2_window_bit_exact():
    m = n = 4096
    k = 12
    rng = np.random.default_rng(0)
    with dlp.Session(dlp.Problem.random(m, n, 2), check_interval=4) as s:
        st, done = s.run(k)
        assert done == k
        res = s.result()
        sample = np.unique(np.concatenate([res.pivot_log["p"], rng.integers(0, m, 48), [m]]))
        rows = np.stack([s.read_rows(int(i), 1)[0] for i in sample])
    log, ref_rows, ref_basis = O.run_generated(m, n, 2, k, sample, nthreads=16)
    assert np.ascontiguousarray(res.pivot_log).tobytes() == np.ascontiguousarray(log).tobytes()
    w = ref_rows.shape[1]   # the session may pad rows further (4 KiB alignment): real columns only
    assert np.ascontiguousarray(rows[:, :w]).tobytes() == ref_rows.tobytes()
    assert not rows[:, w:].any()
    np.testing.assert_array_equal(res.basis, ref_basis)


def test_c3_full_size():
    m = n = 32768
    k = 6
    with dlp.Session(dlp.Problem.random(m, n, 3), check_interval=k) as s:
        # generation: spot rows equal the oracle's row-slice generator
        for first in (0, 12345, m - 3):
            ref = O.gen_tableau(m, n, 3, row_first=first, row_count=3, nthreads=16)[:3]
            got = s.read_rows(first, 3)
            assert np.ascontiguousarray(got[:, :ref.shape[1]]).tobytes() == ref.tobytes()
            assert not got[:, ref.shape[1]:].any()
        st, done = s.run(k)
        assert st == L.RUNNING and done == k
        res = s.result()
        piv_rows = res.pivot_log["p"].astype(np.int64)
        sample = np.unique(np.concatenate([piv_rows, [0, 1, 777, 20000, m - 1]]))
        rows = np.stack([s.read_rows(int(i), 1)[0] for i in sample])
        obj_row = s.read_rows(m, 1)[0]
    # invariants
    _basis_identity(rows, sample, res.basis)
    assert np.all(np.diff(res.pivot_log["objective"]) >= 0)
    assert obj_row[m + n] == res.objective == res.pivot_log["objective"][-1]
    # oracle on the same 17 GB instance (host, 16 threads), compared on sampled rows
    log, ref_rows, _ = O.run_generated(m, n, 3, k, np.concatenate([sample, [m]]), nthreads=16)
    assert np.ascontiguousarray(res.pivot_log).tobytes() == np.ascontiguousarray(log).tobytes()
    w = ref_rows.shape[1]
    assert np.ascontiguousarray(rows[:, :w]).tobytes() == ref_rows[:-1].tobytes()
    assert np.ascontiguousarray(obj_row[:w]).tobytes() == ref_rows[-1].tobytes()


AUTO_K64_FORM = 23   # the streaming K = 64 default at C3: condensed tableau, lookahead with the chain on 64 CUs
                     # of its own and the LDS-ring pass on the rest (dlp_session.cpp pick_form, chain_cus_policy)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _full_blocks_vs_oracle(m, n, seed, k, ci, want_K, defer=0, tableau_digest=None, form=None, lookahead=-1):
    """k pivots in windows of ci (whole K-blocks, then a tail) through the auto
    geometry of the bench (deferred K, pass form, band rows, ld alignment);
    the whole pivot log, every pivot row, random rows and the objective row
    against the oracle on the same generated LP, byte for byte."""
    rng = np.random.default_rng(seed)
    with dlp.Session(dlp.Problem.random(m, n, seed), check_interval=ci, defer=defer, lookahead=lookahead) as s:
        if form is not None:
            s.set_defer_tuning(0, form)
        occ, f, K = s.get_defer_tuning()
        assert K == want_K
        if K == 64:
            assert f == (form or AUTO_K64_FORM) and s.get_tuning()[1] == 768   # the bench's pass
            assert s.lookahead()   # auto from 4 GiB: block b+1 selected during pass b
        if K == 32:
            assert f == 4 and s.get_tuning()[1] == 256   # round 2's first default
            # lookahead is auto only at K = 64 since round 4 (profiles/r04l/): forced here
            assert s.lookahead() == (lookahead == 1)
        done = 0
        while done < k:
            st, d = s.run(min(ci, k - done))
            assert st == L.RUNNING
            done += d
        res = s.result()
        launches = s.update_stats()[0]
        sample = np.unique(np.concatenate([res.pivot_log["p"].astype(np.int64),
                                           rng.integers(0, m, 24), [0, m - 1]]))
        rows = np.stack([s.read_rows(int(i), 1)[0] for i in sample])
        obj_row = s.read_rows(m, 1)[0]
        # the whole tableau (all m + 1 rows) against the oracle's committed digest
        if tableau_digest is not None:
            assert tableau_sha256([s], tableau_digest["width"]) == tableau_digest["tableau_sha256"]
    log, ref_rows, ref_basis = O.run_generated(m, n, seed, k, np.concatenate([sample, [m]]),
                                               nthreads=16)
    assert len(res.pivot_log) == k == len(log)
    bad = [j for j in range(k) if res.pivot_log[j].tobytes() != log[j].tobytes()]
    assert not bad, f"first differing pivot {bad[0]}: gpu {res.pivot_log[bad[0]]} oracle {log[bad[0]]}"
    w = ref_rows.shape[1]
    assert np.ascontiguousarray(rows[:, :w]).tobytes() == ref_rows[:-1].tobytes()
    assert not rows[:, w:].any()
    assert np.ascontiguousarray(obj_row[:w]).tobytes() == ref_rows[-1].tobytes()
    np.testing.assert_array_equal(res.basis, ref_basis)
    return launches


@pytest.mark.parametrize("form", [None, 21, 23])
def test_c3_full_blocks_bit_exact(form):
    """C3 at the bench geometry: 2 full K = 64 blocks through the auto pass (and forms 21
    and 23 explicitly: DPP coefficients, registers / LDS ring; 768-row bands, ld 65664,
    nt), then an 8-pivot tail (a partial block: coefficients of the unused steps zeroed in
    memory); the whole tableau against the oracle's digest."""
    tab = load_golden("digests.json")["c3_tableau"]
    _full_blocks_vs_oracle(32768, 32768, 3, 136, 128, 64,
                           tableau_digest=dict(tab["stops"]["136"], width=tab["width"]), form=form)


def test_c3_k32_lookahead_full_blocks_bit_exact():
    """C3 with K = 32 (form 4, lookahead forced on): 2 full blocks and an 8-pivot tail."""
    _full_blocks_vs_oracle(32768, 32768, 3, 72, 64, 32, defer=32, lookahead=1)


def test_c2_full_blocks_bit_exact():
    """C2: 2 full K = 16 blocks (cache-resident geometry) then a partial one."""
    _full_blocks_vs_oracle(4096, 4096, 2, 40, 32, 16)


@pytest.mark.parametrize("K", [64, 32])
def test_c3_bench_window_digest(K):
    """The exact pivot sequence of the default bench.py run (5 warm-up + 20
    timed blocks of K pivots, then the 20-pivot window; K = 64 is the default,
    K = 32 with lookahead round 2's first) against digests of the oracle's run
    committed in tests/golden/digests.json (tests/golden/make_digests.py): log,
    objective, objective row and sampled constraint rows, bit for bit."""
    g = load_golden("digests.json")["c3_k64" if K == 64 else "c3"]
    m, n = g["m"], g["n"]
    with dlp.Session(dlp.Problem.random(m, n, g["seed"]), check_interval=64 * 20, timing=1,
                     max_pivots=64 * 25 + 22, defer=0 if K == 64 else 32, lookahead=1) as s:
        assert s.get_defer_tuning()[2] == K and s.lookahead()
        for k in (5 * K, 20 * K, 20):
            st, d = s.run(k)
            assert st == L.RUNNING and d == k
        res = s.result()
        rows = {str(i): s.read_rows(i, 1)[0, :g["width"]] for i in g["rows"]}
        obj_row = s.read_rows(m, 1)[0, :g["width"]]
        if K == 64:   # the whole tableau after the bench window (all 32,769 rows)
            tab = load_golden("digests.json")["c3_tableau"]
            assert tableau_sha256([s], tab["width"]) == tab["stops"][str(g["pivots"])]["tableau_sha256"]
    assert len(res.pivot_log) == g["pivots"]
    for k, h in g["log_prefix_sha256"].items():
        assert _sha(res.pivot_log[:int(k)]) == h, f"log prefix {k}"
    assert _sha(res.pivot_log) == g["log_sha256"]
    assert float(res.objective).hex() == g["objective_hex"]
    assert _sha(obj_row) == g["objective_row_sha256"]
    for i, h in g["row_sha256"].items():
        assert _sha(rows[i]) == h, f"row {i}"
    assert _sha(res.basis) == g["basis_sha256"]


@pytest.mark.parametrize("lookahead", [-1, 1])
def test_c2_full_solve_digest(lookahead):
    """C2 solved to optimality on the GPU (deferred K = 16 auto; and with lookahead
    forced on, which auto leaves off at 268 MB) equals the oracle's full solve
    (tests/golden/digests.json): pivot count, log, x, y, basis, objective bits."""
    g = load_golden("digests.json")["c2"]
    res = dlp.solve(dlp.Problem.random(g["m"], g["n"], g["seed"]), max_pivots=200_000,
                    lookahead=lookahead)
    assert res.status == g["status"] == L.OK
    assert res.num_pivots == g["num_pivots"]
    assert _sha(res.pivot_log) == g["log_sha256"]
    assert float(res.objective).hex() == g["objective_hex"]
    assert _sha(res.x) == g["x_sha256"] and _sha(res.y) == g["y_sha256"]
    assert _sha(res.basis) == g["basis_sha256"]


@pytest.mark.parametrize("split", ["stops", "ragged"])
def test_c4_degenerate_2048x4096_digest(split):
    """C4's large degenerate LP (2,048 x 4,096, half the RHS zero)
    through the auto path at this size (deferred K = 16: the tableau is 100 MB, above the small-LP
    launch and below lookahead), against the oracle's committed stops (tests/golden/make_digests.py
    c4_degen_2048x4096): pivot log, basis, objective bits and the WHOLE tableau (2,049 rows).  Every
    pivot of these windows is degenerate (r_p = 0), so each one exercises Bland after a degenerate
    pivot and the exact-tie rule of the ratio test.  "ragged": windows that end inside K = 16 blocks."""
    g = load_golden("digests.json")["c4_degen_2048x4096"]
    stops = sorted(int(k) for k in g["stops"])
    with dlp.Session(dlp.Problem.random(g["m"], g["n"], g["seed"], degenerate=True),
                     check_interval=97, max_pivots=stops[-1] + 1) as s:
        assert s.update_stats()[2] == 16 and not s.lookahead() and not s.small_lp()
        total = 0
        for k in stops:
            windows = [k - total] if split == "stops" else [(k - total) // 3 + 5, k - total - ((k - total) // 3 + 5)]
            for w in windows:
                st, done = s.run(w)
                assert st == L.RUNNING and done == w
                total += w
            want = g["stops"][str(k)]
            res = s.result()
            assert len(res.pivot_log) == k
            assert _sha(res.pivot_log) == want["log_sha256"]
            assert int((res.pivot_log["ratio"] == 0.0).sum()) == want["degenerate_pivots"]
            assert _sha(res.basis) == want["basis_sha256"]
            assert float(res.objective).hex() == want["objective_hex"]
            assert tableau_sha256([s], g["width"]) == want["tableau_sha256"]


@pytest.mark.parametrize("m,n", [(64, 64), (64, 128)])
def test_c5_full_batch(m, n):
    """4,096 independent LPs (C5; BASELINE.json: 64 x 128): EVERY LP of the batch against the
    oracle's committed digests (tests/golden/make_digests.py c5: status, pivot count, objective
    bits, basis and the first 64 pivot-log entries of each LP, hashed in LP order), and sampled
    LPs against the oracle itself."""
    nlp, seed = 4096, 5000
    br = dlp.batched_solve(nlp, m, n, seed, log_cap=64, want_basis=True)
    assert (br.status == 0).all()
    want = load_golden("digests.json")["c5"][f"{m}x{n}"]
    assert (want["nlp"], want["seed"]) == (nlp, seed)
    h = hashlib.sha256()
    for k in range(nlp):
        h.update(np.ascontiguousarray(br.logs[k][:min(64, int(br.num_pivots[k]))]).tobytes())
    got = {"status_sha256": _sha(np.asarray(br.status, np.int32)),
           "num_pivots_sha256": _sha(np.asarray(br.num_pivots, np.int64)),
           "objective_sha256": _sha(np.asarray(br.objective, np.float64)),
           "basis_sha256": _sha(np.asarray(br.basis, np.int32)), "log64_sha256": h.hexdigest()}
    for key, val in got.items():
        assert val == want[key], key
    for k in (0, 1, 777, 2047, 3000, 4095):
        A, b, c = O.gen_dense(m, n, seed + k)
        ref = O.solve_dense(A, b, c, nthreads=1)
        assert br.num_pivots[k] == ref.num_pivots
        assert np.float64(br.objective[k]).tobytes() == np.float64(ref.objective).tobytes()
        np.testing.assert_array_equal(br.basis[k], ref.basis)
        cnt = min(64, ref.num_pivots)
        assert br.logs[k][:cnt].tobytes() == np.ascontiguousarray(ref.pivot_log[:cnt]).tobytes()
