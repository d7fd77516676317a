"""Deferred rank-k update (dlp_defer.hip) against the eager rank-1 path and the
oracle, bit for bit.  K pivots are selected on replayed views of the stale
tableau and applied in one pass; every element must see exactly the eager
sequence of fma / overwrite / skip, so pivot logs, x, y, basis and the whole
tableau (incl. the objective row and padding) are identical for every block
size, poll window (block boundaries anywhere in a window), pass geometry and
cache policy."""
import numpy as np
import pytest

import oracle_py as O

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

pytestmark = pytest.mark.gpu


def _same_log(got, ref):
    assert len(got) == len(ref), (len(got), len(ref))
    g, r = np.ascontiguousarray(got), np.ascontiguousarray(ref)
    if g.tobytes() != r.tobytes():
        for k in range(len(r)):
            if g[k].tobytes() != r[k].tobytes():
                raise AssertionError(f"pivot {k}: gpu {g[k]} oracle {r[k]}")


def _check(res, ref):
    assert res.status == ref.status
    _same_log(res.pivot_log, ref.pivot_log)
    assert np.float64(res.objective).tobytes() == np.float64(ref.objective).tobytes()
    assert res.x.tobytes() == ref.x.tobytes() and res.y.tobytes() == ref.y.tobytes()
    assert res.basis.tobytes() == ref.basis.tobytes()


@pytest.mark.parametrize("K", [2, 3, 8, 16, 32, 64])
@pytest.mark.parametrize("ci,graph", [(5, 1), (16, 1), (64, 1), (100, 0)])
def test_defer_c1_full_solve(K, ci, graph):
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    res = dlp.solve(dlp.Problem.dense(A, b, c), defer=K, check_interval=ci, use_graph=graph)
    _check(res, ref)


@pytest.mark.parametrize("K", [4, 16])
@pytest.mark.parametrize("pricing", [0, 1])
def test_defer_degenerate_bland(K, pricing):
    A, b, c = O.gen_dense(128, 128, 3, degenerate=True)
    ref = O.solve_dense(A, b, c, pricing=pricing)
    res = dlp.solve(dlp.Problem.dense(A, b, c), defer=K, pricing=pricing)
    _check(res, ref)


@pytest.mark.parametrize("K,rb,occ,nt,form", [(16, 16, 0, 0, 0), (16, 64, 4, 1, 0), (16, 256, 2, 1, 1),
                                              (32, 128, 3, 0, 0), (8, 7, 6, 1, 2), (32, 64, 4, 1, 2),
                                              (64, 64, 0, 1, 2), (64, 33, 4, 0, 1), (5, 64, 4, 1, 2),
                                              (16, 64, 0, 1, 3), (32, 37, 4, 0, 3), (64, 64, 2, 1, 3),
                                              (8, 16, 0, 1, 4), (32, 100, 4, 1, 4), (13, 64, 0, 0, 4),
                                              (16, 64, 0, 1, 5), (48, 29, 0, 1, 5), (64, 256, 4, 0, 5),
                                              (48, 64, 0, 1, 3), (24, 128, 0, 0, 3), (40, 64, 0, 1, 5),
                                              (7, 64, 4, 1, 3),
                                              # streamed forms 6-9 (K < 16 runs form 3; K = 24 / 48
                                              # run the partial-block instance of the next template)
                                              (16, 64, 0, 1, 6), (32, 256, 0, 1, 6), (32, 100, 0, 0, 7),
                                              (24, 64, 4, 1, 7), (16, 37, 0, 1, 8), (32, 64, 2, 0, 8),
                                              (64, 128, 0, 1, 9), (48, 64, 0, 1, 9), (8, 64, 0, 1, 6),
                                              (64, 1024, 0, 1, 8), (32, 64, 0, 1, 10), (16, 64, 4, 0, 11),
                                              (64, 64, 0, 1, 12), (32, 37, 0, 1, 13),
                                              (32, 256, 0, 1, 14), (16, 64, 0, 0, 14), (8, 64, 0, 1, 14),
                                              (32, 256, 0, 1, 15), (24, 64, 0, 0, 15), (32, 16, 4, 1, 16),
                                              (16, 64, 0, 0, 17), (64, 32, 0, 1, 18), (32, 8, 0, 1, 19),
                                              (32, 256, 0, 1, 20), (16, 64, 0, 0, 20), (24, 33, 0, 1, 20)])
def test_defer_pass_geometry_and_tableau(K, rb, occ, nt, form):
    """Whole tableau after 45 pivots equals the eager session's, byte for byte."""
    m, n, seed = 300, 520, 5
    prob = dlp.Problem.random(m, n, seed)
    with dlp.Session(prob, defer=1, check_interval=45) as e:
        e.run(45)
        Te = e.tableau()
        le = e.result().pivot_log
    with dlp.Session(prob, defer=K, check_interval=45, rows_per_block=rb, nontemporal=nt) as s:
        s.set_defer_tuning(occ, form)
        s.run(45)
        Td = s.tableau()
        ld = s.result().pivot_log
    _same_log(ld, le)
    assert Td.tobytes() == Te.tobytes()


@pytest.mark.parametrize("form,K,rb", [(6, 32, 64), (7, 16, 64), (8, 32, 128), (9, 64, 64), (10, 32, 64),
                                       (13, 64, 128), (16, 32, 16), (17, 32, 64), (18, 64, 32)])
def test_defer_streamed_forms_many_bands(form, K, rb):
    """Streamed pass forms on 47-94 bands (the work order's band groups of 16,
    the last one partial, and 12-24 column tiles): 2 full blocks and a partial
    one, whole tableau byte-equal to the eager session's."""
    m = n = 3000
    k = 2 * K + 7
    prob = dlp.Problem.random(m, n, 11)
    with dlp.Session(prob, defer=1, check_interval=k) as e:
        e.run(k)
        Te = e.tableau()
        le = e.result().pivot_log
    with dlp.Session(prob, defer=K, check_interval=K, rows_per_block=rb) as s:
        s.set_defer_tuning(0, form)
        done = 0
        while done < k:
            done += s.run(min(K, k - done))[1]
        Td = s.tableau()
        ld = s.result().pivot_log
    _same_log(ld, le)
    assert Td.tobytes() == Te.tobytes()


@pytest.mark.parametrize("K", [8, 16, 32])
@pytest.mark.parametrize("fused", [False, True])
def test_fused_pivot_toggle(K, fused):
    """Ratio test + selection + pivot row in one launch (default for single-rank
    deferred sessions) or in two: both bit-identical to the oracle, incl. the
    optimal stop inside a window (the fused launch's early release)."""
    A, b, c = O.gen_dense(200, 400, 4)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=K, check_interval=37) as s:
        s.set_fused_pivot(fused)
        s.run(10 ** 6)
        res = s.result()
    _check(res, ref)


def test_fused_pivot_unbounded():
    A = np.array([[1.0, -1.0], [-1.0, 0.0]])
    b = np.array([1.0, 0.0])
    c = np.array([1.0, 1.0])
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=8) as s:
        st, _ = s.run(100)
        assert st == L.UNBOUNDED


def test_defer_retune_between_runs():
    A, b, c = O.gen_dense(200, 400, 2)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=16, check_interval=9) as s:
        for k in range(1000):
            s.set_tuning(22 if k % 2 else 26, [16, 64, 200][k % 3], k % 2)
            s.set_defer_tuning([0, 4, 2][k % 3], k % 21)
            st, _ = s.run(11)
            if st != L.RUNNING:
                break
        res = s.result()
    _check(res, ref)


@pytest.mark.parametrize("form", [2, 3, 4, 5, 6, 8])
def test_defer_adalloc_sparse_rows(form):
    """Sparse tableau: most rows untouched by most steps (skip rule in the pass)."""
    p = dlp.Problem.adalloc(200, 200, 1, 0.1, 0.25)
    M, b, c = O.adalloc_lp(200, 200, 0.1, 0.25)
    ref = O.solve_dense(M, b, c)
    with dlp.Session(p, defer=16) as s:
        s.set_defer_tuning(0, form)
        s.run(10 ** 6)
        res = s.result()
    _check(res, ref)


def test_defer_rejects_bad_settings():
    A, b, c = O.gen_dense(20, 30, 1)
    with pytest.raises(L.DLPError):
        dlp.solve(dlp.Problem.dense(A, b, c), defer=65)
    with pytest.raises(L.DLPError):
        dlp.solve(dlp.Problem.dense(A, b, c), defer=8, update_variant=4)   # 1024-column tiles
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=8) as s:
        with pytest.raises(L.DLPError):
            s.set_tuning(4, 8, 1)


def test_defer_update_stats():
    with dlp.Session(dlp.Problem.random(400, 600, 7), defer=8, timing=2, check_interval=40) as s:
        s.run(40)
        n, ms, k = s.update_stats()
    assert k == 8 and n == 5 and ms > 0


@pytest.mark.parametrize("P,K,form", [(1, 8, -1), (2, 4, -1), (2, 16, -1), (3, 32, -1), (2, 64, 21), (3, 64, 21),
                                      (2, 64, 22), (4, 16, -1), (4, 64, 21), (8, 16, -1), (8, 64, 21),
                                      (2, 64, 23), (8, 64, 23)])
def test_defer_step_api_multi_rank_one_gpu(P, K, form):
    """The deferred exchange path (ratio -> candidate all-gather -> select ->
    pivot-row MAX all-reduce -> commit, pass every K pivots) with P row-block
    sessions on one GPU and the host doing the exchanges: the same pivot log,
    objective, x and y as the oracle.  This is the device code the RCCL path of
    bench.py --gpus N runs."""
    m, n, seed = 150, 170, 4
    A, b, c = O.gen_dense(m, n, seed)
    ref = O.solve_dense(A, b, c)
    prob = dlp.Problem.random(m, n, seed)
    sess = [dlp.Session(prob, rank=r, nranks=P, defer=K) for r in range(P)]
    assert all(s.update_stats()[2] == K for s in sess)
    if form >= 0:   # the multi-GPU C3 geometry's pass (K = 64, form 21) on every rank
        for s in sess:
            s.set_defer_tuning(0, form)
    status = L.RUNNING
    for _ in range(10_000):
        cands = np.concatenate([s.step_candidate() for s in sess])
        st, _ = sess[0].status()
        if st != L.RUNNING:
            status = st
            break
        sends = [s.step_select(cands) for s in sess]
        prow = np.max(np.stack(sends), axis=0)
        for s in sess:
            s.step_update(prow)
    assert status == L.OK
    results = [s.result() for s in sess]
    for r in results:
        _same_log(r.pivot_log, ref.pivot_log)
        assert np.float64(r.objective).tobytes() == np.float64(ref.objective).tobytes()
        np.testing.assert_array_equal(r.y, ref.y)
    x = np.sum([r.x for r in results], axis=0)
    assert x.tobytes() == ref.x.tobytes()
    # the stacked local tableaus equal the eager single-rank tableau after the same pivots
    with dlp.Session(prob, defer=1) as e:
        e.run(10 ** 6)
        Te = e.tableau()
    rows = [s.tableau()[:-1] for s in sess]
    Td = np.concatenate(rows + [sess[0].tableau()[-1:]])
    assert Td.tobytes() == Te.tobytes()
    for s in sess:
        s.close()


def test_auto_block_size_policy():
    """defer = 0 (auto): eager under 32 MiB of tableau, K = 16 up to 1 GiB."""
    with dlp.Session(dlp.Problem.random(256, 512, 4, degenerate=True)) as s:
        assert s.update_stats()[2] == 1
    with dlp.Session(dlp.Problem.random(2048, 2048, 2)) as s:   # 2049 x 4097 doubles = 67 MB
        assert s.update_stats()[2] == 16


@pytest.mark.parametrize("form", [21, 22, 23])
@pytest.mark.parametrize("m,n,seed,rb,nt,occ", [(300, 520, 5, 64, 1, 0), (300, 520, 5, 256, 0, 0),
                                                (700, 1337, 7, 1000, 1, 0), (129, 4000, 2, 37, 1, 2),
                                                (1200, 700, 9, 128, 1, 3)])
def test_pass_form21_dpp_full_blocks(m, n, seed, rb, nt, occ, form):
    """Forms 21 (DPP-broadcast coefficients), 22 (MFMA) and 23 (DPP from an LDS ring), K = 64: two full
    blocks and a partial one
    (17 steps: the unused steps' coefficients and pivot rows zeroed at block start), widths that are not a
    multiple of the 256-column tile, bands from 37 to 1000 rows (the last one short),
    pivot rows inside the bands; whole tableau byte-equal to the eager session's."""
    k = 2 * 64 + 17
    prob = dlp.Problem.random(m, n, seed)
    with dlp.Session(prob, defer=1, check_interval=k) as e:
        e.run(k)
        Te = e.tableau()
        le = e.result().pivot_log
    assert len(le) == k
    with dlp.Session(prob, defer=64, check_interval=64, rows_per_block=rb, nontemporal=nt) as s:
        s.set_defer_tuning(occ, form)
        done = 0
        while done < k:
            done += s.run(min(64, k - done))[1]
        Td = s.tableau()
        ld = s.result().pivot_log
    _same_log(ld, le)
    assert Td.tobytes() == Te.tobytes()


@pytest.mark.parametrize("form", [21, 22, 23])
@pytest.mark.parametrize("K", [64, 40])
def test_pass_form21_sparse_and_degenerate(K, form):
    """Form 21 on a sparse tableau (ad-allocation LP: untouched / sparse rows through
    the generic replay) and a degenerate one (Bland), full solves against the oracle;
    K = 40 runs form 3 (form 21 needs 64-step blocks)."""
    p = dlp.Problem.adalloc(200, 200, 1, 0.1, 0.25)
    M, b, c = O.adalloc_lp(200, 200, 0.1, 0.25)
    ref = O.solve_dense(M, b, c)
    with dlp.Session(p, defer=K) as s:
        s.set_defer_tuning(0, form)
        s.run(10 ** 6)
        res = s.result()
    _check(res, ref)
    A, b, c = O.gen_dense(128, 128, 3, degenerate=True)
    ref = O.solve_dense(A, b, c, pricing=0)
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=K, check_interval=100) as s:
        s.set_defer_tuning(0, form)
        s.run(10 ** 6)
        res = s.result()
    _check(res, ref)


def _chunk_digests(sess, rows, chunk=1024):
    """Digests of the touched columns (the first roundup(N+1, 16)) of every row: sessions with
    different row strides (eager 4 KiB, deferred 1 KiB alignment) compare equal."""
    import hashlib
    width = (sess.ncols + 1 + 15) // 16 * 16
    out = []
    for first in range(0, rows + 1, chunk):
        cnt = min(chunk, rows + 1 - first)
        out.append(hashlib.sha256(np.ascontiguousarray(sess.read_rows(first, cnt)[:, :width]).tobytes()).hexdigest())
    return out


@pytest.mark.parametrize("form", [1, 2])
def test_lds_forms_on_streaming_k64_geometry(form):
    """on a streaming K = 64 session the auto band is 768 rows for the
    register-resident forms; the LDS-staged forms 1 / 2 (K * rb * 8 + rb * 4 bytes of LDS)
    must get a band that fits 160 KiB when the form is switched, and stay bit-identical:
    2 full blocks + a 9-pivot tail, whole tableau (chunk digests) equal to the eager session's."""
    m = n = 16384   # 16385 x 32784 doubles = 4.3 GB: streaming, >= 16k rows
    k = 2 * 64 + 9
    prob = dlp.Problem.random(m, n, 21)
    with dlp.Session(prob, defer=64, check_interval=64) as s:
        # lookahead: form 21 beside the chain, form 23 when the chain has CUs of its own (16,384 rows:
        # 64 of them); no lookahead: form 23
        assert s.get_tuning()[1] == 768
        assert s.defer_form() == (21 if s.lookahead() and s.chain_cus() == 0 else 23)
        s.set_defer_tuning(0, form)
        rb = s.get_tuning()[1]
        assert 64 * rb * 8 + rb * 4 + 64 * 4 <= 160 * 1024 and rb >= 256
        done = 0
        while done < k:
            done += s.run(min(64, k - done))[1]
        ld = s.result().pivot_log
        dd = _chunk_digests(s, m)
        s.set_defer_tuning(0, 21)   # back to the DPP form: the auto band follows
        assert s.get_tuning()[1] == 768
    with dlp.Session(prob, defer=1, check_interval=k) as e:
        e.run(k)
        le = e.result().pivot_log
        de = _chunk_digests(e, m)
    _same_log(ld, le)
    assert dd == de
