"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: bit-identical pivot logs (q, p, leaving,
r_p, objective) and bit-identical tableaus / objective / x / y for index and
fp64 pivot work; objective within 1e-9 relative of the HiGHS fixtures."""
import hashlib

import numpy as np
import pytest

import oracle_py as O
from conftest import load_golden

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

pytestmark = pytest.mark.gpu


def _same_log(got, ref):
    assert len(got) == len(ref), (len(got), len(ref))
    g = np.ascontiguousarray(got)
    r = np.ascontiguousarray(ref)
    if g.tobytes() != r.tobytes():
        for k in range(len(r)):
            if g[k].tobytes() != r[k].tobytes():
                raise AssertionError(f"pivot {k}: gpu {g[k]} oracle {r[k]}")


def _solve_both(A, b, c, **opts):
    res = dlp.solve(dlp.Problem.dense(A, b, c), **opts)
    ref = O.solve_dense(A, b, c, pricing=opts.get("pricing", 0), nthreads=8)
    return res, ref


def _check_equal(res, ref):
    assert res.status == ref.status
    _same_log(res.pivot_log, ref.pivot_log)
    assert res.num_pivots == ref.num_pivots
    assert np.float64(res.objective).tobytes() == np.float64(ref.objective).tobytes()
    assert res.x.tobytes() == ref.x.tobytes()
    assert res.y.tobytes() == ref.y.tobytes()
    np.testing.assert_array_equal(res.basis, ref.basis)


@pytest.mark.parametrize("kat", load_golden("kat.json"), ids=lambda k: k["name"])
@pytest.mark.parametrize("pricing", [0, 1])
@pytest.mark.parametrize("defer", [0, 16])  # 0 = auto: eager below 32 MiB
def test_kat(kat, pricing, defer):
    A, b, c = np.array(kat["A"]), np.array(kat["b"]), np.array(kat["c"])
    res, ref = _solve_both(A, b, c, pricing=pricing, defer=defer)
    _check_equal(res, ref)
    assert res.status == kat.get("expected_status", 0)
    if "expected_x" in kat:
        np.testing.assert_allclose(res.x, kat["expected_x"], atol=1e-12)


@pytest.mark.parametrize("case", [c for c in load_golden("generated.json")],
                         ids=lambda c: c["name"])
@pytest.mark.parametrize("defer", [0, 16])  # 0 = auto: eager below 32 MiB
def test_generated_host_input(case, defer):
    """Host-supplied dense LPs (C1, C4 degenerate): bit-identical to the oracle,
    objective within 1e-9 of HiGHS."""
    A, b, c = O.gen_dense(case["m"], case["n"], case["seed"], case["degenerate"])
    res, ref = _solve_both(A, b, c, defer=defer)
    _check_equal(res, ref)
    hi = case["highs"]["objective"]
    assert abs(res.objective - hi) <= 1e-9 * abs(hi)
    assert hashlib.sha256(np.ascontiguousarray(res.pivot_log).tobytes()).hexdigest() == \
        case["oracle"]["log_sha256"]


@pytest.mark.parametrize("m,n,seed,degen", [(200, 400, 1, False), (37, 53, 11, True),
                                            (300, 129, 4, False), (1000, 24, 2, True)])
def test_device_generator_matches_oracle(m, n, seed, degen):
    with dlp.Session(dlp.Problem.random(m, n, seed, degen)) as s:
        T = s.tableau()
    np.testing.assert_array_equal(T, O.gen_tableau(m, n, seed, degen))


def test_aligned_row_stride_generation():
    m, n, seed = 300, 129, 4
    with dlp.Session(dlp.Problem.random(m, n, seed), ld_align=512) as s:
        assert s.ld % 512 == 0 and s.ld >= O.ld(m, n)
        T = s.tableau()
    ref = O.gen_tableau(m, n, seed)
    np.testing.assert_array_equal(T[:, :ref.shape[1]], ref)
    assert not T[:, ref.shape[1]:].any()


def test_device_generated_c1_solve():
    p = dlp.Problem.random(200, 400, 1)
    res = dlp.solve(p)
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    _check_equal(res, ref)


@pytest.mark.parametrize("opts", [dict(rows_per_block=4), dict(rows_per_block=8, nontemporal=0),
                                  dict(rows_per_block=128), dict(use_graph=0, check_interval=1),
                                  dict(check_interval=7, timing=2), dict(timing=1),
                                  dict(ld_align=512, update_variant=12, rows_per_block=8),
                                  dict(ld_align=64, update_variant=17)],
                         ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
def test_launch_options_do_not_change_results(opts):
    A, b, c = O.gen_dense(200, 400, 2)
    res, ref = _solve_both(A, b, c, **opts)
    _check_equal(res, ref)


@pytest.mark.parametrize("defer", [0, 8])
def test_pivot_limit_and_resume(defer):
    A, b, c = O.gen_dense(120, 150, 9)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), check_interval=16, defer=defer) as s:
        st, done = s.run(50)
        assert st == L.RUNNING and done == 50
        st, done2 = s.run(10 ** 6)
        assert st == L.OK and done + done2 == ref.num_pivots
        res = s.result()
    _check_equal(res, ref)


@pytest.mark.parametrize("defer", [0, 8])
def test_max_pivots_reports_limit(defer):
    A, b, c = O.gen_dense(120, 150, 9)
    res = dlp.solve(dlp.Problem.dense(A, b, c), max_pivots=20, check_interval=8, defer=defer)
    assert res.status == L.PIVOT_LIMIT and res.num_pivots == 20
    ref = O.solve_dense(A, b, c, max_pivots=20)
    _same_log(res.pivot_log, ref.pivot_log)


@pytest.mark.parametrize("defer", [0, 4])
def test_unbounded(defer):
    A = np.array([[-1.0, 1.0], [1.0, -2.0]])
    res, ref = _solve_both(A, np.array([1.0, 2.0]), np.array([1.0, 1.0]), defer=defer)
    assert res.status == ref.status == L.UNBOUNDED
    _same_log(res.pivot_log, ref.pivot_log)


def test_empty_and_ragged_shapes():
    # one constraint, one variable; tall-thin; wide-short; rows with all-zero coefficients
    for (A, b, c) in [(np.array([[2.0]]), np.array([3.0]), np.array([1.0])),
                      (O.gen_dense(500, 3, 1)), (O.gen_dense(3, 700, 2))]:
        res, ref = _solve_both(A, b, c)
        _check_equal(res, ref)
    A, b, c = O.gen_dense(40, 30, 3)
    A[5] = 0.0
    A[17] = 0.0
    res, ref = _solve_both(A, b, c)
    _check_equal(res, ref)


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_multi_rank_sessions_one_gpu(P):
    """P row-block sessions on one GPU, exchanged by the host (all-gather of
    the 32-B candidates, int64 MAX all-reduce of the pivot row): same log."""
    m, n, seed = 150, 170, 4
    A, b, c = O.gen_dense(m, n, seed)
    ref = O.solve_dense(A, b, c)
    prob = dlp.Problem.random(m, n, seed)
    sess = [dlp.Session(prob, rank=r, nranks=P) for r in range(P)]
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
    x = np.sum([r.x for r in results], axis=0)   # each basic row lives on one rank
    assert x.tobytes() == ref.x.tobytes()
    # the in-process merge (dlp_sessions_result), ranks in any order
    merged = dlp.Session.merged_result(sess[::-1])
    assert merged.x.tobytes() == ref.x.tobytes() and merged.y.tobytes() == ref.y.tobytes()
    _same_log(merged.pivot_log, ref.pivot_log)
    for s in sess:
        s.close()


@pytest.mark.parametrize("defer", [0, 1, 16])
def test_solve_n_gpus_in_process(defer):
    """dlp_solve with n_gpus = 1: the in-process multi-device path (ncclCommInitAll,
    one host thread per device, RCCL exchange, merged result) on this box's GPU."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    res = dlp.solve(dlp.Problem.dense(A, b, c), n_gpus=1, exchange=L.XCHG_RCCL, defer=defer)
    _check_equal(res, ref)
    with pytest.raises(L.DLPError):
        dlp.solve(dlp.Problem.dense(A, b, c), n_gpus=dlp.device_count() + 1)


@pytest.mark.parametrize("defer", [0, 1, 16, 32])
def test_rccl_exchange_path_single_rank(defer):
    """The RCCL exchange path (all-gather + select kernel + MAX all-reduce; with
    defer > 1 also the commit kernel and the rank-K pass, as bench.py --gpus N
    runs it) on a 1-rank communicator gives the same log as the oracle."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), rank=0, nranks=1,
                     rccl_id=dlp.comm_unique_id(), exchange=L.XCHG_RCCL, timing=2, defer=defer) as s:
        assert s.update_stats()[2] == (defer or 1)
        st, done = s.run(10 ** 6)
        res = s.result()
    assert st == L.OK
    _check_equal(res, ref)


@pytest.mark.parametrize("A_,I_", [(2, 10), (100, 100), (200, 200)])
@pytest.mark.parametrize("defer", [0, 16])  # 0 = auto: eager below 32 MiB
def test_adalloc_bridge(A_, I_, defer):
    """f1: the reference's own generated instance solved exactly on the GPU."""
    rec = [r for r in load_golden("adalloc.json") if (r["A"], r["I"]) == (A_, I_)][0]
    p = dlp.Problem.adalloc(A_, I_, 1, rec["sparsity"], rec["scaling"])
    res = dlp.solve(p, defer=defer)
    M, b, c = O.adalloc_lp(A_, I_, rec["sparsity"], rec["scaling"])
    ref = O.solve_dense(M, b, c)
    _check_equal(res, ref)
    assert abs(res.objective - rec["highs_objective"]) <= 1e-9 * rec["highs_objective"]


def test_batched_c5_small():
    nlp, m, n, seed = 48, 64, 64, 100
    for degen in (False, True):
        br = dlp.batched_solve(nlp, m, n, seed, degenerate=degen, want_basis=True, log_cap=4096)
        for k in range(nlp):
            A, b, c = O.gen_dense(m, n, seed + k, degen)
            ref = O.solve_dense(A, b, c, nthreads=1)
            assert br.status[k] == ref.status
            assert br.num_pivots[k] == ref.num_pivots
            assert np.float64(br.objective[k]).tobytes() == np.float64(ref.objective).tobytes()
            np.testing.assert_array_equal(br.basis[k], ref.basis)
            _same_log(br.logs[k][:ref.num_pivots], ref.pivot_log)


@pytest.mark.parametrize("n", [32, 100, 128, 191])
def test_batched_register_kernel_shapes(n):
    """m = 64: the register-resident batched kernel (one lane per slot; 1, 2, 2, 3 waves
    per LP, the last wave partly idle except at n = 191), dense and degenerate LPs (Bland,
    exact ratio ties), every LP against the oracle."""
    nlp, m, seed = 16, 64, 300 + n
    for degen in (False, True):
        br = dlp.batched_solve(nlp, m, n, seed, degenerate=degen, want_basis=True, log_cap=4096)
        for k in range(nlp):
            A, b, c = O.gen_dense(m, n, seed + k, degen)
            ref = O.solve_dense(A, b, c, nthreads=1)
            assert br.status[k] == ref.status
            assert br.num_pivots[k] == ref.num_pivots
            assert np.float64(br.objective[k]).tobytes() == np.float64(ref.objective).tobytes()
            np.testing.assert_array_equal(br.basis[k], ref.basis)
            _same_log(br.logs[k][:ref.num_pivots], ref.pivot_log)


def test_batched_matches_single_gpu_path():
    br = dlp.batched_solve(4, 32, 96, 7, log_cap=2048)
    for k in range(4):
        res = dlp.solve(dlp.Problem.random(32, 96, 7 + k))
        assert res.num_pivots == br.num_pivots[k]
        _same_log(br.logs[k][:res.num_pivots], res.pivot_log)


@pytest.mark.parametrize("variant", range(L.lib().dlp_update_variants()))
def test_update_variants_bit_identical(variant):
    A, b, c = O.gen_dense(150, 260, 6)
    ref = O.solve_dense(A, b, c)
    for rb, nt in ((4, 1), (64, 0)):
        res = dlp.solve(dlp.Problem.dense(A, b, c), update_variant=variant, rows_per_block=rb,
                        nontemporal=nt, defer=1)
        _check_equal(res, ref)


def test_retune_mid_solve():
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), check_interval=8, defer=1) as s:
        for k, v in enumerate([4, 0, 6, 2, 5, 7, 1, 3] * 100):
            s.set_tuning(v, 4 + 4 * (k % 5), k % 2)
            st, _ = s.run(16)
            if st != L.RUNNING:
                break
        res = s.result()
    _check_equal(res, ref)


def test_release_cached_memory():
    """finished sessions leave their small buffers in a per-process cache;
    dlp_release_cached_memory frees them, and a solve afterwards is unaffected."""
    A, b, c = O.gen_dense(120, 150, 4)
    ref = O.solve_dense(A, b, c)
    dlp.release_cached_memory()
    res = dlp.solve(dlp.Problem.dense(A, b, c), small_lp=-1)
    assert dlp.release_cached_memory(0) > 0   # that solve's device buffers were cached
    assert dlp.release_cached_memory(0) == 0
    dlp.release_cached_memory()               # + the pinned host buffers
    assert dlp.release_cached_memory() == 0
    res2 = dlp.solve(dlp.Problem.dense(A, b, c), small_lp=-1)
    assert res.pivot_log.tobytes() == res2.pivot_log.tobytes() == ref.pivot_log.tobytes()


def test_batched_occupancy_query():
    """dlp_batched_occupancy (bench.py --workload c5's roofline): the register-resident kernel at
    m = 64 (ceil(n / 64) waves per LP), the LDS-resident one otherwise; at least one LP per CU."""
    o128 = dlp.batched_occupancy(64, 128)
    assert o128["register_kernel"] and o128["threads_per_lp"] == 128 and o128["lps_per_cu"] >= 1
    o = dlp.batched_occupancy(64, 64)   # one wave per LP: at least as many LPs per CU
    assert o["register_kernel"] and o["threads_per_lp"] == 64 and o["lps_per_cu"] >= o128["lps_per_cu"]
    o = dlp.batched_occupancy(40, 60)
    assert not o["register_kernel"] and o["threads_per_lp"] in (256, 512) and o["lps_per_cu"] >= 1
