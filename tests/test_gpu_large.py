"""GPU, BASELINE.json full sizes: C2 (4096 x 4096, N = 8192) bit-exact against
the oracle for a window of pivots; C3 (32768 x 32768, N = 65536, 17.2 GB
tableau) against the oracle on sampled rows plus size-independent invariants
(basic columns form an exact identity, objective non-decreasing)."""
import numpy as np
import pytest

import oracle_py as O

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


def test_c5_full_batch():
    """4,096 independent 64 x 64 LPs (C5): statuses and spot LPs vs oracle."""
    nlp, m, n, seed = 4096, 64, 64, 5000
    br = dlp.batched_solve(nlp, m, n, seed, log_cap=0)
    assert (br.status == 0).all()
    for k in (0, 1, 2047, 4095):
        A, b, c = O.gen_dense(m, n, seed + k)
        ref = O.solve_dense(A, b, c, nthreads=1)
        assert br.num_pivots[k] == ref.num_pivots
        assert np.float64(br.objective[k]).tobytes() == np.float64(ref.objective).tobytes()
