"""GPU, BASELINE.json C3 (32768 x 32768, N = 65536) as the multi-GPU row
partition runs it, on ONE MI355X: 8 rank sessions of the same LP (4,096 local
rows x 65,537 columns each, 2.2 GB per rank), the geometry a rank of the
8-GPU split picks by itself (K = 64 deferred blocks through the form-23 pass,
256-row bands, no lookahead), the exchange done by the host (all-gather of the
32-B candidates, int64 MAX all-reduce of the pivot row: the device code the RCCL
path runs, SURVEY.md §8(e), replacing the reference's per-impression
decomposition at R/global_problem.cpp:270-274).

160 pivots = two full 64-pivot blocks and a 32-pivot tail, compared bit for bit
with the oracle's run of the same LP through committed digests
(tests/golden/make_digests.py c3_k64 / c3_tableau): the pivot log, the basis,
the objective and the WHOLE tableau (all 32,769 rows, stacked in global row
order from the 8 ranks)."""
import hashlib

import numpy as np
import pytest

from conftest import load_golden, tableau_sha256

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _drive(sess, k):
    """k pivots through the host exchange (rowblock.run_rowblock's protocol)."""
    for _ in range(k):
        cands = np.concatenate([s.step_candidate() for s in sess])
        st, _ = sess[0].status()
        assert st == L.RUNNING
        sends = [s.step_select(cands) for s in sess]
        prow = np.max(np.stack(sends), axis=0)
        for s in sess:
            s.step_update(prow)


@pytest.mark.parametrize("P", [8])
def test_c3_row_partition_one_gpu(P):
    g = load_golden("digests.json")
    tab = g["c3_tableau"]
    k = 160
    want = tab["stops"][str(k)]
    m, n = tab["m"], tab["n"]
    prob = dlp.Problem.random(m, n, tab["seed"])
    sess = [dlp.Session(prob, rank=r, nranks=P, check_interval=64) for r in range(P)]
    try:
        for r, s in enumerate(sess):
            occ, form, K = s.get_defer_tuning()
            assert (K, form) == (64, 23), (r, K, form)   # the auto multi-rank geometry (no lookahead)
            assert s.get_tuning()[1] == 256               # 256-row bands below 16k local rows
            assert not s.lookahead()
            assert s.rows in (m // P, m // P + 1)
        _drive(sess, k)
        logs = [s.result().pivot_log for s in sess]
        for lg in logs:
            assert len(lg) == k
            assert _sha(lg) == want["log_sha256"] == g["c3_k64"]["log_prefix_sha256"][str(k)]
        merged = dlp.Session.merged_result(sess)
        assert _sha(merged.basis) == want["basis_sha256"]
        assert float(merged.objective).hex() == want["objective_hex"]
        assert tableau_sha256(sess, tab["width"]) == want["tableau_sha256"]
    finally:
        for s in sess:
            s.close()
