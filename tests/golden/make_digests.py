#!/usr/bin/env python3
"""Generate tests/golden/digests.json: oracle digests of long runs at the
BASELINE.json full sizes, too slow for the oracle inside a GPU test but cheap
for the GPU to reproduce.  Run in the build container (CPU only):

    python tests/golden/make_digests.py [c2] [c3]

  c2  C2 4096 x 4096 seed 2 (dense family) solved to optimality by the oracle:
      pivot count, status, sha256 of the pivot log / x / y, objective bits.
  c3  C3 32768 x 32768 seed 3: the exact pivot sequence of round 2's first
      bench.py default (5 warm-up + 20 timed blocks of K = 32 pivots, then a
      20-pivot window = 820 pivots): sha256 of the log, the objective row and
      sampled constraint rows after those pivots.
  c3_k64  the same LP through the current default (K = 64 blocks: 5 + 20 blocks
      of 64 pivots, then the 20-pivot window = 1620 pivots).
  c3_tableau  whole-tableau digests of the same LP: after 136
      pivots (test_c3_full_blocks_bit_exact), 160 (the 8-rank row partition,
      tests/test_gpu_c3_rowblock.py), 1620 (the bench window) and 1876 (+ the
      bench's 256-pivot second-exchange window at N > 1): sha256 of all
      32,769 rows (objective row last), each its first `width` doubles, streamed
      in row order; plus the log prefix and basis digests at each stop.
  c5  every LP of the C5 batches (4,096 x 64x128 and 4,096 x 64x64, seed 5000): per-field
      digests of status, pivot count, objective bits, basis and the first 64 log entries.
  rank_split  bench.py's c3r4 LP (8192 x 57344 seed 34) split over 2 processes of
      4,096 rows (the per-process rank path, tests/test_gpu_ranks.py): per-rank block
      digests, objective row, log and basis at 136 / 200 / 264 pivots.
  rank_split_c3  C3 itself (32768 x 32768 seed 3) split over 2, 3, 4 and 8 processes (the
      rank geometries of the N = 2, 4, 8 scaling runs, and a ragged 3-way split of 10,922 /
      10,923 / 10,923 rows): the same digests at 136 / 200 pivots, with the block digests of
      each split ("blocks": {"2": [...], "3": [...], "4": [...], "8": [...]}).
  c4_degen_2048x4096  C4's large degenerate LP (2048 x 4096 seed 4, degenerate family: b_i = 0
      on half the rows, Bland after every degenerate pivot): whole-tableau, log, basis and
      objective digests at 500, 2,000 and 30,000 pivots, plus the degenerate-pivot count.

The digests hash little-endian fp64 / int32 bytes of the oracle's outputs
(tests/oracle_py.py), so the GPU side compares bit for bit."""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_py as O  # noqa: E402

OUT = os.path.join(HERE, "digests.json")
C3_PIVOTS = 5 * 32 + 20 * 32 + 20
C3_K64_PIVOTS = 5 * 64 + 20 * 64 + 20
C3_ROWS = [0, 1, 777, 12345, 20000, 32767]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def c2():
    m = n = 4096
    t0 = time.time()
    A, b, c = O.gen_dense(m, n, 2)
    r = O.solve_dense(A, b, c, nthreads=os.cpu_count() or 8, log_cap=200_000)
    return {"m": m, "n": n, "seed": 2, "status": r.status, "num_pivots": int(r.num_pivots),
            "objective_hex": float(r.objective).hex(), "log_sha256": sha(r.pivot_log),
            "x_sha256": sha(r.x), "y_sha256": sha(r.y), "basis_sha256": sha(r.basis),
            "oracle_seconds": time.time() - t0}


def c3(pivots=C3_PIVOTS):
    m = n = 32768
    t0 = time.time()
    rows = np.array(C3_ROWS + [m], np.int64)   # + the objective row
    log, out, basis = O.run_generated(m, n, 3, pivots, rows, nthreads=os.cpu_count() or 8)
    w = ((n + m + 1) + 15) // 16 * 16
    return {"m": m, "n": n, "seed": 3, "pivots": int(len(log)), "log_sha256": sha(log),
            "log_prefix_sha256": {str(k): sha(log[:k]) for k in (160, 800, 820, 1600) if k <= len(log)},
            "objective_hex": float(log[-1]["objective"]).hex(),
            "rows": C3_ROWS, "width": w,
            "row_sha256": {str(i): sha(out[k, :w]) for k, i in enumerate(C3_ROWS)},
            "objective_row_sha256": sha(out[-1, :w]), "basis_sha256": sha(basis),
            "oracle_seconds": time.time() - t0}


def tableau_sha(T, w, chunk=512):
    h = hashlib.sha256()
    for r in range(0, T.shape[0], chunk):
        h.update(np.ascontiguousarray(T[r:r + chunk, :w]).tobytes())
    return h.hexdigest()


def c3_tableau(stops=(136, 160, C3_K64_PIVOTS, C3_K64_PIVOTS + 256)):
    m = n = 32768
    t0 = time.time()
    w = ((n + m + 1) + 15) // 16 * 16
    out = {"m": m, "n": n, "seed": 3, "width": w, "rows": m + 1, "stops": {}}

    def at(k, T, log, basis):
        out["stops"][str(k)] = {"log_sha256": sha(log), "tableau_sha256": tableau_sha(T, w),
                                "basis_sha256": sha(basis), "objective_hex": float(log[-1]["objective"]).hex(),
                                "oracle_seconds": time.time() - t0}
        print(k, out["stops"][str(k)], flush=True)

    O.run_generated_stops(m, n, 3, list(stops), at, nthreads=os.cpu_count() or 8)
    return out


def rank_split(m=8192, n=57344, seed=34, P=2, stops=(136, 200, 264), Ps=None):
    """The per-process rank path of a scaling run: bench.py's c3r4 LP
    (8192 x 57344 seed 34) row-partitioned over P = 2 processes, so that each rank holds
    4,096 x 65,537 — exactly one rank of C3's 8-GPU split.  At each stop: the log and
    basis digests, the objective bits, and one sha256 per rank's row block (rows
    [floor(r m / P), floor((r+1) m / P)), each row its first `width` doubles) plus one of
    the objective row, so every process can check its own block without the others'.
    Ps: several splits of the same run, their block digests under "blocks" keyed by P."""
    t0 = time.time()
    w = ((n + m + 1) + 15) // 16 * 16
    out = {"m": m, "n": n, "seed": seed, "P": P, "width": w, "stops": {}}
    if Ps:
        out["Ps"] = list(Ps)

    def blocks(T, p):
        cuts = [r * m // p for r in range(p + 1)]
        return [tableau_sha(T[cuts[r]:cuts[r + 1]], w) for r in range(p)]

    def at(k, T, log, basis):
        rec = {"log_sha256": sha(log), "basis_sha256": sha(basis),
               "objective_hex": float(log[-1]["objective"]).hex(),
               "objective_row_sha256": sha(T[m, :w]), "oracle_seconds": time.time() - t0}
        if Ps:
            rec["blocks"] = {str(p): blocks(T, p) for p in Ps}
        else:
            rec["block_sha256"] = blocks(T, P)
        out["stops"][str(k)] = rec
        print(k, rec, flush=True)

    O.run_generated_stops(m, n, seed, list(stops), at, nthreads=os.cpu_count() or 8)
    return out


def c4_degen(m=2048, n=4096, seed=4, stops=(500, 2000, 30000)):
    """the 50%-zero-RHS degenerate LP at 2,048 x 4,096, the
    size the small-LP launch does not cover (auto: the deferred K = 16 path).  Whole-tableau
    digests (all 2,049 rows, objective row last, each its first `width` doubles) at each stop."""
    t0 = time.time()
    w = ((n + m + 1) + 15) // 16 * 16
    out = {"m": m, "n": n, "seed": seed, "degenerate": True, "width": w, "stops": {}}

    def at(k, T, log, basis):
        rec = {"log_sha256": sha(log), "basis_sha256": sha(basis), "tableau_sha256": tableau_sha(T, w),
               "objective_hex": float(log[-1]["objective"]).hex(),
               "degenerate_pivots": int((log["ratio"] == 0.0).sum()),
               "oracle_seconds": time.time() - t0}
        out["stops"][str(k)] = rec
        print(k, rec, flush=True)

    O.run_generated_stops(m, n, seed, list(stops), at, degenerate=True, nthreads=os.cpu_count() or 8)
    return out


C5_SHAPES = [(64, 64), (64, 128)]


def c5_records(st, npiv, obj, basis, logs):
    """The per-LP digests of a C5 batch (GPU and oracle alike): status, pivot count, objective
    bits, basis and the first <= 64 log entries of every LP, each field hashed in LP order."""
    h = hashlib.sha256()
    for k in range(len(st)):
        h.update(np.ascontiguousarray(logs[k][:min(64, int(npiv[k]))]).tobytes())
    return {"status_sha256": sha(np.asarray(st, np.int32)), "num_pivots_sha256": sha(np.asarray(npiv, np.int64)),
            "objective_sha256": sha(np.asarray(obj, np.float64)), "basis_sha256": sha(np.asarray(basis, np.int32)),
            "log64_sha256": h.hexdigest()}


def c5(nlp=4096, seed=5000):
    """C5 (BASELINE.json: 4,096 independent 64 x 128 LPs) and its 64 x 64 twin: the oracle's
    solve of EVERY LP of the batch (LP k = generated dense LP of seed `seed + k`), digested
    per field (all 4,096 LPs pinned, not a sample)."""
    out = {}
    for m, n in C5_SHAPES:
        t0 = time.time()
        st = np.zeros(nlp, np.int32)
        npiv = np.zeros(nlp, np.int64)
        obj = np.zeros(nlp)
        basis = np.zeros((nlp, m), np.int32)
        logs = []
        for k in range(nlp):
            A, b, c = O.gen_dense(m, n, seed + k)
            r = O.solve_dense(A, b, c, nthreads=1)
            st[k], npiv[k], obj[k] = r.status, r.num_pivots, r.objective
            basis[k] = r.basis
            logs.append(np.ascontiguousarray(r.pivot_log[:64]))
        d = {"m": m, "n": n, "nlp": nlp, "seed": seed, "max_pivots": int(npiv.max()),
             "all_optimal": bool((st == 0).all())}
        d.update(c5_records(st, npiv, obj, basis, logs))
        d["oracle_seconds"] = time.time() - t0
        out[f"{m}x{n}"] = d
    return out


def main():
    which = sys.argv[1:] or ["c2", "c3"]
    d = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            d = json.load(f)
    for w in which:
        d[w] = {"c2": c2, "c3": c3, "c3_k64": lambda: c3(C3_K64_PIVOTS), "c3_tableau": c3_tableau,
                "c5": c5, "rank_split": rank_split,
                "rank_split_c3": lambda: rank_split(32768, 32768, 3, P=2, stops=(136, 200), Ps=(2, 3, 4, 8)),
                "c4_degen_2048x4096": c4_degen}[w]()
        with open(OUT, "w") as f:
            json.dump(d, f, indent=1)
        print(w, json.dumps(d[w]), flush=True)


if __name__ == "__main__":
    main()
