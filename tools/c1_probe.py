import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import distributedlpsolver_amd as dlp
import oracle_py as O
A, b, c = O.gen_dense(200, 400, 1)
p = dlp.Problem.dense(A, b, c)
for kw in ({}, {"small_lp": 1}, {"small_lp": -1}, {"small_lp": 1, "max_pivots": 4096}):
    ts = []
    for _ in range(4):
        t0 = time.perf_counter(); r = dlp.solve(p, **kw); ts.append(1e3 * (time.perf_counter() - t0))
    print(kw, r.num_pivots, [round(t, 2) for t in ts], file=sys.stderr, flush=True)
