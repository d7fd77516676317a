import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L
import oracle_py as O
m, n, seed = 150, 170, 4
A, b, c = O.gen_dense(m, n, seed)
ref = O.solve_dense(A, b, c)
for K in (16, 2):
  for win in (1, 5, 16):
    sa = dlp.Session(dlp.Problem.random(m, n, seed), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(), defer=K, check_interval=win)
    sb = dlp.Session(dlp.Problem.random(m, n, seed), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(), defer=K, check_interval=win, exchange=L.XCHG_PEER)
    print("K", K, "win", win, "modes", sa.get_exchange(), sb.get_exchange(), flush=True)
    done = 0
    for it in range(400):
        sta, da = sa.run(win); stb, db = sb.run(win)
        done += da
        la, lb = sa.result().pivot_log, sb.result().pivot_log
        if la.tobytes() != lb.tobytes() or da != db:
            k = next((i for i in range(min(len(la), len(lb))) if la[i].tobytes() != lb[i].tobytes()), None)
            print("diverge after", done, "pivots: first differing log entry", k, la[k] if k is not None else None, lb[k] if k is not None else None, da, db)
            Ta, Tb = sa.tableau(), sb.tableau()
            d = np.argwhere(Ta != Tb)
            print("tableau diffs", len(d), d[:10], flush=True)
            break
        Ta, Tb = sa.tableau(), sb.tableau()
        if Ta.tobytes() != Tb.tobytes():
            d = np.argwhere(Ta != Tb)
            print("tableau differs after", done, "pivots (logs equal):", len(d), d[:10], Ta[tuple(d[0])], Tb[tuple(d[0])], flush=True)
            break
        if sta != L.RUNNING and sta != L.PIVOT_LIMIT:
            print("both ended", sta, stb, done, "oracle", ref.num_pivots, flush=True); break
    sa.close(); sb.close()
