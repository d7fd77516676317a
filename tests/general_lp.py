"""General-LP test helpers: fixture records, a seeded
random general-LP generator (every row / column bound type; feasible and dual
feasible, hence optimal), and an MPS writer used to exercise the product's MPS
reader.  Test infrastructure; shared by tests/ and tests/golden/make_golden.py."""
from __future__ import annotations

import numpy as np

import oracle_py as O

INF = float("inf")


def mk(name, source, A, row_lo, row_hi, col_lo, col_hi, c, c0=0.0, sense=1, **expect):
    A = np.asarray(A, float)
    m, n = A.shape
    return dict(name=name, source=source, m=m, n=n, A=A.ravel().tolist(),
                row_lo=[float(v) for v in row_lo], row_hi=[float(v) for v in row_hi],
                col_lo=[float(v) for v in np.broadcast_to(col_lo, (n,))],
                col_hi=[float(v) for v in np.broadcast_to(col_hi, (n,))],
                c=[float(v) for v in c], c0=float(c0), sense=int(sense), **expect)


def random_general(name, m, n, seed, sense=1, c0=0.0, frac_eq=0.2):
    """Feasible and dual-feasible (hence optimal) random general LP: every row / column type."""
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((m, n)) * (rng.random((m, n)) < 0.6)
    ckind = rng.choice(6, size=n, p=[0.35, 0.15, 0.15, 0.1, 0.15, 0.1])   # lo0 box hi free lo fixed
    x0 = rng.uniform(-2, 2, n)
    cl = np.full(n, -INF); ch = np.full(n, INF)
    for j, k in enumerate(ckind):
        if k == 0: cl[j] = 0.0; x0[j] = abs(x0[j])
        elif k == 1: cl[j] = x0[j] - rng.uniform(0, 2); ch[j] = x0[j] + rng.uniform(0, 2)
        elif k == 2: ch[j] = x0[j] + rng.uniform(0, 2)
        elif k == 4: cl[j] = x0[j] - rng.uniform(0, 2)
        elif k == 5: cl[j] = ch[j] = x0[j]
    ax = A @ x0
    rest = 1.0 - 0.35 - 0.25 - frac_eq
    rkind = rng.choice(5, size=m, p=[0.35, 0.25, frac_eq, 0.75 * rest, 0.25 * rest])   # L G E ranged free
    rl = np.full(m, -INF); rh = np.full(m, INF)
    for i, k in enumerate(rkind):
        if k == 0: rh[i] = ax[i] + rng.uniform(0, 1)
        elif k == 1: rl[i] = ax[i] - rng.uniform(0, 1)
        elif k == 2: rl[i] = rh[i] = ax[i]
        elif k == 3: rl[i] = ax[i] - rng.uniform(0, 1); rh[i] = ax[i] + rng.uniform(0, 1)
    # dual-feasible c (min form): c = A^T y + d with sign-correct y, d
    y = rng.uniform(0, 1, m)
    y[rkind == 0] *= -1
    y[rkind == 2] = rng.uniform(-1, 1, int((rkind == 2).sum()))
    y[rkind == 3] *= rng.choice([-1, 1], int((rkind == 3).sum()))
    y[rkind == 4] = 0.0
    d = rng.uniform(0, 1, n)
    d[ckind == 2] *= -1
    d[ckind == 3] = 0.0
    d[(ckind == 1) | (ckind == 5)] = rng.uniform(-1, 1, int(((ckind == 1) | (ckind == 5)).sum()))
    c = A.T @ y + d
    if sense == -1:
        c = -c
    return mk(name, f"build: random general LP seed {seed} (feasible, dual feasible)", A, rl, rh,
              cl, ch, c, c0=c0, sense=sense)




def fixture_lp(cs) -> "O.GeneralLP":
    return O.GeneralLP(np.array(cs["A"], float).reshape(cs["m"], cs["n"]), cs["row_lo"],
                       cs["row_hi"], cs["col_lo"], cs["col_hi"], cs["c"], cs["c0"], cs["sense"])


def lp_arrays(lp):
    return (lp.A, lp.row_lo, lp.row_hi, lp.col_lo, lp.col_hi, lp.c, lp.c0, lp.sense)


def _num(v: float) -> str:
    return repr(float(v))


def write_mps(path, lp, rng=None, name="RANDLP"):
    """Write a general LP as free-format MPS with every section: OBJSENSE, ROWS
    (N/L/G/E), COLUMNS (two entries per line where possible), RHS (incl. an
    objective constant), RANGES (L/G/E rows, both E signs), BOUNDS (UP LO FX
    FR MI PL BV, with and without a set name).  Returns the general arrays the
    MPS semantics define (ranged bounds recomputed as rhs -+ |R|)."""
    rng = rng or np.random.default_rng(0)
    m, n = lp.A.shape
    rl, rh = lp.row_lo.copy(), lp.row_hi.copy()
    cl, ch = lp.col_lo.copy(), lp.col_hi.copy()
    lines = [f"NAME          {name}", "OBJSENSE", "    MAX" if lp.sense == -1 else "    MIN",
             "ROWS", " N  OBJ"]
    kinds, rhs, rng_v = [], [], []
    for i in range(m):
        lo, hi = rl[i], rh[i]
        if np.isfinite(lo) and np.isfinite(hi) and lo == hi:
            kinds.append("E"); rhs.append(lo); rng_v.append(None)
        elif np.isfinite(lo) and np.isfinite(hi):
            k = rng.integers(3)
            if k == 0:
                kinds.append("L"); rhs.append(hi); rng_v.append(hi - lo)
                rl[i] = hi - abs(hi - lo)
            elif k == 1:
                kinds.append("G"); rhs.append(lo); rng_v.append(-(hi - lo))
                rh[i] = lo + abs(hi - lo)
            else:
                kinds.append("E"); rhs.append(lo); rng_v.append(hi - lo)
                rh[i] = lo + abs(hi - lo)
        elif np.isfinite(hi):
            kinds.append("L"); rhs.append(hi); rng_v.append(None)
        elif np.isfinite(lo):
            kinds.append("G"); rhs.append(lo); rng_v.append(None)
        else:
            kinds.append("N"); rhs.append(0.0); rng_v.append(None)
        lines.append(f" {kinds[-1]}  R{i}")
    lines.append("COLUMNS")
    for j in range(n):
        ent = [("OBJ", lp.c[j])] if lp.c[j] != 0 else []
        ent += [(f"R{i}", lp.A[i, j]) for i in range(m) if lp.A[i, j] != 0]
        if not ent:
            ent = [("OBJ", 0.0)]
        for k in range(0, len(ent), 2):
            pair = ent[k:k + 2]
            lines.append(f"    X{j}  " + "  ".join(f"{r}  {_num(v)}" for r, v in pair))
    lines.append("RHS")
    if lp.c0 != 0:
        lines.append(f"    RHS  OBJ  {_num(-lp.c0)}")
    for i in range(m):
        if kinds[i] != "N" and rhs[i] != 0:
            lines.append(f"    RHS  R{i}  {_num(rhs[i])}")
    if any(v is not None for v in rng_v):
        lines.append("RANGES")
        for i in range(m):
            if rng_v[i] is not None:
                lines.append(f"    RNG  R{i}  {_num(rng_v[i])}")
    lines.append("BOUNDS")
    for j in range(n):
        lo, hi = cl[j], ch[j]
        setname = "BND  " if rng.integers(2) else ""
        if np.isfinite(lo) and np.isfinite(hi) and lo == hi:
            lines.append(f" FX {setname}X{j}  {_num(lo)}")
        elif lo == 0 and hi == 1 and rng.integers(2):
            lines.append(f" BV {setname}X{j}")
        elif not np.isfinite(lo) and not np.isfinite(hi):
            lines.append(f" FR {setname}X{j}")
        else:
            if not np.isfinite(lo):
                if np.isfinite(hi) and hi < 0 and rng.integers(2):
                    lines.append(f" UP {setname}X{j}  {_num(hi)}")   # UP < 0, lower 0 -> -inf
                    continue
                lines.append(f" MI {setname}X{j}")
            elif lo != 0:
                lines.append(f" LO {setname}X{j}  {_num(lo)}")
            if np.isfinite(hi):
                lines.append(f" UP {setname}X{j}  {_num(hi)}")
            elif rng.integers(2):
                lines.append(f" PL {setname}X{j}")
    lines.append("ENDATA")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    keep = [i for i in range(m) if kinds[i] != "N"]
    return (lp.A[keep], rl[keep], rh[keep], cl, ch, lp.c, lp.c0, lp.sense)
