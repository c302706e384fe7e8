"""Host restatements of single reference operations, for the kernel tests.

Each follows the reference function's operation order exactly (so results are
compared bit for bit):  mxm (amg_setup.c:1894), transpose (:2000), mpm (:1684),
mxmpoint (:1807), apply_M (amg_tools.c:76), min_skel (:2198), build_csr (:3612).
Pure Python -- small matrices only.
"""
import numpy as np

from omp_amg_amd.abi import Csr


def rand_csr(rng, rn, cn, density, ints=False, minrow=0):
    ro = [0]
    cols, vals = [], []
    for i in range(rn):
        k = max(minrow, rng.binomial(cn, density))
        c = np.sort(rng.choice(cn, size=min(k, cn), replace=False))
        v = rng.integers(-3, 4, size=len(c)).astype(float) if ints else rng.standard_normal(len(c))
        if ints:
            v[v == 0] = 1.0
        cols.extend(c.tolist())
        vals.extend(v.tolist())
        ro.append(len(cols))
    return Csr(rn, cn, np.array(ro, dtype=np.int64), np.array(cols, dtype=np.int64), np.array(vals))


def spgemm(A, B):
    ro, cols, vals = [0], [], []
    for i in range(A.rn):
        acc = {}
        s, e = A.row_off[i], A.row_off[i + 1]
        for ka in range(s, e):
            if ka + 1 < e and A.col[ka + 1] == A.col[ka]:
                continue
            k, av = A.col[ka], A.a[ka]
            for kb in range(B.row_off[k], B.row_off[k + 1]):
                j = B.col[kb]
                acc[j] = acc.get(j, 0.0) + B.a[kb] * av
        for j in sorted(acc):
            if acc[j] != 0.0:
                cols.append(j)
                vals.append(acc[j])
        ro.append(len(cols))
    return Csr(A.rn, B.cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))


def transpose(A):
    ent = []
    for i in range(A.rn):
        for k in range(A.row_off[i], A.row_off[i + 1]):
            ent.append((A.col[k], i, A.a[k]))
    ent.sort(key=lambda t: (t[0], t[1]))   # stable
    ro = np.zeros(A.cn + 1, dtype=np.int64)
    for c, _, _ in ent:
        ro[c + 1] += 1
    return Csr(A.cn, A.rn, np.cumsum(ro), np.array([t[1] for t in ent], dtype=np.int64),
               np.array([t[2] for t in ent]))


def mpm(alpha, A, beta, B):
    ro, cols, vals = [0], [], []
    for i in range(A.rn):
        ja, ea, jb, eb = A.row_off[i], A.row_off[i + 1], B.row_off[i], B.row_off[i + 1]
        while ja < ea or jb < eb:
            if ja < ea and jb < eb:
                if A.col[ja] == B.col[jb]:
                    s = alpha * A.a[ja] + beta * B.a[jb]
                    if s != 0.0:
                        cols.append(A.col[ja]); vals.append(s)
                    ja += 1; jb += 1
                elif A.col[ja] < B.col[jb]:
                    cols.append(A.col[ja]); vals.append(alpha * A.a[ja]); ja += 1
                else:
                    cols.append(B.col[jb]); vals.append(beta * B.a[jb]); jb += 1
            elif ja == ea:
                cols.append(B.col[jb]); vals.append(beta * B.a[jb]); jb += 1
            else:
                cols.append(A.col[ja]); vals.append(alpha * A.a[ja]); ja += 1
        ro.append(len(cols))
    return Csr(A.rn, A.cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))


def mxmpoint(A, B):
    ro, cols, vals = [0], [], []
    for i in range(A.rn):
        ja, ea, jb, eb = A.row_off[i], A.row_off[i + 1], B.row_off[i], B.row_off[i + 1]
        while ja < ea and jb < eb:
            if A.col[ja] == B.col[jb]:
                cols.append(A.col[ja]); vals.append(A.a[ja] * B.a[jb]); ja += 1; jb += 1
            elif A.col[ja] < B.col[jb]:
                ja += 1
            else:
                jb += 1
        ro.append(len(cols))
    return Csr(A.rn, A.cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))


def spmv(A, x, alpha=0.0, y=None, beta=1.0):
    z = np.zeros(A.rn)
    for i in range(A.rn):
        t = 0.0
        for k in range(A.row_off[i], A.row_off[i + 1]):
            t += A.a[k] * x[A.col[k]]
        z[i] = beta * t if (alpha == 0.0 or y is None) else alpha * y[i] + beta * t
    return z


def min_skel(R):
    ro = np.arange(R.rn + 1, dtype=np.int64)
    cols, vals = [], []
    for i in range(R.rn):
        ym, j = -np.finfo(float).max, 0
        for k in range(R.row_off[i], R.row_off[i + 1]):
            if R.a[k] > ym:
                ym, j = R.a[k], R.col[k]
        cols.append(j)
        vals.append(1.0 if ym > 0.0 else 0.0)
    return Csr(R.rn, R.cn, ro, np.array(cols, dtype=np.int64), np.array(vals))


def same(X, Y):
    return (X.rn == Y.rn and X.cn == Y.cn and np.array_equal(X.row_off, Y.row_off)
            and np.array_equal(X.col, Y.col)
            and np.array_equal(np.asarray(X.a).view(np.uint64), np.asarray(Y.a).view(np.uint64)))


def expand_pick(X):
    """expand_support's pick per row (amg_setup.c:1000-1115): |X| ranked by descending
    value, ties in column order (glibc qsort, stable); running sum of the nonzero
    values against half the total; the first N = 1 + #{sum - V < 0} ranks (capped at
    the row length) are picked.  Returns the picked pattern as a Csr of ones."""
    ro, cols = [0], []
    for i in range(X.rn):
        s, e = X.row_off[i], X.row_off[i + 1]
        v = np.abs(np.asarray(X.a[s:e]))
        order = sorted(range(e - s), key=lambda q: (-v[q], q))
        sv = [v[q] for q in order]
        tot = 0.0
        for x in sv:
            if x != 0.0:
                tot += x
        V = tot * 0.5
        c = 0
        if V != 0.0:
            run = 0.0
            for x in sv:
                if x != 0.0:
                    run += x
                if run - V < 0:
                    c += 1
        N = min(c + 1, e - s)
        picked = sorted(int(X.col[s + q]) for q in order[:N])
        cols.extend(picked)
        ro.append(len(cols))
    return Csr(X.rn, X.cn, np.array(ro), np.array(cols, dtype=np.int64), np.ones(len(cols)))
