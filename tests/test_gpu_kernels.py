"""Kernel-level parity of the HIP primitives against host restatements of the
reference operations (tests/refops.py), bit for bit, through the library's
test hooks (amgd_testapi.c)."""
import zlib

import numpy as np
import pytest

import refops
import omp_amg_amd as oa

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_spgemm_short_rows(seed):
    rng = np.random.default_rng(seed)
    A = refops.rand_csr(rng, 300, 200, 0.03, ints=(seed == 2))
    B = refops.rand_csr(rng, 200, 250, 0.03, ints=(seed == 2))
    X = oa.test_csr_op(0, A, B)
    assert refops.same(X, refops.spgemm(A, B))


@pytest.mark.parametrize("seed", [3, 4])
def test_spgemm_tiny_rows(seed):
    """rows of <= 32 products (k_sg_tiny, one thread per row, registers): duplicate A
    columns (last one wins), exact cancellation to zero (dropped), -0.0 products
    (the sum starts at +0.0), empty B rows, and rows just past the limit mixed in"""
    rng = np.random.default_rng(seed)
    rn, kn, cn = 2000, 300, 120
    Bro, Bcol, Ba = [0], [], []
    for k in range(kn):
        L = int(rng.integers(0, 9))
        c = np.sort(rng.choice(cn, size=L, replace=False))
        v = rng.integers(-2, 3, size=L).astype(float)
        v[v == 0] = -0.0
        Bcol += c.tolist(); Ba += v.tolist(); Bro.append(len(Bcol))
    Aro, Acol, Aa = [0], [], []
    for i in range(rn):
        L = int(rng.integers(0, 6 if i % 7 else 40))
        c = np.sort(rng.integers(0, kn, size=L))          # repeats: duplicate columns
        v = rng.integers(-2, 3, size=L).astype(float)
        v[v == 0] = -0.0
        Acol += c.tolist(); Aa += v.tolist(); Aro.append(len(Acol))
    A = refops.Csr(rn, kn, np.array(Aro), np.array(Acol), np.array(Aa))
    B = refops.Csr(kn, cn, np.array(Bro), np.array(Bcol), np.array(Ba))
    assert refops.same(oa.test_csr_op(0, A, B), refops.spgemm(A, B))


def test_spgemm_long_rows_and_cancellation():
    rng = np.random.default_rng(7)
    A = refops.rand_csr(rng, 40, 600, 0.5, ints=True)          # > 1024 products per row
    B = refops.rand_csr(rng, 600, 900, 0.05, ints=True)
    X = oa.test_csr_op(0, A, B)
    R = refops.spgemm(A, B)
    assert refops.same(X, R)


@pytest.mark.parametrize("sort", [1, 0])
def test_spgemm_dense_overflow_rows(sort):
    """rows with more than 4096 distinct columns: their products sorted by column (stable:
    ascending k within a column) and each column summed from +0 (sort=1, the default), or the
    one-block dense-slab kernel (sort=0)"""
    rng = np.random.default_rng(8)
    A = refops.rand_csr(rng, 12, 1500, 0.5)
    B = refops.rand_csr(rng, 1500, 7000, 0.02)
    R = refops.spgemm(A, B)
    for flat in (False, True):
        oa.route_stats(reset=True)
        oa.spgemm_dr_sort(sort)
        oa.spgemm_win(0)            # wide rows stay in the hash / dense bins (no windows)
        oa.spgemm_flat(flat)
        try:
            X = oa.test_csr_op(0, A, B)
        finally:
            oa.spgemm_dr_sort(-1)
            oa.spgemm_win(-1)
            oa.spgemm_flat(False)
        routes = oa.route_stats(reset=True)
        assert routes["sg_long"] > 0
        assert (routes["sg_drsort"] > 0) == bool(sort)
        assert refops.same(X, R)


@pytest.mark.parametrize("sort", [1, 0])
@pytest.mark.parametrize("case", ["cancel_dups", "kseq_wide", "empty_mix"])
def test_spgemm_dense_rows_sorted(case, sort):
    """dense rows with duplicate A columns (the last one wins), exact cancellation to +0 /
    -0 (dropped), rows of both k-sequential and flat products, dense rows next to empty and
    short rows: the sorted path against the host restatement, bit for bit"""
    rng = np.random.default_rng({"cancel_dups": 71, "kseq_wide": 72, "empty_mix": 73}[case])
    if case == "cancel_dups":
        A = refops.rand_csr(rng, 10, 900, 0.6, ints=True)
        B = refops.rand_csr(rng, 900, 9000, 0.01, ints=True)
        cols, vals, ro = [], [], [0]
        for i in range(A.rn):
            for k in range(A.row_off[i], A.row_off[i + 1]):
                cols.append(A.col[k]); vals.append(A.a[k])
                if k % 5 == 0:
                    cols.append(A.col[k]); vals.append(-A.a[k])
            ro.append(len(cols))
        A = refops.Csr(A.rn, A.cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))
    elif case == "kseq_wide":
        A = refops.rand_csr(rng, 16, 300, 0.5, ints=True)
        B = refops.rand_csr(rng, 300, 20000, 0.01, ints=True)
    else:
        A = refops.rand_csr(rng, 60, 1200, 0.02, ints=True)
        ro = A.row_off.copy()
        # rows 7 and 31 dense, row 8 emptied
        dense = {7: np.arange(0, 1200, 2), 31: np.arange(1, 1200, 3)}
        cols, vals, ro = [], [], [0]
        for i in range(A.rn):
            if i in dense:
                c = dense[i]
                v = rng.integers(-2, 3, size=c.size).astype(float)
            elif i == 8:
                c, v = np.array([], dtype=np.int64), np.array([])
            else:
                c = A.col[A.row_off[i]:A.row_off[i + 1]]
                v = A.a[A.row_off[i]:A.row_off[i + 1]]
            cols += list(c); vals += list(v); ro.append(len(cols))
        A = refops.Csr(A.rn, A.cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))
        B = refops.rand_csr(rng, 1200, 15000, 0.006, ints=True)
    R = refops.spgemm(A, B)
    for win in (0, -1):
        oa.route_stats(reset=True)
        oa.spgemm_dr_sort(sort)
        oa.spgemm_win(win)
        try:
            X = oa.test_csr_op(0, A, B)
        finally:
            oa.spgemm_dr_sort(-1)
            oa.spgemm_win(-1)
        routes = oa.route_stats(reset=True)
        if win == 0:
            assert routes["sg_long"] > 0 and (routes["sg_drsort"] > 0) == bool(sort)
        assert refops.same(X, R)


@pytest.mark.parametrize("win", [0, 4096, 8192, 16384])
@pytest.mark.parametrize("case", ["narrow", "wide", "dense_rows", "dups_cancel", "wide_span"])
def test_spgemm_kseq_long_b_rows(case, win):
    """k-sequential kernels (mean B row >= 64): every numeric bin incl. the dense slab,
    duplicate columns in A rows (last one wins) and exact cancellation; wide rows by the
    LDS hash (win 0) or the dense-accumulator column windows (several windows per row,
    A rows longer than one layer table)"""
    rng = np.random.default_rng({"narrow": 31, "wide": 32, "dense_rows": 33, "dups_cancel": 34,
                                 "wide_span": 35}[case])
    if case == "narrow":        # mean B row ~100: wave-sized blocks for the small bins
        A = refops.rand_csr(rng, 400, 300, 0.02)
        B = refops.rand_csr(rng, 300, 3000, 0.035)
    elif case == "wide":        # mean B row ~600: 256-thread blocks everywhere
        A = refops.rand_csr(rng, 200, 150, 0.04)
        B = refops.rand_csr(rng, 150, 6000, 0.1)
    elif case == "dense_rows":  # > 4096 distinct columns in some rows
        A = refops.rand_csr(rng, 20, 200, 0.3)
        B = refops.rand_csr(rng, 200, 9000, 0.05)
    elif case == "wide_span":   # ~300-entry A rows, outputs spanning 40000 columns
        A = refops.rand_csr(rng, 12, 600, 0.5, ints=True)
        B = refops.rand_csr(rng, 600, 40000, 0.007, ints=True)
    else:
        A = refops.rand_csr(rng, 150, 120, 0.05, ints=True)
        B = refops.rand_csr(rng, 120, 400, 0.3, ints=True)
        # duplicate a few A columns in place (sorted rows keep them adjacent)
        cols, vals, ro = [], [], [0]
        for i in range(A.rn):
            s, e = A.row_off[i], A.row_off[i + 1]
            for k in range(s, e):
                cols.append(A.col[k]); vals.append(A.a[k])
                if k % 7 == 0:
                    cols.append(A.col[k]); vals.append(A.a[k] + 1.0)
            ro.append(len(cols))
        A = refops.Csr(A.rn, A.cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))
    assert B.a.size >= 64 * B.rn
    R = refops.spgemm(A, B)
    oa.spgemm_flat(False)
    oa.spgemm_win(win)
    try:
        X = oa.test_csr_op(0, A, B)
    finally:
        oa.spgemm_win(-1)
    oa.spgemm_flat(True)
    try:
        Y = oa.test_csr_op(0, A, B)
    finally:
        oa.spgemm_flat(False)
    assert refops.same(X, R)
    assert refops.same(Y, R)


def _banded(rng, rn, kn, cn, width, dens, blen, span, ints=True, dups=False, empty_every=0):
    """A: row i holds k in [i*kn/rn, +width) at density dens (neighbouring rows share most
    k, like the Galerkin products' rows); B: rows of ~blen columns in a band of `span`"""
    ro, cols, vals = [0], [], []
    for i in range(rn):
        if empty_every and i % empty_every == 0:
            ro.append(len(cols))
            continue
        k0 = i * kn // rn
        ks = [k for k in range(k0, min(kn, k0 + width)) if rng.random() < dens]
        for k in ks:
            v = float(rng.integers(-3, 4)) if ints else rng.standard_normal()
            cols.append(k); vals.append(v)
            if dups and rng.random() < 0.1:          # duplicate column: the last one wins
                cols.append(k); vals.append(v + 1.0)
        ro.append(len(cols))
    A = refops.Csr(rn, kn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))
    ro, cols, vals = [0], [], []
    for k in range(kn):
        c0 = k * (cn - span) // max(1, kn - 1)
        c = np.sort(rng.choice(span, size=min(span, blen), replace=False)) + c0
        v = rng.integers(-3, 4, size=len(c)).astype(float) if ints else rng.standard_normal(len(c))
        cols += c.tolist(); vals += v.tolist(); ro.append(len(cols))
    B = refops.Csr(kn, cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))
    return A, B


@pytest.mark.parametrize("win", [0, 1024, 2048, 8192, -1])
@pytest.mark.parametrize("case", ["banded", "long_a", "dups_cancel", "ragged", "wide_span",
                                  "huge_a", "gapped", "dense_rows"])
def test_spgemm_wave_windows(case, win):
    """wave-private windowed kernel (k_sg_wwin: one wavefront per row, its own LDS window,
    no barrier per layer; 32768-column bit-map windows for the symbolic counts, 1024-column
    numeric windows) with every wide row routed to it (win > 0, at several routing
    widths), none (0: LDS hash kernels) or the default routing (-1): vs the host
    restatement, bit for bit -- rows of more than 64 layers (cursors in scratch),
    duplicate A columns, exact cancellation, empty rows, column clusters far apart
    (skipped windows), B-row runs past 64 entries inside one window"""
    rng = np.random.default_rng({"banded": 91, "long_a": 92, "dups_cancel": 93, "ragged": 94,
                                 "wide_span": 95, "huge_a": 96, "gapped": 97, "dense_rows": 98}[case])
    if case == "banded":
        A, B = _banded(rng, 301, 400, 6000, 60, 0.7, 150, 3000, ints=False)
    elif case == "long_a":
        A, B = _banded(rng, 70, 900, 8000, 400, 0.8, 100, 4000)
    elif case == "dups_cancel":
        A, B = _banded(rng, 157, 300, 5000, 50, 0.8, 160, 2500, dups=True)
    elif case == "ragged":
        A, B = _banded(rng, 203, 350, 7000, 90, 0.6, 120, 3500, empty_every=5)
    elif case == "wide_span":
        A, B = _banded(rng, 41, 500, 60000, 200, 0.7, 90, 30000)
    elif case == "huge_a":          # 1100-1300 layers per row: 18-21 chunks of 64
        A = refops.rand_csr(rng, 6, 1400, 0.85)
        B = refops.rand_csr(rng, 1400, 3000, 0.03)
    elif case == "gapped":
        A = refops.rand_csr(rng, 30, 300, 0.3, ints=True)
        B = refops.rand_csr(rng, 300, 6000, 0.02, ints=True)
        shift = np.array([0, 70000, 250000, 1000000])[B.col // 1500]
        B = refops.Csr(B.rn, 1006000, B.row_off, B.col + shift, B.a)
    else:                           # dense B rows: > 64 entries of one layer per window
        A = refops.rand_csr(rng, 20, 200, 0.3)
        B = refops.rand_csr(rng, 200, 9000, 0.2)
    assert B.a.size >= 64 * B.rn
    R = refops.spgemm(A, B)
    oa.spgemm_flat(False)
    oa.spgemm_win(win)
    oa.route_stats(reset=True)
    try:
        X = oa.test_csr_op(0, A, B)
    finally:
        oa.spgemm_win(-1)
    routes = oa.route_stats(reset=True)
    if win > 0:
        assert routes["sg_wwin"] > 0
    if win == 0:
        assert routes["sg_wwin"] == 0
    assert refops.same(X, R)


@pytest.mark.parametrize("case", ["flat", "banded", "dense_rows", "tiny"])
def test_spgemm_symbolic_reuse(case):
    """a product's symbolic phase kept (amgd_spgemm_sym_next(1)) and taken over by the next
    product on the same operand patterns with other values (the Galerkin Af*W after the
    interpolation loop's last one): the numeric kernels alone give mxm's bits, including
    sums that now cancel to an exact zero; operands of another pattern are refused by the
    pattern hash and the product runs in full"""
    rng = np.random.default_rng({"flat": 61, "banded": 62, "dense_rows": 63, "tiny": 64}[case])
    if case == "flat":
        A = refops.rand_csr(rng, 300, 200, 0.03, ints=True)
        B = refops.rand_csr(rng, 200, 250, 0.03, ints=True)
    elif case == "banded":
        A, B = _banded(rng, 301, 400, 6000, 60, 0.7, 150, 3000)
    elif case == "dense_rows":
        A = refops.rand_csr(rng, 20, 200, 0.3, ints=True)
        B = refops.rand_csr(rng, 200, 9000, 0.05, ints=True)
    else:
        A = refops.rand_csr(rng, 2000, 300, 0.005, ints=True)
        B = refops.rand_csr(rng, 300, 120, 0.03, ints=True)

    def revalue(M):
        v = rng.integers(-2, 3, size=M.a.size).astype(float)
        return refops.Csr(M.rn, M.cn, M.row_off, M.col, v)

    A2, B2 = revalue(A), revalue(B)
    st0 = oa.spgemm_sym_stats()
    oa.spgemm_sym(1)
    X1 = oa.test_csr_op(0, A, B)
    oa.spgemm_sym(2)
    X2 = oa.test_csr_op(0, A2, B2)
    st1 = oa.spgemm_sym_stats()
    assert refops.same(X1, refops.spgemm(A, B))
    assert refops.same(X2, refops.spgemm(A2, B2))
    assert st1["kept"] == st0["kept"] + 1 and st1["reused"] == st0["reused"] + 1
    # another pattern: one entry of A moved to a free column of its row
    col = A.col.copy()
    r = int(np.argmax(np.diff(A.row_off) > 0))
    k = int(A.row_off[r])
    free = sorted(set(range(A.cn)) - set(col[A.row_off[r]:A.row_off[r + 1]].tolist()))
    col[k] = free[0]
    o = slice(int(A.row_off[r]), int(A.row_off[r + 1]))
    order = np.argsort(col[o], kind="stable")
    col[o] = col[o][order]
    a3 = A.a.copy()
    a3[o] = a3[o][order]
    A3 = refops.Csr(A.rn, A.cn, A.row_off, col, a3)
    oa.spgemm_sym(1)
    oa.test_csr_op(0, A, B)
    oa.spgemm_sym(2)
    X3 = oa.test_csr_op(0, A3, B)
    st2 = oa.spgemm_sym_stats()
    assert refops.same(X3, refops.spgemm(A3, B))
    assert st2["reused"] == st1["reused"], "a kept state was taken by another pattern"
    oa.spgemm_sym(-1)


@pytest.mark.parametrize("case", ["short", "long_b", "wide", "tiny", "nonpositive"])
def test_spgemm_pattern(case):
    """amgd_spgemm_pattern (the constraint operator's pattern W_skel * W_skel'): operands
    with all values > 0 give exactly mxm's pattern (no sum can cancel), every stored value
    nonzero; any value <= 0 falls back to the full product (same bits as mxm)"""
    rng = np.random.default_rng({"short": 71, "long_b": 72, "wide": 73, "tiny": 74, "nonpositive": 75}[case])
    if case == "short":
        A, B = refops.rand_csr(rng, 400, 300, 0.02), refops.rand_csr(rng, 300, 350, 0.02)
    elif case == "long_b":
        A, B = refops.rand_csr(rng, 300, 200, 0.03), refops.rand_csr(rng, 200, 3000, 0.04)
    elif case == "wide":
        A, B = refops.rand_csr(rng, 60, 300, 0.3), refops.rand_csr(rng, 300, 9000, 0.03)
    elif case == "tiny":
        A, B = refops.rand_csr(rng, 3000, 500, 0.002), refops.rand_csr(rng, 500, 400, 0.006)
    else:
        A, B = refops.rand_csr(rng, 200, 150, 0.05, ints=True), refops.rand_csr(rng, 150, 300, 0.1, ints=True)
    if case != "nonpositive":
        A = refops.Csr(A.rn, A.cn, A.row_off, A.col, np.ones_like(A.a))
        B = refops.Csr(B.rn, B.cn, B.row_off, B.col, np.abs(B.a) + 0.5)
    R = refops.spgemm(A, B)
    X = oa.test_csr_op(20, A, B)
    assert np.array_equal(X.row_off, R.row_off) and np.array_equal(X.col, R.col)
    assert np.all(X.a != 0.0)
    if case == "nonpositive":
        assert refops.same(X, R)


@pytest.mark.parametrize("seed", [81, 82])
def test_cols_masked_is_transpose_of_rows_masked(seed):
    """R0 rows (expand_support): (rows_masked(Af, bad))' is built as cols_masked(Af', bad)
    -- the same entries in the same order as the transpose, short and long rows"""
    import ctypes as C
    rng = np.random.default_rng(seed)
    B = refops.rand_csr(rng, 700, 500, 0.02 if seed == 81 else 0.3)
    bad = (rng.random(B.rn) < 0.4).astype(np.uint8)
    Bm = refops.Csr(B.rn, B.cn, *_rows_masked(B, bad))
    R = refops.transpose(Bm)
    Bt = refops.transpose(B)
    L = oa.lib()
    L.amgd_test_cols_masked.argtypes = [C.POINTER(oa.HCsr), C.c_void_p, C.POINTER(oa.HCsr)]
    ha = oa._to_hcsr(Bt.row_off, Bt.col, Bt.a, Bt.rn, Bt.cn)
    hx = oa.HCsr()
    assert L.amgd_test_cols_masked(C.byref(ha), bad.ctypes.data, C.byref(hx)) == 0
    X = oa._from_hcsr(hx)
    assert refops.same(X, R)


def _rows_masked(B, m):
    ro, cols, vals = [0], [], []
    for i in range(B.rn):
        if m[i]:
            s, e = B.row_off[i], B.row_off[i + 1]
            cols += B.col[s:e].tolist(); vals += B.a[s:e].tolist()
        ro.append(len(cols))
    return np.array(ro), np.array(cols, dtype=np.int64), np.array(vals)


@pytest.mark.parametrize("case", ["wide", "dense_rows", "wide_span", "long_a_rows", "gapped"])
def test_spgemm_symbolic_windows(case):
    """symbolic pass of rows with many products: the wave-private 32768-column bit-map
    windows (k_sg_wwin MODE 2) -- several windows per row, A rows past 64 layers with
    cursors in scratch, column clusters far apart"""
    rng = np.random.default_rng({"wide": 51, "dense_rows": 52, "wide_span": 53, "long_a_rows": 54,
                                 "gapped": 55}[case])
    if case == "wide":
        A = refops.rand_csr(rng, 200, 150, 0.04)
        B = refops.rand_csr(rng, 150, 6000, 0.1)
    elif case == "dense_rows":
        A = refops.rand_csr(rng, 20, 200, 0.3)
        B = refops.rand_csr(rng, 200, 9000, 0.05)
    elif case == "wide_span":
        A = refops.rand_csr(rng, 12, 600, 0.5, ints=True)
        B = refops.rand_csr(rng, 600, 200000, 0.0015, ints=True)
    elif case == "gapped":      # column clusters far apart: windows with no column are skipped
        A = refops.rand_csr(rng, 30, 300, 0.3, ints=True)
        B = refops.rand_csr(rng, 300, 6000, 0.02, ints=True)
        shift = np.array([0, 70000, 250000, 1000000])[B.col // 1500]
        B = refops.Csr(B.rn, 1006000, B.row_off, B.col + shift, B.a)
    else:                       # 1100-1300 entries per A row
        A = refops.rand_csr(rng, 4, 1400, 0.85)
        B = refops.rand_csr(rng, 1400, 3000, 0.03)
    assert B.a.size >= 64 * B.rn
    R = refops.spgemm(A, B)
    oa.route_stats(reset=True)
    X = oa.test_csr_op(0, A, B)
    assert oa.route_stats(reset=True)["sg_wwin_sym"] > 0
    assert refops.same(X, R)


def test_spgemm_empty_rows():
    rng = np.random.default_rng(3)
    A = refops.rand_csr(rng, 50, 40, 0.02)
    B = refops.rand_csr(rng, 40, 30, 0.0)                        # B all empty
    X = oa.test_csr_op(0, A, B)
    assert X.nnz == 0 and X.rn == 50


@pytest.mark.parametrize("seed", [0, 1])
def test_transpose(seed):
    rng = np.random.default_rng(seed)
    A = refops.rand_csr(rng, 500, 300, 0.02)
    assert refops.same(oa.test_csr_op(1, A), refops.transpose(A))


@pytest.mark.parametrize("rn,cn,density", [(40, 20000, 0.0005), (3, 5000, 0.001), (30, 700, 0.0)])
def test_transpose_empty_column_runs(rn, cn, density):
    # row offsets come from the sorted column keys; runs of > 64 empty columns
    # (leading, trailing, interior) take the queued block-wide fill
    rng = np.random.default_rng(rn)
    A = refops.rand_csr(rng, rn, cn, density)
    assert refops.same(oa.test_csr_op(1, A), refops.transpose(A))


def test_mpm_and_mxmpoint():
    rng = np.random.default_rng(5)
    A = refops.rand_csr(rng, 200, 150, 0.05, ints=True)
    B = refops.rand_csr(rng, 200, 150, 0.05, ints=True)
    assert refops.same(oa.test_csr_op(2, A, B, 1.0, -1.0), refops.mpm(1.0, A, -1.0, B))
    assert refops.same(oa.test_csr_op(2, A, B, 1.0, 1.0), refops.mpm(1.0, A, 1.0, B))
    assert refops.same(oa.test_csr_op(3, A, B), refops.mxmpoint(A, B))


def test_mxmpoint_long_rows():
    """wave-per-row pointwise product (mean row >= 32): bisection + ballot placement on
    strictly increasing rows, lane 0's sequential merge on rows with a repeated or an
    unsorted column (the merge's own pairing), empty rows on either side"""
    rng = np.random.default_rng(17)
    rn, cn = 300, 2000

    def build(dens, tweak):
        ro, cols, vals = [0], [], []
        for i in range(rn):
            c = np.sort(rng.choice(cn, size=0 if i in (5, 6) and tweak == "a" else
                                   int(rng.binomial(cn, dens)), replace=False))
            if i == 7 and tweak == "b" and len(c) > 3:
                c[1] = c[0]                      # repeated column
            if i == 9 and tweak == "a" and len(c) > 3:
                c[0], c[1] = c[1], c[0]          # unsorted pair
            cols += c.tolist(); vals += rng.standard_normal(len(c)).tolist(); ro.append(len(cols))
        return refops.Csr(rn, cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))
    A, B = build(0.05, "a"), build(0.06, "b")
    assert A.row_off[-1] + B.row_off[-1] >= 32 * rn
    assert refops.same(oa.test_csr_op(3, A, B), refops.mxmpoint(A, B))
    assert refops.same(oa.test_csr_op(3, B, A), refops.mxmpoint(B, A))


def test_spmv_ordered():
    rng = np.random.default_rng(11)
    A = refops.rand_csr(rng, 1000, 800, 0.01)
    L = refops.rand_csr(rng, 300, 5000, 0.6)                     # long rows: direct path
    x = rng.standard_normal(800)
    y = rng.standard_normal(1000)
    assert np.array_equal(oa.test_spmv(A, x), refops.spmv(A, x))
    assert np.array_equal(oa.test_spmv(A, x, 1.0, y, -1.0), refops.spmv(A, x, 1.0, y, -1.0))
    xl = rng.standard_normal(5000)
    assert np.array_equal(oa.test_spmv(L, xl), refops.spmv(L, xl))


def _ragged_long_rows(rng):
    """mean row >= 32: ragged rows, empty rows, rows shorter and longer than the lane
    kernel's 16-entry rounds; 1037 rows, so 64-row groups end mid-wave"""
    rn, cn = 1000 + 37, 3000
    ro, cols, vals = [0], [], []
    for i in range(rn):
        k = int(rng.choice([0, 1, 15, 16, 17, 40, 63, 64, 65, 300, 1200]))
        c = np.sort(rng.choice(cn, size=k, replace=False))
        cols.extend(c.tolist())
        vals.extend((rng.standard_normal(k) * 10.0 ** rng.integers(-8, 8, size=k)).tolist())
        ro.append(len(cols))
    L = refops.Csr(rn, cn, np.array(ro, dtype=np.int64), np.array(cols, dtype=np.int64),
                   np.array(vals))
    assert L.a.size >= 32 * rn
    return L


def _rowsums(L):
    return refops.spmv(L, np.ones(L.cn))          # a*1.0 == a: the ordered row sums


@pytest.fixture(params=[-1, 4, 16, 64], ids=["rw_auto", "rw4", "rw16", "rw64"])
def rw(request):
    """rows per wavefront of the lane-per-row kernel (-1: chosen by row count)"""
    oa.spmv_rw(request.param)
    yield request.param
    oa.spmv_rw(-1)


@pytest.fixture(params=[0, 1], ids=["pipe", "pair"])
def chunk(request):
    """whole-matrix long-row products: per-row segments with the gather one round ahead
    (k_spmv_pipe, whole-matrix and listed rows); "pair": products with x through
    k_spmv_pair (two entries per 16 B load, rows walked from an even offset)"""
    oa.spmv_pair(request.param)
    yield request.param
    oa.spmv_pair(-1)


def _adversarial_rows(rng, rn=700):
    """rows built to break a parallel ordered sum: monotone positive sums crossing many
    binades, exact ties at the running sum's half-ulp, leading / interleaved zeros and
    -0, cancellation to exact zero mid-row, subnormals, huge magnitudes, mixed signs
    hovering around a binade edge, inf and nan"""
    ro, cols, vals = [0], [], []
    cn = 2000
    kinds = ["pos", "ties", "zeros", "cancel", "sub", "huge", "hover", "mixed", "inf"]
    for i in range(rn):
        kind = kinds[i % len(kinds)]
        L = int(rng.choice([1, 2, 63, 64, 65, 130, 257, 600]))
        if kind == "pos":
            v = np.abs(rng.standard_normal(L)) * 2.0 ** rng.integers(-3, 4, L)
        elif kind == "ties":
            v = np.where(rng.random(L) < 0.5, 2.0 ** -53, 1.0) * (1 + (rng.random(L) < 0.3))
            v[0] = 1.0
        elif kind == "zeros":
            v = np.where(rng.random(L) < 0.6, 0.0, rng.standard_normal(L))
            v[: L // 2] = -0.0
        elif kind == "cancel":
            h = rng.standard_normal((L + 1) // 2)
            v = np.concatenate([h, -h])[:L]
        elif kind == "sub":
            v = rng.standard_normal(L) * 2.0 ** -1070
        elif kind == "huge":
            v = rng.standard_normal(L) * 2.0 ** rng.integers(900, 1020, L)
        elif kind == "hover":
            v = np.where(rng.random(L) < 0.5, 1.0, -1.0) * 2.0 ** -52
            v[0] = 1.0
        elif kind == "mixed":
            v = rng.standard_normal(L) * 10.0 ** rng.integers(-12, 12, L)
        else:
            v = rng.standard_normal(L)
            v[L // 2] = np.inf if i % 2 else np.nan
        c = np.sort(rng.choice(cn, size=L, replace=False))
        cols.extend(c.tolist())
        vals.extend(v.tolist())
        ro.append(len(cols))
    return refops.Csr(rn, cn, np.array(ro, dtype=np.int64), np.array(cols, dtype=np.int64),
                      np.array(vals))


@pytest.fixture(params=[-1, 64], ids=["long4096", "long64"])
def mv_long(request):
    """listed products: rows past 4096 (default) / 64 entries take k_rows_exact"""
    oa.mv_long(request.param)
    yield request.param
    oa.mv_long(-1)


@pytest.mark.parametrize("sl_min", [1 << 40, 0], ids=["wave", "lane"])
def test_spmv_adversarial_rows(sl_min, rw, mv_long, chunk, resolve):
    """long-row SpMV / row sums / listed rows on adversarial rows through the wave-per-row
    and the lane-per-row kernels (every RW) and, for listed rows past the long-row
    threshold, the block-per-row binade scan, bit for bit against the sequential loop
    (nan compared as nan)"""
    A = _adversarial_rows(np.random.default_rng(77))
    with np.errstate(all="ignore"):
        want_s = _rowsums(A)
        x = np.where(np.random.default_rng(3).random(A.cn) < 0.5, 1.0, 0.5)
        want = refops.spmv(A, x)
    oa.spmv_sl_min(sl_min)
    try:
        got_s = oa.test_spmv_f(A, None)
        got = oa.test_spmv(A, x)
        rows = np.arange(A.rn, dtype=np.uint32)[::-1].copy()
        got_l = oa.test_spmv_rows(A, rows, x, np.zeros(A.rn))
        got_ls = oa.test_spmv_rows(A, rows, None, np.zeros(A.rn))
    finally:
        oa.spmv_sl_min(-1)
    for g, w in ((got_s, want_s), (got, want), (got_l, want), (got_ls, want_s)):
        assert np.array_equal(g.view(np.uint64), w.view(np.uint64)) or \
            np.array_equal(np.isnan(g), np.isnan(w)) and np.array_equal(g[~np.isnan(g)].view(np.uint64),
                                                                       w[~np.isnan(w)].view(np.uint64))


def test_spmv_rows_multichunk_exact(resolve):
    """listed rows of 4097 - 130000 entries (many 4096-entry chunks each) through the
    grid-wide speculation + per-row resolve: sums growing across binades, exact ties,
    cancellation to zero, mixed magnitudes, an inf -- bit for bit the sequential loop,
    listed in any order and beside short rows"""
    rng = np.random.default_rng(61)
    cn = 200000
    lens = [4097, 9000, 50000, 130000, 5, 70000, 8193, 0, 20000]
    ro, cols, vals = [0], [], []
    for q, L in enumerate(lens):
        kind = q % 5
        if kind == 0:
            v = np.abs(rng.standard_normal(L)) * 2.0 ** rng.integers(-3, 4, L)
        elif kind == 1:
            v = np.where(rng.random(L) < 0.5, 2.0 ** -53, 1.0) * (1 + (rng.random(L) < 0.3))
        elif kind == 2:
            h = rng.standard_normal((L + 1) // 2)
            v = np.concatenate([h, -h])[:L]
        elif kind == 3:
            v = rng.standard_normal(L) * 10.0 ** rng.integers(-12, 12, L)
        else:
            v = rng.standard_normal(L)
            if L > 10:
                v[L // 3] = np.inf
        c = np.sort(rng.choice(cn, size=L, replace=False))
        cols.extend(c.tolist())
        vals.extend(v.tolist())
        ro.append(len(cols))
    A = refops.Csr(len(lens), cn, np.array(ro, dtype=np.int64), np.array(cols, dtype=np.int64),
                   np.array(vals))
    x = np.where(rng.random(cn) < 0.5, 1.0, 0.75)
    with np.errstate(all="ignore"):
        want = refops.spmv(A, x)
        want_s = _rowsums(A)
    rows = np.array([3, 0, 8, 5, 2, 7, 1, 6, 4], dtype=np.uint32)
    z0 = np.full(A.rn, -7.25)
    got = oa.test_spmv_rows(A, rows, x, z0)
    got_s = oa.test_spmv_rows(A, rows, None, z0)
    for g, w in ((got, want), (got_s, want_s)):
        assert np.array_equal(g.view(np.uint64), w.view(np.uint64)), np.nonzero(g != w)


@pytest.mark.parametrize("sl_min", [1 << 40, 0], ids=["wave", "lane"])
def test_spmv_long_rows_ragged(sl_min, rw, chunk):
    """long-row SpMV kernels on ragged rows: wave-per-row (default below 2^20 rows) and
    lane-per-row (forced with the row threshold at 0), with and without y, the f row
    mask and x = NULL (ordered row sums)"""
    rng = np.random.default_rng(31)
    L = _ragged_long_rows(np.random.default_rng(23))
    rn, cn = L.rn, L.cn
    x = rng.standard_normal(cn)
    y = rng.standard_normal(rn)
    f = (rng.random(rn) < 0.7).astype(np.uint8)
    oa.spmv_sl_min(sl_min)
    try:
        assert np.array_equal(oa.test_spmv(L, x), refops.spmv(L, x))
        assert np.array_equal(oa.test_spmv(L, x, 1.0, y, -1.0), refops.spmv(L, x, 1.0, y, -1.0))
        assert np.array_equal(oa.test_spmv_f(L, x, 1.0, y, -1.0, f),
                              refops.spmv(L, x, 1.0, y, -1.0) * (f != 0))
        assert np.array_equal(oa.test_spmv_f(L, None), _rowsums(L))
    finally:
        oa.spmv_sl_min(-1)


@pytest.mark.parametrize("sl_min", [1 << 40, 0], ids=["wave", "lane"])
def test_spmv_rows_listed(sl_min, rw, mv_long, chunk):
    """listed-row products (amgd_spmv_rows): wave-per-row list kernel below the row
    threshold, lane-per-row k_spmv_pipe<true> with it forced to 0; unlisted rows untouched"""
    rng = np.random.default_rng(29)
    L = _ragged_long_rows(np.random.default_rng(23))
    x = rng.standard_normal(L.cn)
    rows = np.sort(rng.choice(L.rn, size=700, replace=False)).astype(np.uint32)
    rows = np.concatenate([rows[1::2], rows[::2]])               # unsorted list
    z0 = np.full(L.rn, -7.25)
    want = z0.copy()
    want[rows] = refops.spmv(L, x)[rows]
    want_s = z0.copy()
    want_s[rows] = _rowsums(L)[rows]
    oa.spmv_sl_min(sl_min)
    try:
        assert np.array_equal(oa.test_spmv_rows(L, rows, x, z0), want)
        assert np.array_equal(oa.test_spmv_rows(L, rows, None, z0), want_s)
    finally:
        oa.spmv_sl_min(-1)


def test_min_skel():
    rng = np.random.default_rng(4)
    R = refops.rand_csr(rng, 300, 100, 0.03)
    R.a = np.abs(R.a)
    R.a[::7] = 0.0
    assert refops.same(oa.test_csr_op(4, R), refops.min_skel(R))


def test_build_csr_drops_zeros_and_empty_rows():
    rng = np.random.default_rng(9)
    n = 60
    I = rng.integers(0, n, 400).astype(np.uint32)
    J = rng.integers(0, n, 400).astype(np.uint32)
    key = np.unique(I.astype(np.int64) * n + J)
    I, J = (key // n).astype(np.uint32), (key % n).astype(np.uint32)
    V = rng.standard_normal(len(I))
    V[::9] = 0.0
    perm = rng.permutation(len(I))
    X = oa.test_build(I[perm], J[perm], V[perm])
    # host restatement of build_csr (amg_setup.c:3612)
    keep = V != 0
    rn = int(I.max()) + 1
    rows = np.zeros(rn, bool)
    rows[I[keep]] = True
    newid = np.cumsum(rows) - 1
    m = keep & rows[J] if J.max() < rn else keep
    order = np.lexsort((J[m], I[m]))
    ii, jj, vv = I[m][order], J[m][order], V[m][order]
    ro = np.zeros(rows.sum() + 1, dtype=np.int64)
    np.add.at(ro, newid[ii] + 1, 1)
    assert np.array_equal(X.row_off, np.cumsum(ro))
    assert np.array_equal(X.col, newid[jj])
    assert np.array_equal(X.a, vv)


def test_device_math_is_ieee():
    """sqrt, 1/x and x/y must round like the host (the reference's sqrt/div)."""
    rng = np.random.default_rng(0)
    a = np.abs(rng.standard_normal(100000)) * 10.0 ** rng.integers(-30, 30, 100000)
    b = rng.standard_normal(100000) * 10.0 ** rng.integers(-30, 30, 100000)
    assert np.array_equal(oa.test_math(0, a), np.sqrt(a))
    assert np.array_equal(oa.test_math(1, a), 1.0 / a)
    assert np.array_equal(oa.test_math(2, a, b), a / b)


def _seq(p):
    s = 0.0
    for x in p.tolist():
        s += x
    return s


@pytest.fixture(params=[1, 0, 2], ids=["wave_resolve", "block_resolve", "block_nosplit"])
def resolve(request):
    """the speculation's resolution walk: one wavefront per sum, one block (default) with the
    long rows' split records, or one block without them"""
    oa.resolve_wave(1 if request.param == 1 else 0)
    oa.seg_split(0 if request.param == 2 else 1)
    yield request.param
    oa.resolve_wave(-1)
    oa.seg_split(-1)


def test_spmv_rows_binade_jumps(resolve):
    """long listed rows whose running sum jumps into higher binades now and then (the
    anisotropic orphan rows: a strong entry ~10^3 x the sum so far), jumps at and next to
    512-entry chunk boundaries, two jumps in one chunk, negative sums, a jump that lands on
    a tie: the split records (one crossing per chunk, O(1)) and the binade scan give the
    sequential loop's bits"""
    rng = np.random.default_rng(97)
    cn = 400000
    rows = []
    for q in range(8):
        L = int(rng.integers(20000, 140000))
        v = np.abs(rng.standard_normal(L)) * 1e-3
        pos = np.sort(rng.choice(L, size=max(4, L // 700), replace=False))
        if q == 1:
            pos = np.unique(np.concatenate([pos, [511, 512, 1023, 1024, 1535, 1600]]))
        if q == 2:
            pos = np.unique(np.concatenate([pos, [5000, 5100, 5200]]))   # several in one chunk
        run = 0.0
        last = 0
        for t, p in enumerate(pos):
            run += v[last:p].sum()
            if t % 2 == 0:                            # up: ~10^3 x the sum so far
                v[p] = (run + 1e-3) * rng.uniform(500.0, 3000.0)
            else:                                     # down again (no overflow over many jumps)
                v[p] = -run * (1.0 - 1.0 / rng.uniform(500.0, 3000.0))
            run += v[p]
            last = p + 1
        if q == 3:
            v = -v
        if q == 4:
            v[pos[len(pos) // 2]] = 2.0 ** 40        # exact power of two: ties near the jump
            v[pos[len(pos) // 2] + 1: pos[len(pos) // 2] + 50] = 2.0 ** -13
        rows.append(v)
    ro, cols, vals = [0], [], []
    for v in rows:
        c = np.sort(rng.choice(cn, size=v.size, replace=False))
        cols.extend(c.tolist()); vals.extend(v.tolist()); ro.append(len(cols))
    A = refops.Csr(len(rows), cn, np.array(ro, dtype=np.int64), np.array(cols, dtype=np.int64),
                   np.array(vals))
    x = np.where(rng.random(cn) < 0.5, 1.0, 0.75)
    want = refops.spmv(A, x)
    want_s = _rowsums(A)
    order = np.arange(A.rn, dtype=np.uint32)[::-1].copy()
    oa.mv_long(64)                    # every listed row past 64 entries: the exact grid path
    try:
        got = oa.test_spmv_rows(A, order, x, np.zeros(A.rn))
        got_s = oa.test_spmv_rows(A, order, None, np.zeros(A.rn))
    finally:
        oa.mv_long(-1)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    assert np.array_equal(got_s.view(np.uint64), want_s.view(np.uint64))


@pytest.mark.parametrize("kind", ["normal", "positive", "ints", "ties", "zeros", "range", "cancel",
                                  "hover", "big", "pos_big", "spikes", "jumps"])
def test_exact_dot_matches_sequential(kind, resolve):
    """The binade-parallel exact sum (single block below 64K products, chunk
    speculation over all CUs above, resolved by one wavefront or one block) equals the
    left-to-right loop bit for bit."""
    rng = np.random.default_rng(zlib.crc32(kind.encode()))
    n = 3000000 if kind in ("big", "pos_big", "spikes", "jumps") else 300000
    if kind == "normal":
        a, b = rng.standard_normal(n), rng.standard_normal(n)
    elif kind == "positive":
        a = np.abs(rng.standard_normal(n)); b = a.copy()
    elif kind == "ints":
        a, b = rng.integers(-5, 6, n).astype(float), rng.integers(-5, 6, n).astype(float)
    elif kind == "ties":
        a = np.ones(n); a[0] = 2.0 ** 53; b = np.ones(n)
    elif kind == "zeros":
        a = rng.standard_normal(n); a[: n // 2] = 0.0; a[n // 2 + 5: n // 2 + 9000] = 0.0; b = rng.standard_normal(n)
    elif kind == "hover":     # running sum crosses the binade boundary at 1.0 again and again
        a = rng.choice([-1.0, 1.0], n) * 2.0 ** -30; a[0] = 1.0; b = np.ones(n)
    elif kind == "big":       # more chunks than one record batch
        a, b = rng.standard_normal(n) + 0.01, rng.standard_normal(n) + 0.02
    elif kind == "pos_big":   # monotone sum: binade crossings inside chunks, long passing runs
        a = np.abs(rng.standard_normal(n)) + 1e-3; b = np.abs(rng.standard_normal(n)) + 1e-3
    elif kind == "spikes":    # products far above the running sum now and then (huge grid steps)
        a = rng.standard_normal(n) * 1e-6; a[rng.integers(0, n, 40)] = 1e12; b = np.ones(n)
    elif kind == "jumps":     # one binade jump (up or back down) in most 4096-chunks, some on the
        # chunk's first / last product: the dots' split records, O(1) per chunk
        a = np.abs(rng.standard_normal(n)) * 1e-3
        pos = np.concatenate([np.arange(1, 73) * 4096 + rng.integers(0, 4096, 72), [4096 * 80, 4096 * 81 - 1]])
        run = 0.0
        last = 0
        for t, p in enumerate(np.sort(pos)):
            run += a[last:p].sum()
            a[p] = (run + 1e-3) * rng.uniform(2.0, 3000.0) if t % 3 != 2 else -run * (1.0 - 1.0 / rng.uniform(2.0, 50.0))
            run += a[p]
            last = p + 1
        b = np.ones(n)
    elif kind == "range":
        a = rng.standard_normal(n) * 10.0 ** rng.integers(-40, 40, n); b = rng.standard_normal(n)
    else:
        a = rng.standard_normal(n); a[1::2] = -a[::2][: len(a[1::2])]; b = np.ones(n)
    for mode in (0, 1, 2):
        if mode == 0:
            ref = _seq(a * b)
        elif mode == 1:
            ref = _seq(a * a)
        else:
            ref = _seq((a * b) * b)
        got = oa.test_dot(mode, a, b)
        plain = oa.test_dot(mode, a, b, plain=True)
        assert np.float64(got).view(np.uint64) == np.float64(ref).view(np.uint64), (mode, got, ref)
        assert np.float64(plain).view(np.uint64) == np.float64(ref).view(np.uint64), (mode, plain, ref)


@pytest.mark.parametrize("n", [4096, 4097, 8191, 20000, 65535, 65536])
def test_exact_dot_short_speculation(n):
    """the chunk speculation forced down to one-chunk dots (dot_spec_min(1)), with and without
    the split records: the left-to-right loop's bits on sums that cross binades in most chunks"""
    rng = np.random.default_rng(n)
    a = np.abs(rng.standard_normal(n)) + 1e-3
    a[rng.integers(0, n, 6)] *= 1e4
    b = rng.standard_normal(n)
    oa.dot_spec_min(1)
    try:
        for split in (1, 0):
            oa.dot_split(split)
            for mode, ref in ((0, _seq(a * b)), (1, _seq(a * a)), (2, _seq((a * b) * b))):
                got = oa.test_dot(mode, a, b)
                assert np.float64(got).view(np.uint64) == np.float64(ref).view(np.uint64), (split, mode, got, ref)
    finally:
        oa.dot_spec_min(-1)
        oa.dot_split(-1)


def _dup_cols(A, rng, frac=0.1):
    """duplicate some entries of A's rows (the reference's mxm: the last one wins)"""
    ro, cols, vals = [0], [], []
    for i in range(A.rn):
        for k in range(A.row_off[i], A.row_off[i + 1]):
            cols.append(A.col[k]); vals.append(A.a[k])
            if rng.random() < frac:
                cols.append(A.col[k]); vals.append(rng.standard_normal())
        ro.append(len(cols))
    return refops.Csr(A.rn, A.cn, np.array(ro), np.array(cols, dtype=np.int64), np.array(vals))


@pytest.mark.parametrize("case", ["short_b_rows", "block_bin", "sym_overflow", "dups"])
def test_spgemm_row_bins(case):
    """every row bin of the SpGEMM: wave hashes of 512/2048/4096 slots, the
    256-thread 8192-slot hash, symbolic overflow to the dense slab, long A rows
    over short B rows (many k layers per chunk), duplicate A columns"""
    rng = np.random.default_rng({"short_b_rows": 11, "block_bin": 12, "sym_overflow": 13,
                                 "dups": 14}[case])
    if case == "short_b_rows":        # Af*W shape: long A rows, 1..6 entries per B row
        A = refops.rand_csr(rng, 120, 3000, 0.3)
        B = refops.rand_csr(rng, 3000, 5000, 0.0007, minrow=1)
    elif case == "block_bin":         # 2048 < distinct <= 4096
        A = refops.rand_csr(rng, 24, 2000, 0.5, ints=True)
        B = refops.rand_csr(rng, 2000, 3000, 0.013, ints=True)
    elif case == "sym_overflow":      # > 8192 distinct: symbolic overflow, dense slab
        A = refops.rand_csr(rng, 6, 1000, 0.4)
        B = refops.rand_csr(rng, 1000, 20000, 0.02)
    else:
        A = _dup_cols(refops.rand_csr(rng, 80, 900, 0.2, ints=True), rng)
        B = refops.rand_csr(rng, 900, 1200, 0.01, ints=True)
    assert refops.same(oa.test_csr_op(0, A, B), refops.spgemm(A, B))


def _oracle_qfactor(W, A):
    import ctypes as C
    import os
    lib = C.CDLL(os.path.join(os.path.dirname(__file__), "..", "oracle", "build", "liboracle.so"))
    nzs = np.diff(W.row_off)
    Q = np.zeros(int((nzs * (nzs + 1) // 2).sum()) + 1)
    wro = np.ascontiguousarray(W.row_off, dtype=np.uint64)
    wcol = np.ascontiguousarray(W.col, dtype=np.uint32)
    aro = np.ascontiguousarray(A.row_off, dtype=np.uint64)
    acol = np.ascontiguousarray(A.col, dtype=np.uint32)
    aa = np.ascontiguousarray(A.a, dtype=np.float64)
    lib.oracle_qfactor(C.c_uint32(W.rn), wro.ctypes.data_as(C.c_void_p), wcol.ctypes.data_as(C.c_void_p),
                       C.c_uint32(A.rn), aro.ctypes.data_as(C.c_void_p), acol.ctypes.data_as(C.c_void_p),
                       aa.ctypes.data_as(C.c_void_p), Q.ctypes.data_as(C.c_void_p))
    return Q[:-1]


def _qfactor_case(structure):
    from omp_amg_amd import problems
    m = 20
    Ai, Aj, Av = problems.poisson3d(m, 27)
    o = np.lexsort((Aj, Ai))
    aro, acol, aa = problems.coo_to_csr_np(np.asarray(Ai)[o], np.asarray(Aj)[o], np.asarray(Av)[o])
    A = refops.Csr(m ** 3, m ** 3, aro, acol, aa)
    rng = np.random.default_rng(21)
    ro, cols = [0], []
    if structure == "tiers":
        sizes = [1, 5, 31, 32, 33, 40, 64, 65, 100, 128, 129, 256, 257, 300, 512, 513, 1024, 1025, 1400]
        for nz in sizes:
            lo = int(rng.integers(0, m ** 3 - 3 * nz))
            c = np.sort(rng.choice(np.arange(lo, lo + 3 * nz), size=nz, replace=False))
            cols.extend(c.tolist())
            ro.append(len(cols))
    elif structure == "blocks":                # huge supports made of disjoint components
        blk = lambda a, n: np.arange(a, a + n)
        for parts in ([blk(400, 500), blk(4000, 600)],                  # two tier-sized ones
                      [blk(800, 1300), blk(4400, 1200), np.arange(7000, 7600, 9)],
                      [blk(0, 300), np.arange(1000, 3000, 2), blk(5000, 200)]):
            c = np.unique(np.concatenate(parts))
            cols.extend(c.tolist()); ro.append(len(cols))
        for nz in (20, 700):                   # ordinary tiers beside them
            c = np.sort(rng.choice(np.arange(m ** 3), size=nz, replace=False))
            cols.extend(c.tolist()); ro.append(len(cols))
    else:                                      # huge supports only
        if structure == "scattered":           # isolated points: a diagonal Gram matrix
            c = np.sort(rng.choice(np.arange(0, m ** 3, 7), size=1100, replace=False))
            cols.extend(c.tolist()); ro.append(len(cols))
        c = np.arange(2000, 3300)              # a contiguous block: fill-in
        cols.extend(c.tolist()); ro.append(len(cols))
        c = np.sort(rng.choice(np.arange(m ** 3), size=1500, replace=False))
        cols.extend(c.tolist()); ro.append(len(cols))
    ro.append(len(cols))                      # one empty support
    W = refops.Csr(len(ro) - 1, m ** 3, np.array(ro), np.array(cols, dtype=np.int64),
                   np.ones(len(cols)))
    return W, A


@pytest.mark.parametrize("structure,mode,coop_lds", [("tiers", 1, -1), ("tiers", 0, -1),
                                                     ("scattered", 1, -1), ("scattered", 2, -1),
                                                     ("scattered", 0, -1), ("scattered", 0, 0),
                                                     ("scattered", 2, 1200)])
def test_qfactor_tiers_bitexact(structure, mode, coop_lds):
    """Q factors for supports in every tier (LDS 32 / 64 / 128 / block / huge) against
    the oracle's restatement of interp's Q loop, bit for bit.  Huge supports run the
    sparse kernel (mode 1), the dense cooperative kernel (mode 0), or the sparse
    kernel with a capacity too small to finish, which must hand over to the dense one.
    coop_lds: supports above it run the dense kernel's global-memory variant (the one
    supports past 8192 points take).  Component splitting is off here (see
    test_qfactor_split_bitexact)"""
    W, A = _qfactor_case(structure)
    oa.qf_sparse(mode)
    oa.qf_coop_lds(coop_lds)
    oa.qf_split(0)
    oa.qf_stats()
    try:
        X = oa.test_csr_op(5, W, A)
    finally:
        oa.qf_sparse(1)
        oa.qf_coop_lds(-1)
        oa.qf_split(-1)
    st = oa.qf_stats()
    nhuge = int((np.diff(W.row_off) > 1024).sum())
    if mode == 0:
        assert st == {"sparse": 0, "fallback": 0, "split": 0}
    elif mode == 2:
        assert st == {"sparse": 0, "fallback": nhuge, "split": 0}
    else:
        assert st["sparse"] + st["fallback"] == nhuge and st["sparse"] > 0, st
    ref = _oracle_qfactor(W, A)
    assert X.nnz == len(ref)
    assert np.array_equal(X.a.view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("structure,mode", [("blocks", 1), ("blocks", 0), ("blocks", 2),
                                            ("scattered", 1), ("tiers", 1)])
def test_qfactor_split_bitexact(structure, mode):
    """huge supports whose Gram matrix is block-diagonal (several connected components
    of A on the support) are factored per component -- through the ordinary tiers, or
    the huge kernels for components past 1024 points -- and scattered into a -0-filled
    triangle: bit for bit the oracle's one sequential factor, cross-component -0 included.
    'blocks' holds two-, three- and many-component supports; 'scattered' a diagonal one
    (1100 components) and a random one; a single-component support stays whole.
    mode: 1 automatic (components up to 8192 points dense), 0 dense, 2 forced sparse"""
    W, A = _qfactor_case(structure)
    oa.qf_sparse(mode)
    oa.qf_split(1)
    oa.qf_stats()
    try:
        X = oa.test_csr_op(5, W, A)
    finally:
        oa.qf_sparse(1)
        oa.qf_split(-1)
    st = oa.qf_stats()
    if structure == "blocks":                # 2 + 3 + 69 components; 1300 / 1200 stay huge,
        # factored dense unless a sparse mode is forced (mode 2: sparse, then the fallback)
        assert st["split"] == 3 and st["sparse"] + st["fallback"] == (2 if mode == 2 else 0), st
    elif structure == "scattered":
        assert st["split"] >= 1, st
    ref = _oracle_qfactor(W, A)
    assert X.nnz == len(ref)
    assert np.array_equal(X.a.view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("structure,split", [("tiers", 0), ("blocks", 1)])
def test_qfactor_blocked_tiers_bitexact(structure, split):
    """the blocked tiers (256 / 512 / 1024 points), bit for bit the oracle"""
    W, A = _qfactor_case(structure)
    oa.qf_split(split)
    oa.route_stats(reset=True)
    try:
        X = oa.test_csr_op(5, W, A)
    finally:
        oa.qf_split(-1)
    if structure == "tiers":
        r = oa.route_stats(reset=True)
        assert r["qf_t512"] > 0 and r["qf_t1024"] > 0, r
    ref = _oracle_qfactor(W, A)
    assert X.nnz == len(ref)
    assert np.array_equal(X.a.view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("structure", ["tiers", "scattered"])
def test_qapply_huge_grid_path(structure):
    """Q application of huge supports by the grid-wide kernels (threshold lowered to 600
    points) equals the one-work-group path bit for bit (default threshold 8192)"""
    W, A = _qfactor_case(structure)
    X1 = oa.test_csr_op(7, W, A)
    oa.qa_huge(600)
    try:
        X2 = oa.test_csr_op(7, W, A)
    finally:
        oa.qa_huge(-1)
    assert int((np.diff(W.row_off) > 600).sum()) > 0
    assert np.array_equal(X1.a.view(np.uint64), X2.a.view(np.uint64))


@pytest.mark.parametrize("tile", [16, 32])
def test_qapply_lds_tiles(tile):
    """Q application of 33..512-point supports with U staged through LDS in 64 x tile
    tiles equals the row-per-lane kernel bit for bit (every tier size, a partial last
    row group, an empty support)"""
    W, A = _qfactor_case("tiers")
    oa.qa_tile(0)
    try:
        X1 = oa.test_csr_op(7, W, A)
        oa.qa_tile(tile)
        X2 = oa.test_csr_op(7, W, A)
    finally:
        oa.qa_tile(-1)
    assert np.array_equal(X1.a.view(np.uint64), X2.a.view(np.uint64))


@pytest.mark.parametrize("case", ["short", "long", "ties", "over_lds"])
def test_expand_pick(case):
    """expand_support's per-row pick: short rows (rank-count kernel), long rows (LDS
    bitonic sort), tied values (stable order), rows past the LDS sort capacity"""
    rng = np.random.default_rng({"short": 41, "long": 42, "ties": 43, "over_lds": 44}[case])
    if case == "short":
        X = refops.rand_csr(rng, 300, 200, 0.04)
    elif case == "long":
        X = refops.rand_csr(rng, 60, 5000, 0.05, minrow=70)
    elif case == "ties":
        X = refops.rand_csr(rng, 80, 3000, 0.05, ints=True, minrow=70)
    else:
        X = refops.rand_csr(rng, 6, 9000, 0.5)
        X.a[::5] = 0.0
    assert oa.test_csr_op(6, X).nnz == refops.expand_pick(X).nnz
    assert refops.same(oa.test_csr_op(6, X), refops.expand_pick(X))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_mpm_long_rows_rank_placement(seed):
    """rows of >= 64 merged entries take the wave-per-row rank placement:
    disjoint, overlapping and cancelling (exact-zero dropped) entries, short rows
    mixed in, and a row with a repeated column (left to the sequential merge); seed 2:
    rows of 1 000 - 5 000 entries, around the 2048 columns staged in LDS for the searches"""
    rng = np.random.default_rng(seed)
    if seed == 2:
        A = refops.rand_csr(rng, 60, 30000, 0.1, ints=True)
        C = refops.rand_csr(rng, 60, 30000, 0.05, ints=True)
    else:
        A = refops.rand_csr(rng, 300, 3000, 0.03, ints=True)
        C = refops.rand_csr(rng, 300, 3000, 0.03, ints=True)
    # B: A's pattern, half the values equal (A - B cancels there), plus C's entries
    a2 = A.a.copy()
    flip = rng.random(len(a2)) < 0.5
    a2[flip] += 1.0
    B = refops.Csr(A.rn, A.cn, A.row_off.copy(), A.col.copy(), a2)
    BC = refops.mpm(1.0, B, 1.0, C)
    for (x, al, y, be) in [(A, 1.0, C, 1.0), (A, 1.0, A, -1.0), (A, 1.0, BC, -1.0),
                           (BC, 2.0, A, 0.5)]:
        assert refops.same(oa.test_csr_op(2, x, y, al, be), refops.mpm(al, x, be, y))
    # a repeated column in one long row
    col = A.col.copy()
    s, e = A.row_off[7], A.row_off[8]
    if e - s >= 2:
        col[s + 1] = col[s]
    D = refops.Csr(A.rn, A.cn, A.row_off.copy(), col, A.a.copy())
    assert refops.same(oa.test_csr_op(2, D, C, 1.0, -1.0), refops.mpm(1.0, D, -1.0, C))


def _tab_matrix(rng, rn, cn, mean, far_every=0):
    """long rows clustered around their diagonal position (a band of ~1200 columns, like
    a coarse level's R), ragged lengths, some empty rows; every (40 far_every)-th row also
    takes 8000 columns across the whole range (its tile has too many distinct columns for
    the gather table: it runs the direct gathers)"""
    ro, cols = [0], []
    for i in range(rn):
        L = 0 if i % 97 == 5 else int(rng.integers(mean // 2, 3 * mean // 2 + 1))
        L = min(L, cn)
        c0 = int(i * cn / rn)
        band = np.arange(max(0, c0 - 600), min(cn, c0 + 600))
        c = rng.choice(band, size=min(L, len(band)), replace=False)
        if far_every and i % (far_every * 40) == 3:
            c = np.concatenate([c, rng.choice(cn, size=8000, replace=False)])
        c = np.unique(c)
        cols.extend(c.tolist())
        ro.append(len(cols))
    n = len(cols)
    v = rng.standard_normal(n) * 2.0 ** rng.integers(-30, 30, n)
    v[rng.random(n) < 0.05] = 0.0
    v[rng.random(n) < 0.02] *= -0.0
    return refops.Csr(rn, cn, np.array(ro, dtype=np.int64), np.array(cols, dtype=np.int64), v)


@pytest.mark.parametrize("mean,far", [(48, 0), (60, 41), (150, 0), (150, 13), (700, 0), (700, 9)],
                         ids=["rw64", "rw64-direct", "rw16", "rw16-direct", "rw4", "rw4-direct"])
def test_spmv_gather_table(mean, far):
    """the gather-table SpMV of pinned long-row matrices (k_spmv_tab: per tile of rows the
    distinct columns' x in LDS, 16-bit slots per entry; tiles too wide run the direct
    gathers): bit for bit the sequential products -- plain, with alpha*y + beta, the f row
    mask, and the fused selection's first largest product per row -- in the 64- and 16-row
    shapes (mean rows from 256 on take no table: the paired-load kernel, checked alike)"""
    rng = np.random.default_rng(mean + far)
    rn = 4800
    A = _tab_matrix(rng, rn, 40000, mean, far)
    x = rng.standard_normal(A.cn) * 2.0 ** rng.integers(-8, 8, A.cn)
    y = rng.standard_normal(rn)
    f = (rng.random(rn) < 0.8).astype(np.uint8)
    oa.spmv_sl_min(0)
    oa.spmv_tab(1)                 # (off by default: AMGD_MV_TAB)
    try:
        z, _, st = oa.test_spmv_tab(A, x)
        z2, _, _ = oa.test_spmv_tab(A, x, 1.0, y, -1.0, f)
        z3, amx, _ = oa.test_spmv_tab(A, x, amx=True)
        zp = oa.test_spmv(A, x)
    finally:
        oa.spmv_sl_min(-1)
        oa.spmv_tab(-1)
    if mean >= 256:
        # coarse levels' long rows: no table (measured slower), the paired-load kernel
        assert st["builds"] == 0, st
    else:
        assert st["builds"] == 1 and st["tiles"] > 0, st
        if far:
            assert 0 < st["direct"] < st["tiles"], st
        else:
            assert st["direct"] == 0, st
    want = refops.spmv(A, x)
    assert np.array_equal(z.view(np.uint64), want.view(np.uint64))
    assert np.array_equal(zp.view(np.uint64), want.view(np.uint64))
    want2 = refops.spmv(A, x, 1.0, y, -1.0) * (f != 0)
    assert np.array_equal(z2.view(np.uint64), want2.view(np.uint64))
    assert np.array_equal(z3.view(np.uint64), want.view(np.uint64))
    # first largest product per row, strict > from -DBL_MAX (k_fs_select's rule)
    for i in range(rn):
        s, e = int(A.row_off[i]), int(A.row_off[i + 1])
        p = A.a[s:e] * x[A.col[s:e]]
        best, bv = ~np.uint64(0), -np.finfo(np.float64).max
        for q in range(e - s):
            if p[q] > bv:
                bv, best = p[q], np.uint64(s + q)
        assert amx[i] == best, (i, amx[i], best)
