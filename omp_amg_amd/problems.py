"""Synthetic CSR/COO problems for parity tests and the bench.

BASELINE.json configs:
  [0] crs_test/serial_amg on the bundled amgdmp_{i,j,p}.dat   -> load_amgdmp()
  [1] 3D 7-point Poisson 256^3                                 -> poisson3d(m=256, stencil=7)
  [2] Nek5000 SEM pressure Laplacian, E hexes, order N         -> sem_laplacian(...)
  [3] 3D 27-point Poisson 512^3                                -> poisson3d(m=512, stencil=27)
  [4] anisotropic 3D Poisson eps=1e-3                          -> poisson3d(m, 7, eps=1e-3)

All generators return 0-based COO (Ai, Aj, Av) sorted row-major with unique
(i, j) pairs and no explicit zeros -- the assembled form the reference's dump
writes (amg.c:949-1045) and `build_csr` expects (amg_setup.c:3612).
"""
from __future__ import annotations

import os

import numpy as np


def _stencil_offsets(stencil: int, dim: int):
    if dim == 2:
        if stencil == 5:
            return [(0, -1), (-1, 0), (0, 0), (1, 0), (0, 1)]
        if stencil == 9:
            return [(dx, dy) for dy in (-1, 0, 1) for dx in (-1, 0, 1)]
    if dim == 3:
        if stencil == 7:
            return [(0, 0, -1), (0, -1, 0), (-1, 0, 0), (0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1)]
        if stencil == 27:
            return [(dx, dy, dz) for dz in (-1, 0, 1) for dy in (-1, 0, 1) for dx in (-1, 0, 1)]
    raise ValueError(f"unsupported stencil {stencil} in {dim}D")


def poisson3d(m: int, stencil: int = 7, eps: float = 1.0, mx: int | None = None,
              my: int | None = None, dtype_idx=np.uint32, rows_range: tuple | None = None):
    """Dirichlet-eliminated finite-difference Laplacian on an mx*my*m grid.

    7-point: diagonal 2(1+1+eps)-ish weights with the z-coupling scaled by eps
    (eps < 1 gives the anisotropic case).  27-point: the trilinear-FE-like stencil
    26 on the diagonal and -1 off it.  Rows are ordered x fastest.
    rows_range=(r0, r1): only the entries of rows r0..r1-1 -- exactly that slice of the
    full (row-major sorted) COO, so the slices of all ranks concatenate to the matrix
    (the partitioned bench: each rank generates its own rows).
    """
    mx = m if mx is None else mx
    my = m if my is None else my
    mz = m
    n = mx * my * mz
    offs = _stencil_offsets(stencil, 3)
    r0, r1 = rows_range if rows_range is not None else (0, n)
    idx = np.arange(r0, r1, dtype=np.int64)
    x = idx % mx
    y = (idx // mx) % my
    z = idx // (mx * my)
    rows, cols, vals = [], [], []
    for (dx, dy, dz) in offs:
        X, Y, Z = x + dx, y + dy, z + dz
        ok = (X >= 0) & (X < mx) & (Y >= 0) & (Y < my) & (Z >= 0) & (Z < mz)
        r = idx[ok]
        c = (X + mx * (Y + my * Z))[ok]
        if stencil == 7:
            if (dx, dy, dz) == (0, 0, 0):
                v = np.full(r.shape, 4.0 + 2.0 * eps)
            elif dz != 0:
                v = np.full(r.shape, -eps)
            else:
                v = np.full(r.shape, -1.0)
        else:
            v = np.full(r.shape, 26.0 if (dx, dy, dz) == (0, 0, 0) else -1.0)
        rows.append(r)
        cols.append(c)
        vals.append(v)
    return _finish(np.concatenate(rows), np.concatenate(cols), np.concatenate(vals), dtype_idx)


def poisson2d(m: int, stencil: int = 5, mx: int | None = None, dtype_idx=np.uint32):
    mx = m if mx is None else mx
    n = mx * m
    idx = np.arange(n, dtype=np.int64)
    x = idx % mx
    y = idx // mx
    rows, cols, vals = [], [], []
    for (dx, dy) in _stencil_offsets(stencil, 2):
        X, Y = x + dx, y + dy
        ok = (X >= 0) & (X < mx) & (Y >= 0) & (Y < m)
        r = idx[ok]
        c = (X + mx * Y)[ok]
        if stencil == 5:
            v = np.full(r.shape, 4.0 if (dx, dy) == (0, 0) else -1.0)
        else:
            v = np.full(r.shape, 8.0 if (dx, dy) == (0, 0) else -1.0)
        rows.append(r)
        cols.append(c)
        vals.append(v)
    return _finish(np.concatenate(rows), np.concatenate(cols), np.concatenate(vals), dtype_idx)


def _gll(N: int):
    """Gauss-Lobatto-Legendre points and weights of order N (N+1 points)."""
    from numpy.polynomial import legendre as L
    if N == 1:
        return np.array([-1.0, 1.0]), np.array([1.0, 1.0])
    c = np.zeros(N + 1)
    c[-1] = 1.0
    inner = np.sort(np.real(L.legroots(L.legder(c))))
    z = np.concatenate([[-1.0], inner, [1.0]])
    PN = L.legval(z, c)
    w = 2.0 / (N * (N + 1) * PN * PN)
    return z, w


def _gll_deriv(z):
    n = len(z)
    D = np.zeros((n, n))
    from numpy.polynomial import legendre as L
    N = n - 1
    c = np.zeros(n)
    c[-1] = 1.0
    P = L.legval(z, c)
    for i in range(n):
        for j in range(n):
            if i != j:
                D[i, j] = P[i] / (P[j] * (z[i] - z[j]))
    D[0, 0] = -N * (N + 1) / 4.0
    D[N, N] = N * (N + 1) / 4.0
    return D


def sem_laplacian(ex: int, ey: int, ez: int, N: int, seed: int = 0, jitter: float = 0.0,
                  dtype_idx=np.uint32):
    """Assembled spectral-element Laplacian (GLL, order N) on an ex*ey*ez box of
    hexes with Dirichlet boundary rows/cols removed -- the unstructured,
    high-nnz/row operator class of BASELINE config [2] (Nek5000 SEM, E hexes).

    Element matrices are the tensor-product stiffness on an affine (optionally
    jittered in size) hex; assembly sums shared GLL nodes (gs-style).  Entries
    below 1e-14 relative are dropped to keep the pattern free of numerical zeros.
    """
    rng = np.random.default_rng(seed)
    z, w = _gll(N)
    D = _gll_deriv(z)
    n1 = N + 1
    K1 = D.T @ np.diag(w) @ D          # 1D stiffness
    M1 = np.diag(w)                    # 1D (lumped) mass
    gx, gy, gz = ex * N + 1, ey * N + 1, ez * N + 1

    # element-local stiffness for unit cube scaled by h
    def elem(hx, hy, hz):
        Kx = np.kron(M1, np.kron(M1, K1)) * (hy * hz / hx) * 0.5
        Ky = np.kron(M1, np.kron(K1, M1)) * (hx * hz / hy) * 0.5
        Kz = np.kron(K1, np.kron(M1, M1)) * (hx * hy / hz) * 0.5
        return Kx + Ky + Kz

    li = np.arange(n1)
    lz, ly, lx = np.meshgrid(li, li, li, indexing="ij")
    lx, ly, lz = lx.ravel(), ly.ravel(), lz.ravel()
    # the element matrix of an affine hex is a sum of Kronecker products with the
    # diagonal GLL mass, so most of its (N+1)^6 entries are exact zeros: keep only
    # its structural pattern (identical for every element) before assembly
    pat = np.flatnonzero(elem(1.0, 1.0, 1.0).ravel() != 0)
    pr, pc = pat // n1 ** 3, pat % n1 ** 3
    loc = lx + gx * (ly + gy * lz)                       # node offsets inside an element
    kz, ky, kx = np.meshgrid(np.arange(ez), np.arange(ey), np.arange(ex), indexing="ij")
    base = (kx.ravel() * N + gx * (ky.ravel() * N + gy * kz.ravel() * N)).astype(np.int64)
    if jitter == 0.0:
        ke = np.broadcast_to(elem(1.0, 1.0, 1.0).ravel()[pat], (len(base), len(pat)))
    else:                                                # element order = the loop order kz, ky, kx
        ke = np.stack([elem(*(1.0 + jitter * (rng.random(3) - 0.5))).ravel()[pat]
                       for _ in range(len(base))])
    r = (base[:, None] + loc[pr][None, :]).ravel()
    c = (base[:, None] + loc[pc][None, :]).ravel()
    v = np.ascontiguousarray(ke).ravel()
    # assemble duplicates (summed in element order, like gs)
    ntot = gx * gy * gz
    key = r * ntot + c
    del r, c
    order = np.argsort(key, kind="stable")
    key, v = key[order], v[order]
    del order
    uk, start = np.unique(key, return_index=True)
    vs = np.add.reduceat(v, start)
    r, c = uk // ntot, uk % ntot
    # Dirichlet: drop boundary nodes
    X, Y, Z = r % gx, (r // gx) % gy, r // (gx * gy)
    bx = (X == 0) | (X == gx - 1) | (Y == 0) | (Y == gy - 1) | (Z == 0) | (Z == gz - 1)
    Xc, Yc, Zc = c % gx, (c // gx) % gy, c // (gx * gy)
    bc = (Xc == 0) | (Xc == gx - 1) | (Yc == 0) | (Yc == gy - 1) | (Zc == 0) | (Zc == gz - 1)
    keep = ~bx & ~bc
    r, c, vs = r[keep], c[keep], vs[keep]
    scale = np.abs(vs).max()
    keep = np.abs(vs) > 1e-14 * scale
    r, c, vs = r[keep], c[keep], vs[keep]
    # renumber interior nodes densely
    u, inv = np.unique(np.concatenate([r, c]), return_inverse=True)
    r, c = inv[: len(r)], inv[len(r):]
    return _finish(r, c, vs, dtype_idx)


def _finish(r, c, v, dtype_idx):
    order = np.lexsort((c, r))
    return (r[order].astype(dtype_idx), c[order].astype(dtype_idx),
            np.ascontiguousarray(v[order], dtype=np.float64))


def load_amgdmp(directory: str):
    """Read the reference's bundled test matrix (serial_amg.c:64-91 format):
    each file is doubles, first one the 3.14159 endian marker, indices 1-based."""
    def rd(name):
        d = np.fromfile(os.path.join(directory, name), dtype="<f8")
        if abs(d[0] - 3.14159) > 1e-6:
            d = d.byteswap()
        return d[1:]
    i = rd("amgdmp_i.dat")
    j = rd("amgdmp_j.dat")
    p = rd("amgdmp_p.dat")
    return (i.astype(np.int64) - 1).astype(np.uint32), (j.astype(np.int64) - 1).astype(np.uint32), p


def coo_to_csr_np(Ai, Aj, Av):
    """Sorted-COO -> CSR (host helper for tests/bench; not the product path)."""
    Ai = np.asarray(Ai, dtype=np.int64)
    n = int(max(Ai.max(), np.asarray(Aj).max())) + 1 if len(Ai) else 0
    ro = np.zeros(n + 1, dtype=np.int64)
    np.add.at(ro, Ai + 1, 1)
    return np.cumsum(ro), np.asarray(Aj, dtype=np.int64), np.asarray(Av, dtype=np.float64)
