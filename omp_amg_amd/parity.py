"""Hierarchy (de)serialisation and comparison used by the parity tests.

Comparison policy (DESIGN.md "Parity"):
  * integer work -- level sizes, C/F masks, idc/idf ids, every CSR pattern
    (row_off, col) -- must be identical;
  * doubles -- bit-identical when `exact=True` (oracle vs compiled reference),
    otherwise within `rtol` relative (HIP path vs oracle, whose global
    reductions are tree-ordered on the GPU).
"""
from __future__ import annotations

import numpy as np

from .abi import Csr, Hierarchy, Level

_CSR_FIELDS = ("A", "Af", "W", "AfP")
_VEC_FIELDS = ("C", "F", "D", "idc", "idf")
_SCAL_FIELDS = ("n", "nnz", "m", "rho", "nnzf", "nnzfp")


def to_npz_dict(h: Hierarchy, prefix: str = "") -> dict:
    d = {prefix + "nlevels": np.int64(h.nlevels), prefix + "nullspace": np.int64(h.nullspace),
         prefix + "tolc": np.float64(h.tolc), prefix + "gamma": np.float64(h.gamma),
         prefix + "id": h.id}
    for l, lev in enumerate(h.levels):
        p = f"{prefix}L{l}_"
        for f in _SCAL_FIELDS:
            v = getattr(lev, f)
            if v is not None:
                d[p + f] = np.float64(v)
        for f in _VEC_FIELDS:
            v = getattr(lev, f)
            if v is not None:
                d[p + f] = v
        for f in _CSR_FIELDS:
            m = getattr(lev, f)
            if m is not None:
                d[p + f + "_shape"] = np.array([m.rn, m.cn], dtype=np.int64)
                d[p + f + "_ro"] = m.row_off.astype(np.int64)
                d[p + f + "_col"] = m.col.astype(np.int32)
                d[p + f + "_a"] = m.a
    return d


def from_npz(z, prefix: str = "") -> Hierarchy:
    nl = int(z[prefix + "nlevels"])
    h = Hierarchy(nl, int(z[prefix + "nullspace"]), float(z[prefix + "tolc"]),
                  float(z[prefix + "gamma"]), np.asarray(z[prefix + "id"]))
    for l in range(nl):
        p = f"{prefix}L{l}_"

        def csr(f):
            if p + f + "_shape" not in z:
                return None
            rn, cn = (int(x) for x in z[p + f + "_shape"])
            return Csr(rn, cn, np.asarray(z[p + f + "_ro"], dtype=np.int64),
                       np.asarray(z[p + f + "_col"], dtype=np.int64), np.asarray(z[p + f + "_a"]))
        lev = Level(n=float(z[p + "n"]), nnz=float(z[p + "nnz"]), A=csr("A"))
        for f in _SCAL_FIELDS[2:]:
            if p + f in z:
                setattr(lev, f, float(z[p + f]))
        for f in _VEC_FIELDS:
            if p + f in z:
                setattr(lev, f, np.asarray(z[p + f]))
        for f in _CSR_FIELDS[1:]:
            setattr(lev, f, csr(f))
        h.levels.append(lev)
    return h


def _vals_equal(x: np.ndarray, y: np.ndarray, exact: bool, rtol: float, scale: float | None = None):
    if x.shape != y.shape:
        return False, np.inf
    if x.size == 0:
        return True, 0.0
    if exact:
        same = np.array_equal(x.view(np.uint64), y.view(np.uint64))
        return same, 0.0 if same else float(np.max(np.abs(x - y)))
    # relative to the largest magnitude in the array: values that cancel to
    # tiny numbers are judged against the operator's scale, not themselves
    s = scale if scale is not None else max(float(np.max(np.abs(x))), 1e-300)
    err = float(np.max(np.abs(x - y))) / s
    return err <= rtol, err


def compare(h1: Hierarchy, h2: Hierarchy, *, exact: bool = True, rtol: float = 1e-12,
            levels: int | None = None) -> list[str]:
    """Return a list of mismatch descriptions (empty == parity)."""
    bad: list[str] = []
    if h1.nlevels != h2.nlevels:
        bad.append(f"nlevels {h1.nlevels} != {h2.nlevels}")
    if h1.nullspace != h2.nullspace:
        bad.append(f"nullspace {h1.nullspace} != {h2.nullspace}")
    nl = min(h1.nlevels, h2.nlevels) if levels is None else min(levels, h1.nlevels, h2.nlevels)
    for l in range(nl):
        a, b = h1.levels[l], h2.levels[l]
        for f in ("n", "nnz", "nnzf", "nnzfp", "m"):
            x, y = getattr(a, f), getattr(b, f)
            if x != y:
                bad.append(f"L{l}.{f}: {x} != {y}")
        if a.rho is not None and b.rho is not None:
            ok, err = _vals_equal(np.array([a.rho]), np.array([b.rho]), exact, max(rtol, 1e-9))
            if not ok:
                bad.append(f"L{l}.rho: {a.rho} vs {b.rho}")
        for f in ("C", "F", "idc", "idf"):
            x, y = getattr(a, f), getattr(b, f)
            if x is None and y is None:
                continue
            if x is None or y is None or not np.array_equal(x, y):
                bad.append(f"L{l}.{f} differs")
        if a.D is not None:
            ok, err = _vals_equal(a.D, b.D, exact, max(rtol, 1e-9))
            if not ok:
                bad.append(f"L{l}.D err={err:.3g}")
        for f in _CSR_FIELDS:
            x, y = getattr(a, f), getattr(b, f)
            if x is None and y is None:
                continue
            if x is None or y is None:
                bad.append(f"L{l}.{f} missing")
                continue
            if (x.rn, x.cn) != (y.rn, y.cn) or not np.array_equal(x.row_off, y.row_off) \
                    or not np.array_equal(x.col, y.col):
                bad.append(f"L{l}.{f} pattern differs ({x.rn}x{x.cn} nnz {x.nnz} vs {y.rn}x{y.cn} nnz {y.nnz})")
                continue
            ok, err = _vals_equal(x.a, y.a, exact, rtol)
            if not ok:
                bad.append(f"L{l}.{f} values err={err:.3g}")
    return bad
