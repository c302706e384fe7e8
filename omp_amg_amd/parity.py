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


def first_diff(h1: Hierarchy, h2: Hierarchy) -> list[dict]:
    """Every differing array of two hierarchies with its first differing position: for a
    CSR, the first row whose offsets, columns or values differ, with both rows' (column,
    value) lists from the first differing entry on (a few each); for a vector, the first
    index and both values.  Used by the partitioned tests' failure reports."""
    out: list[dict] = []
    nl = min(h1.nlevels, h2.nlevels)
    if h1.nlevels != h2.nlevels:
        out.append({"what": "nlevels", "a": int(h1.nlevels), "b": int(h2.nlevels)})
    for l in range(nl):
        a, b = h1.levels[l], h2.levels[l]
        for f in _VEC_FIELDS:
            x, y = getattr(a, f), getattr(b, f)
            if x is None or y is None:
                if (x is None) != (y is None):
                    out.append({"what": f"L{l}_{f}", "missing": "a" if x is None else "b"})
                continue
            x, y = np.asarray(x), np.asarray(y)
            if x.shape != y.shape:
                out.append({"what": f"L{l}_{f}", "len": [int(x.size), int(y.size)]})
                continue
            xv = x.view(np.uint64) if x.dtype == np.float64 else x
            yv = y.view(np.uint64) if y.dtype == np.float64 else y
            d = np.nonzero(xv != yv)[0]
            if d.size:
                i = int(d[0])
                out.append({"what": f"L{l}_{f}", "count": int(d.size), "index": i,
                            "a": x[i].item(), "b": y[i].item()})
        for f in _CSR_FIELDS:
            x, y = getattr(a, f), getattr(b, f)
            if x is None or y is None:
                if (x is None) != (y is None):
                    out.append({"what": f"L{l}_{f}", "missing": "a" if x is None else "b"})
                continue
            if (x.rn, x.cn) != (y.rn, y.cn):
                out.append({"what": f"L{l}_{f}", "shape": [[x.rn, x.cn], [y.rn, y.cn]]})
                continue
            ro1, ro2 = x.row_off.astype(np.int64), y.row_off.astype(np.int64)
            bad_rows = []
            for r in range(x.rn):
                s1, e1, s2, e2 = ro1[r], ro1[r + 1], ro2[r], ro2[r + 1]
                if e1 - s1 != e2 - s2 or not np.array_equal(x.col[s1:e1], y.col[s2:e2]) or \
                        not np.array_equal(x.a[s1:e1].view(np.uint64), y.a[s2:e2].view(np.uint64)):
                    bad_rows.append(r)
                    if len(bad_rows) > 64:
                        break
            if not bad_rows:
                continue
            r = bad_rows[0]
            s1, e1, s2, e2 = ro1[r], ro1[r + 1], ro2[r], ro2[r + 1]
            c1, c2 = x.col[s1:e1], y.col[s2:e2]
            v1, v2 = x.a[s1:e1], y.a[s2:e2]
            k = 0
            while k < min(len(c1), len(c2)) and c1[k] == c2[k] and v1[k].view(np.uint64) == v2[k].view(np.uint64):
                k += 1
            out.append({"what": f"L{l}_{f}", "first_row": int(r), "rows_differing_at_least": len(bad_rows),
                        "row_len": [int(e1 - s1), int(e2 - s2)], "entry": int(k),
                        "a": [[int(c), float(v)] for c, v in zip(c1[k:k + 4], v1[k:k + 4])],
                        "b": [[int(c), float(v)] for c, v in zip(c2[k:k + 4], v2[k:k + 4])],
                        "pattern_same": bool(np.array_equal(ro1, ro2) and np.array_equal(x.col, y.col))})
    return out
