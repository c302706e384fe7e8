"""ctypes mirror of the drop-in C ABI (include/amg_setup.h).

`struct csr_mat` and `struct amg_setup_data` are laid out exactly as the
reference declares them (amg_tools.h:5-8 and amg_tools.h:25-50) with gslib's
`uint` = `unsigned long` (the reference Makefile builds with -DUSE_LONG,
Makefile:12).  The same reader therefore works on the hierarchy produced by

  * the product library (omp_amg_amd/libomp_amg_amd.so, HIP path),
  * the CPU oracle (oracle/build/liboracle.so, test infrastructure), and
  * the compiled reference (oracle/_ref/libref_amg.so, test infrastructure),

because all three export `amg_setup(n, Ai, Aj, Av, data)` (amg_setup.h:5).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

amg_uint = C.c_ulong


class CsrMat(C.Structure):
    # amg_tools.h:5-8
    _fields_ = [("rn", amg_uint), ("cn", amg_uint),
                ("row_off", C.POINTER(amg_uint)), ("col", C.POINTER(amg_uint)),
                ("a", C.POINTER(C.c_double))]


class AmgSetupData(C.Structure):
    # amg_tools.h:25-50 (field order matters)
    _fields_ = [("tolc", C.c_double), ("gamma", C.c_double),
                ("n", C.POINTER(C.c_double)), ("nnz", C.POINTER(C.c_double)),
                ("nnzf", C.POINTER(C.c_double)), ("nnzfp", C.POINTER(C.c_double)),
                ("m", C.POINTER(C.c_double)), ("rho", C.POINTER(C.c_double)),
                ("A", C.POINTER(C.POINTER(CsrMat))),
                ("id", C.POINTER(amg_uint)),
                ("idc", C.POINTER(C.POINTER(amg_uint))),
                ("idf", C.POINTER(C.POINTER(amg_uint))),
                ("C", C.POINTER(C.POINTER(C.c_double))),
                ("F", C.POINTER(C.POINTER(C.c_double))),
                ("D", C.POINTER(C.POINTER(C.c_double))),
                ("Af", C.POINTER(C.POINTER(CsrMat))),
                ("W", C.POINTER(C.POINTER(CsrMat))),
                ("AfP", C.POINTER(C.POINTER(CsrMat))),
                ("nlevels", amg_uint), ("nullspace", amg_uint)]


@dataclass
class Csr:
    rn: int
    cn: int
    row_off: np.ndarray
    col: np.ndarray
    a: np.ndarray

    @property
    def nnz(self) -> int:
        return int(self.row_off[-1]) if len(self.row_off) else 0

    def to_dense(self) -> np.ndarray:
        d = np.zeros((self.rn, self.cn))
        for i in range(self.rn):
            s, e = self.row_off[i], self.row_off[i + 1]
            d[i, self.col[s:e]] += self.a[s:e]
        return d


@dataclass
class Level:
    n: float
    nnz: float
    A: Csr
    C: np.ndarray | None = None      # coarse mask (0/1 doubles), amg_setup.c:182
    F: np.ndarray | None = None
    D: np.ndarray | None = None      # scaled Jacobi diagonal, amg_setup.c:261
    m: float | None = None           # Chebyshev iterations
    rho: float | None = None
    nnzf: float | None = None
    nnzfp: float | None = None
    idc: np.ndarray | None = None
    idf: np.ndarray | None = None
    Af: Csr | None = None
    W: Csr | None = None
    AfP: Csr | None = None


@dataclass
class Hierarchy:
    nlevels: int
    nullspace: int
    tolc: float
    gamma: float
    id: np.ndarray
    levels: list = field(default_factory=list)


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def read_csr(p) -> Csr:
    m = p.contents
    rn, cn = int(m.rn), int(m.cn)
    ro = _arr(m.row_off, rn + 1, np.int64)
    nz = int(ro[-1])
    return Csr(rn, cn, ro, _arr(m.col, nz, np.int64), _arr(m.a, nz, np.float64))


def read_setup_data(d: AmgSetupData) -> Hierarchy:
    """Copy every per-level array out of a filled `struct amg_setup_data`."""
    nl = int(d.nlevels)
    if nl == 0:                       # failed setup (omp_amg_amd: out of HBM): empty data
        return Hierarchy(0, 0, float(d.tolc), float(d.gamma), np.zeros(0, dtype=np.int64))
    n0 = int(d.n[0])
    h = Hierarchy(nl, int(d.nullspace), float(d.tolc), float(d.gamma),
                  _arr(d.id, n0, np.int64))
    for l in range(nl):
        lev = Level(n=float(d.n[l]), nnz=float(d.nnz[l]), A=read_csr(d.A[l]))
        if l < nl - 1:
            rn = int(d.n[l])
            nc = int(d.n[l + 1])
            lev.C = _arr(d.C[l], rn, np.float64)
            lev.F = _arr(d.F[l], rn, np.float64)
            lev.D = _arr(d.D[l], rn - nc, np.float64)
            lev.m = float(d.m[l])
            lev.rho = float(d.rho[l])
            lev.nnzf = float(d.nnzf[l])
            lev.nnzfp = float(d.nnzfp[l])
            lev.idc = _arr(d.idc[l], nc, np.int64)
            lev.idf = _arr(d.idf[l], rn - nc, np.int64)
            lev.Af = read_csr(d.Af[l])
            lev.W = read_csr(d.W[l])
            lev.AfP = read_csr(d.AfP[l])
        h.levels.append(lev)
    return h


@contextlib.contextmanager
def quiet_stdout(enabled: bool = True):
    """Silence C-level stdout (the reference prints per-level progress)."""
    if not enabled:
        yield
        return
    libc = C.CDLL(None)
    libc.fflush(None)
    fd = os.dup(1)
    dn = os.open(os.devnull, os.O_WRONLY)
    os.dup2(dn, 1)
    try:
        yield
    finally:
        libc.fflush(None)
        os.dup2(fd, 1)
        os.close(fd)
        os.close(dn)


def srand(seed: int = 1) -> None:
    """Reset libc's rand() stream; the reference's Lanczos start vector is
    rand()/RAND_MAX (amg_setup.c:2447), so every parity run starts from seed 1."""
    C.CDLL(None).srand(C.c_uint(seed))


class Comm(C.Structure):
    # gslib comm.h:85-88 (non-MPI build), include/crs.h
    _fields_ = [("id", amg_uint), ("np", amg_uint), ("c", C.c_int)]


def bind_crs(lib: C.CDLL) -> C.CDLL:
    """crs.h (reference crs.h:15-20) + the export hook of omp_amg_amd.h"""
    lib.crs_setup.argtypes = [amg_uint, C.POINTER(C.c_ulong), amg_uint, C.POINTER(amg_uint),
                              C.POINTER(amg_uint), C.POINTER(C.c_double), amg_uint, C.POINTER(Comm)]
    lib.crs_setup.restype = C.c_void_p
    lib.crs_free.argtypes = [C.c_void_p]
    lib.crs_free.restype = None
    lib.amgd_crs_export.argtypes = [C.c_void_p, C.POINTER(AmgSetupData)]
    lib.amgd_crs_export.restype = C.c_int
    return lib


def crs_setup(lib: C.CDLL, n: int, ids, Ai, Aj, Av, null_space: int = 0, rank: int = 0,
              np_: int = 1, *, seed: int = 1, quiet: bool = True):
    """crs_setup(n, id, nz, Ai, Aj, A, null_space, comm) of crs.h on a local matrix
    (local indices Ai/Aj < n, global ids `ids`, 1-based, 0 = not a dof); returns the
    opaque handle (None where the library returned NULL)"""
    bind_crs(lib)
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    Ai = np.ascontiguousarray(Ai, dtype=np.uint64)
    Aj = np.ascontiguousarray(Aj, dtype=np.uint64)
    Av = np.ascontiguousarray(Av, dtype=np.float64)
    comm = Comm(rank, np_, 0)
    srand(seed)
    with quiet_stdout(quiet):
        h = lib.crs_setup(n, ids.ctypes.data_as(C.POINTER(C.c_ulong)), len(Av),
                          Ai.ctypes.data_as(C.POINTER(amg_uint)), Aj.ctypes.data_as(C.POINTER(amg_uint)),
                          Av.ctypes.data_as(C.POINTER(C.c_double)), null_space, C.byref(comm))
    return h or None


def crs_export(lib: C.CDLL, handle) -> Hierarchy:
    """the hierarchy crs_setup keeps in HBM (amgd_crs_export), as a host copy"""
    bind_crs(lib)
    bind_setup(lib)
    libc = C.CDLL(None)
    libc.malloc.restype = C.c_void_p
    libc.malloc.argtypes = [C.c_size_t]
    raw = libc.malloc(C.sizeof(AmgSetupData))
    C.memset(raw, 0, C.sizeof(AmgSetupData))
    dp = C.cast(raw, C.POINTER(AmgSetupData))
    if lib.amgd_crs_export(handle, dp) != 0:
        raise RuntimeError("amgd_crs_export failed")
    h = read_setup_data(dp.contents)
    lib.free_data(C.pointer(dp))
    return h


def bind_setup(lib: C.CDLL) -> C.CDLL:
    lib.amg_setup.argtypes = [amg_uint, C.POINTER(amg_uint), C.POINTER(amg_uint),
                              C.POINTER(C.c_double), C.POINTER(AmgSetupData)]
    lib.amg_setup.restype = None
    lib.free_data.argtypes = [C.POINTER(C.POINTER(AmgSetupData))]
    lib.free_data.restype = None
    return lib


def run_setup(lib: C.CDLL, Ai, Aj, Av, *, seed: int = 1, quiet: bool = True,
              libc_malloc: bool = True) -> Hierarchy:
    """Call `amg_setup` of any of the three libraries on COO input and return a
    host copy of the hierarchy.  Ai/Aj are 0-based (serial_amg.c:89-90)."""
    Ai = np.ascontiguousarray(Ai, dtype=np.uint64)
    Aj = np.ascontiguousarray(Aj, dtype=np.uint64)
    Av = np.ascontiguousarray(Av, dtype=np.float64)
    nz = len(Av)
    assert len(Ai) == nz and len(Aj) == nz
    libc = C.CDLL(None)
    libc.malloc.restype = C.c_void_p
    libc.malloc.argtypes = [C.c_size_t]
    # data is malloc'ed so that free_data() (which calls free(*data)) is legal
    raw = libc.malloc(C.sizeof(AmgSetupData))
    C.memset(raw, 0, C.sizeof(AmgSetupData))
    dp = C.cast(raw, C.POINTER(AmgSetupData))
    srand(seed)
    with quiet_stdout(quiet):
        lib.amg_setup(nz, Ai.ctypes.data_as(C.POINTER(amg_uint)),
                      Aj.ctypes.data_as(C.POINTER(amg_uint)),
                      Av.ctypes.data_as(C.POINTER(C.c_double)), dp)
    h = read_setup_data(dp.contents)
    pp = C.pointer(dp)
    lib.free_data(pp)
    return h
