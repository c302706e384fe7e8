"""omp_amg_amd -- MI355X-native AMG setup (hand-written HIP for gfx950) behind
the gslib C ABI of nicooff/omp_amg (amg_setup.h / crs.h).

Python here is only a ctypes mirror of that C ABI for tests and the bench:

  lib()                      -> ctypes.CDLL of omp_amg_amd/libomp_amg_amd.so (built in-tree)
  amg_setup(Ai, Aj, Av)      -> abi.Hierarchy     (reference amg_setup.h:5, host COO in)
  DeviceSetup                -> device-resident COO -> hierarchy in HBM (omp_amg_amd.h)
  stats()                    -> per-phase times of the last setup
  shard.*                    -> multi-GPU row sharding (RCCL / host transport / one-process sim)

The product path is the HIP library only: if it is missing or no GPU is
visible these functions raise -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libomp_amg_amd.so")
_lib = None


class AmgdStats(C.Structure):
    _fields_ = [("t_total_ms", C.c_double), ("t_build_ms", C.c_double),
                ("t_coarsen_ms", C.c_double), ("t_smoother_ms", C.c_double),
                ("t_interp_ms", C.c_double), ("t_rap_ms", C.c_double),
                ("t_copy_ms", C.c_double), ("rap_kernel_ms", C.c_double),
                ("rap_out_nnz", C.c_uint64), ("rap_bytes", C.c_uint64),
                ("rows0", C.c_uint64), ("nnz0", C.c_uint64),
                ("nlevels", C.c_uint32), ("ub_events", C.c_uint32),
                ("peak_bytes", C.c_size_t), ("spmv_kernel_ms", C.c_double),
                ("spmv_bytes", C.c_uint64), ("spmv_bytes_strict", C.c_uint64),
                ("spmv_launches", C.c_uint64), ("rap_launches", C.c_uint64),
                ("spmv_rw_ms", C.c_double * 3), ("spmv_rw_bytes_strict", C.c_uint64 * 3),
                ("spmv_rw_launches", C.c_uint64 * 3),
                ("ub_site", C.c_uint8 * 8), ("ub_level", C.c_uint8 * 8)]


class HCsr(C.Structure):
    """host CSR used by the kernel test hooks (amgd_testapi.c)"""
    _fields_ = [("rn", C.c_uint32), ("cn", C.c_uint32), ("nnz", C.c_uint64),
                ("ro", C.POINTER(C.c_uint64)), ("col", C.POINTER(C.c_uint32)),
                ("a", C.POINTER(C.c_double))]


def build(force: bool = False, jobs: int = 8) -> str:
    """Compile the HIP library in-tree for gfx950 (make -C omp_amg_amd/csrc)."""
    args = ["make", "-C", os.path.join(HERE, "csrc"), f"-j{jobs}"]
    if force:
        subprocess.run(["make", "-C", os.path.join(HERE, "csrc"), "clean"], check=True)
    subprocess.run(args, check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run omp_amg_amd.build() (no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        abi.bind_setup(L)
        L.amgd_set_exact_dots.argtypes = [C.c_int]
        L.amgd_init.argtypes = [C.c_int]
        L.amgd_init.restype = C.c_int
        L.amgd_error.restype = C.c_char_p
        L.amgd_setup_device.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.POINTER(C.c_void_p), C.c_int]
        L.amgd_setup_device.restype = C.c_int
        L.amgd_hier_export.argtypes = [C.c_void_p, C.POINTER(abi.AmgSetupData)]
        L.amgd_hier_free.argtypes = [C.POINTER(C.c_void_p)]
        L.amgd_get_stats.argtypes = [C.POINTER(AmgdStats)]
        L.amgd_dev_alloc.argtypes = [C.c_size_t]
        L.amgd_dev_alloc.restype = C.c_void_p
        L.amgd_dev_free.argtypes = [C.c_void_p]
        L.amgd_dev_upload.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.amgd_dev_download.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.amgd_test_csr.argtypes = [C.c_int, C.POINTER(HCsr), C.POINTER(HCsr), C.c_double,
                                    C.c_double, C.POINTER(HCsr)]
        L.amgd_test_spmv.argtypes = [C.POINTER(HCsr), C.c_void_p, C.c_double, C.c_void_p,
                                     C.c_double, C.c_void_p]
        L.amgd_test_spmv_f.argtypes = [C.POINTER(HCsr), C.c_void_p, C.c_double, C.c_void_p,
                                       C.c_double, C.c_void_p, C.c_void_p]
        L.amgd_test_spmv_rows.argtypes = [C.POINTER(HCsr), C.c_void_p, C.c_uint32, C.c_void_p,
                                          C.c_void_p]
        L.amgd_test_spmv_sl_min.argtypes = [C.c_int64]
        L.amgd_test_build.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.POINTER(HCsr)]
        L.amgd_test_math.argtypes = [C.c_int, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.amgd_test_free.argtypes = [C.POINTER(HCsr)]
        L.amgd_test_dot.argtypes = [C.c_int, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        L.amgd_test_dot.restype = C.c_double
        L.amgd_test_lmop_mode.argtypes = [C.c_int]
        L.amgd_test_spgemm_flat.argtypes = [C.c_int]
        L.amgd_test_spgemm_win.argtypes = [C.c_int]
        L.amgd_test_qf_reuse.argtypes = [C.c_int]
        L.amgd_test_sg_pattern.argtypes = [C.c_int]
        L.amgd_test_lmop_wave.argtypes = [C.c_int]
        L.amgd_test_lmop_small.argtypes = [C.c_int]
        L.amgd_test_lmop_stats.argtypes = [C.POINTER(C.c_uint64), C.c_int]
        L.amgd_test_lmop_prune.argtypes = [C.c_int]
        L.amgd_test_qf_sparse.argtypes = [C.c_int]
        L.amgd_test_qf_stats.argtypes = [C.POINTER(C.c_uint64)]
        L.amgd_test_qf_coop_lds.argtypes = [C.c_int]
        L.amgd_test_qf_split.argtypes = [C.c_int]
        L.amgd_test_mv_long.argtypes = [C.c_int64]
        L.amgd_test_fs_long.argtypes = [C.c_int64]
        L.amgd_test_spmv_rw.argtypes = [C.c_int]
        L.amgd_test_spmv_pair.argtypes = [C.c_int]
        L.amgd_test_spmv_rw_bounds.argtypes = [C.c_int, C.c_int]
        L.amgd_test_d2h_poll.argtypes = [C.c_int]
        L.amgd_test_fs_amx.argtypes = [C.c_int]
        L.amgd_test_qa_tile.argtypes = [C.c_int]
        L.amgd_test_qa_huge.argtypes = [C.c_int]
        L.amgd_test_spmv_shard_calls.restype = C.c_uint64
        L.amgd_test_route_stats.argtypes = [C.POINTER(C.c_uint64), C.c_int]
        L.amgd_comm_rccl_uid.argtypes = [C.c_char_p]
        L.amgd_comm_rccl_uid.restype = C.c_int
        L.amgd_comm_init_rccl.argtypes = [C.c_int, C.c_int, C.c_char_p]
        L.amgd_comm_init_rccl.restype = C.c_int
        L.amgd_comm_init_host.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.amgd_comm_init_host.restype = C.c_int
        L.amgd_comm_init_sim.argtypes = [C.c_int]
        L.amgd_comm_init_sim.restype = C.c_int
        L.amgd_comm_set_min_work.argtypes = [C.c_double]
        L.amgd_comm_stats.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_double)]
        _lib = L
    return _lib


def init(device: int = 0) -> None:
    L = lib()
    if L.amgd_init(device) != 0:
        raise RuntimeError("omp_amg_amd: no usable HIP device: " + L.amgd_error().decode())


def amg_setup(Ai, Aj, Av, *, seed: int = 1) -> abi.Hierarchy:
    """Drop-in `amg_setup` (amg_setup.h:5) on host COO, through the C ABI."""
    init()
    return abi.run_setup(lib(), Ai, Aj, Av, seed=seed, quiet=False)


def stats() -> dict:
    st = AmgdStats()
    lib().amgd_get_stats(C.byref(st))
    out = {}
    for f, _ in AmgdStats._fields_:
        v = getattr(st, f)
        out[f] = list(v) if hasattr(v, "__len__") else v
    return out


class DeviceSetup:
    """COO resident in HBM -> hierarchy resident in HBM (omp_amg_amd.h)."""

    def __init__(self, Ai, Aj, Av):
        init()
        L = lib()
        self.nz = len(Av)
        Ai = np.ascontiguousarray(Ai, dtype=np.uint32)
        Aj = np.ascontiguousarray(Aj, dtype=np.uint32)
        Av = np.ascontiguousarray(Av, dtype=np.float64)
        self.di = L.amgd_dev_alloc(Ai.nbytes + 8)
        self.dj = L.amgd_dev_alloc(Aj.nbytes + 8)
        self.dv = L.amgd_dev_alloc(Av.nbytes + 8)
        L.amgd_dev_upload(self.di, Ai.ctypes.data, Ai.nbytes)
        L.amgd_dev_upload(self.dj, Aj.ctypes.data, Aj.nbytes)
        L.amgd_dev_upload(self.dv, Av.ctypes.data, Av.nbytes)
        self.h = C.c_void_p()

    def run(self, seed: int = 1, exact_dots: bool = True) -> dict:
        L = lib()
        L.amgd_set_exact_dots(1 if exact_dots else 0)
        if self.h:
            L.amgd_hier_free(C.byref(self.h))
        abi.srand(seed)
        rc = L.amgd_setup_device(self.nz, self.di, self.dj, self.dv, C.byref(self.h), 0)
        if rc != 0:
            raise RuntimeError("amgd_setup_device failed: " + L.amgd_error().decode())
        return stats()

    def export(self) -> abi.Hierarchy:
        L = lib()
        libc = C.CDLL(None)
        libc.malloc.restype = C.c_void_p
        raw = libc.malloc(C.sizeof(abi.AmgSetupData))
        C.memset(raw, 0, C.sizeof(abi.AmgSetupData))
        dp = C.cast(raw, C.POINTER(abi.AmgSetupData))
        L.amgd_hier_export(self.h, dp)
        h = abi.read_setup_data(dp.contents)
        L.free_data(C.pointer(dp))
        return h

    def close(self):
        L = lib()
        if self.h:
            L.amgd_hier_free(C.byref(self.h))
        for p in (self.di, self.dj, self.dv):
            if p:
                L.amgd_dev_free(p)
        self.di = self.dj = self.dv = None


# ---------------------------------------------------------------- test hooks
def _to_hcsr(ro, col, a, rn, cn):
    ro = np.ascontiguousarray(ro, dtype=np.uint64)
    col = np.ascontiguousarray(col, dtype=np.uint32)
    a = np.ascontiguousarray(a, dtype=np.float64)
    h = HCsr(rn, cn, int(ro[-1]), ro.ctypes.data_as(C.POINTER(C.c_uint64)),
             col.ctypes.data_as(C.POINTER(C.c_uint32)), a.ctypes.data_as(C.POINTER(C.c_double)))
    h._keep = (ro, col, a)
    return h


def _from_hcsr(h):
    rn, nz = h.rn, h.nnz
    ro = np.ctypeslib.as_array(h.ro, shape=(rn + 1,)).astype(np.int64)
    col = np.ctypeslib.as_array(h.col, shape=(max(nz, 1),))[:nz].astype(np.int64)
    a = np.ctypeslib.as_array(h.a, shape=(max(nz, 1),))[:nz].copy()
    out = abi.Csr(rn, h.cn, ro, col, a)
    lib().amgd_test_free(C.byref(h))
    return out


def test_csr_op(op: int, A: abi.Csr, B: abi.Csr | None = None, alpha=1.0, beta=1.0) -> abi.Csr:
    """op: 0 spgemm, 1 transpose, 2 mpm, 3 mxmpoint, 4 min_skel (kernel test hooks)."""
    init()
    ha = _to_hcsr(A.row_off, A.col, A.a, A.rn, A.cn)
    hb = _to_hcsr(B.row_off, B.col, B.a, B.rn, B.cn) if B is not None else None
    hx = HCsr()
    rc = lib().amgd_test_csr(op, C.byref(ha), C.byref(hb) if hb else None, alpha, beta, C.byref(hx))
    if rc != 0:
        raise RuntimeError(f"amgd_test_csr({op}) failed rc={rc}")
    return _from_hcsr(hx)


def test_spmv(A: abi.Csr, x, alpha=0.0, y=None, beta=1.0):
    init()
    ha = _to_hcsr(A.row_off, A.col, A.a, A.rn, A.cn)
    x = np.ascontiguousarray(x, dtype=np.float64)
    z = np.zeros(A.rn)
    yy = None if y is None else np.ascontiguousarray(y, dtype=np.float64)
    lib().amgd_test_spmv(C.byref(ha), x.ctypes.data, alpha, None if yy is None else yy.ctypes.data,
                         beta, z.ctypes.data)
    return z


def test_spmv_f(A: abi.Csr, x=None, alpha=0.0, y=None, beta=1.0, f=None):
    """amgd_spmv with every option (x None: ordered row sums; f: u8 row mask)"""
    init()
    ha = _to_hcsr(A.row_off, A.col, A.a, A.rn, A.cn)
    xx = None if x is None else np.ascontiguousarray(x, dtype=np.float64)
    yy = None if y is None else np.ascontiguousarray(y, dtype=np.float64)
    ff = None if f is None else np.ascontiguousarray(f, dtype=np.uint8)
    z = np.zeros(A.rn)
    rc = lib().amgd_test_spmv_f(C.byref(ha), None if xx is None else xx.ctypes.data, alpha,
                                None if yy is None else yy.ctypes.data, beta,
                                None if ff is None else ff.ctypes.data, z.ctypes.data)
    if rc != 0:
        raise RuntimeError("amgd_test_spmv_f failed")
    return z


def test_spmv_tab(A: abi.Csr, x, alpha=0.0, y=None, beta=1.0, f=None, amx=False):
    """amgd_spmv on a pinned matrix: the gather-table kernel (k_spmv_tab).  Returns
    (z, amx or None, {builds, tiles, direct})"""
    init()
    L = lib()
    L.amgd_test_spmv_tab.argtypes = [C.POINTER(HCsr), C.c_void_p, C.c_double, C.c_void_p, C.c_double,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    ha = _to_hcsr(A.row_off, A.col, A.a, A.rn, A.cn)
    xx = np.ascontiguousarray(x, dtype=np.float64)
    yy = None if y is None else np.ascontiguousarray(y, dtype=np.float64)
    ff = None if f is None else np.ascontiguousarray(f, dtype=np.uint8)
    z = np.zeros(A.rn)
    m = np.zeros(A.rn, dtype=np.uint64) if amx else None
    st = np.zeros(3, dtype=np.uint64)
    rc = L.amgd_test_spmv_tab(C.byref(ha), xx.ctypes.data, alpha, None if yy is None else yy.ctypes.data, beta,
                              None if ff is None else ff.ctypes.data, z.ctypes.data,
                              None if m is None else m.ctypes.data, st.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"amgd_test_spmv_tab failed rc={rc}")
    return z, m, {"builds": int(st[0]), "tiles": int(st[1]), "direct": int(st[2])}


def resolve_wave(on: int) -> None:
    """exact sums' (dots, long rows) resolution walk: 1 one wavefront, 0 one 1024-thread
    block (default), -1 environment (AMGD_RESOLVE=wave: the wavefront)"""
    lib().amgd_test_resolve_wave(int(on))


def seg_split(on: int) -> None:
    """long-row exact sums: a chunk with one binade crossing resolved from its split record
    (1, default) or re-summed by the binade scan (0); -1: as AMGD_SEG_SPLIT says"""
    lib().amgd_test_seg_split(int(on))


def dot_split(on: int) -> None:
    """exact dots: a chunk with one binade crossing resolved from its split record (1, default)
    or re-summed by the binade scan (0); -1: as AMGD_DOT_SPLIT says (seg_split(0) turns off both)"""
    lib().amgd_test_dot_split(int(on))


def dot_spec_min(chunks: int) -> None:
    """exact dots: the length (in 4096-product chunks) from which the chunk speculation runs
    instead of one block's binade scan; -1: as AMGD_DOT_SPEC_MIN says (default 16)"""
    lib().amgd_test_dot_spec_min(int(chunks))


def spmv_tab(on: int) -> None:
    """gather tables for pinned long-row matrices (1 default, 0 off, -1 environment)"""
    lib().amgd_test_spmv_tab_on(int(on))


def test_spmv_rows(A: abi.Csr, rows, x=None, z0=None):
    """amgd_spmv_rows: products (x None: ordered sums) of the listed rows only; the
    other entries of z keep z0"""
    init()
    ha = _to_hcsr(A.row_off, A.col, A.a, A.rn, A.cn)
    rows = np.ascontiguousarray(rows, dtype=np.uint32)
    xx = None if x is None else np.ascontiguousarray(x, dtype=np.float64)
    z = np.zeros(A.rn) if z0 is None else np.array(z0, dtype=np.float64)
    rc = lib().amgd_test_spmv_rows(C.byref(ha), rows.ctypes.data, len(rows),
                                   None if xx is None else xx.ctypes.data, z.ctypes.data)
    if rc != 0:
        raise RuntimeError("amgd_test_spmv_rows failed")
    return z


def spmv_sl_min(n: int) -> None:
    """row count from which whole-matrix and listed-row SpMVs with long rows run lane-per-row
    instead of wave-per-row (0: always, the default; -1: environment / default).  Same sums."""
    lib().amgd_test_spmv_sl_min(int(n))


def spmv_rw(rw: int) -> None:
    """rows per wavefront of the lane-per-row SpMV kernel: 4, 16 or 64 (-1: by row count).
    Same sums either way."""
    lib().amgd_test_spmv_rw(int(rw))


def spmv_rw_bounds(code: int) -> None:
    """row-count bounds of the lane SpMV's 16 / 64-row shapes as lo * 100 + hi (log2 of
    the row counts, e.g. 1622 = 2^16 / 2^22, the default; -1: default).  A/B only."""
    code = int(code)
    lib().amgd_test_spmv_rw_bounds(code // 100 if code > 0 else 0, code % 100 if code > 0 else 0)


def qa_tile(t: int) -> None:
    """Q application of 33..512-point supports: U staged through LDS in 64 x t tiles
    (16 / 32) or the row-per-lane kernel (0); -1 back to the default.  Same sums."""
    lib().amgd_test_qa_tile(int(t))


def fs_amx(on: int) -> None:
    """find_support's selection after a full sweep: from the fused first maxima of the
    w = R' rs product (1, default) or by its own pass over the bad columns (0); -1 back to
    the default.  Same selections."""
    lib().amgd_test_fs_amx(int(on))


def d2h_poll(on: int) -> None:
    """small readbacks polled from host-coherent memory (1, default) or blocking copies
    (0); -1 back to the default.  A/B only: same results."""
    lib().amgd_test_d2h_poll(int(on))


def spmv_pair(on: int) -> None:
    """products with x through the paired-load lane kernel k_spmv_pair (1), the
    single-load k_spmv_pipe (0), or as AMGD_MV_PAIR says (-1).  Same sums either way."""
    lib().amgd_test_spmv_pair(int(on))


def test_build(Ai, Aj, Av) -> abi.Csr:
    init()
    Ai = np.ascontiguousarray(Ai, dtype=np.uint32)
    Aj = np.ascontiguousarray(Aj, dtype=np.uint32)
    Av = np.ascontiguousarray(Av, dtype=np.float64)
    hx = HCsr()
    lib().amgd_test_build(len(Av), Ai.ctypes.data, Aj.ctypes.data, Av.ctypes.data, C.byref(hx))
    return _from_hcsr(hx)


def test_math(op: int, a, b=None):
    init()
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(a if b is None else b, dtype=np.float64)
    out = np.zeros_like(a)
    lib().amgd_test_math(op, len(a), a.ctypes.data, b.ctypes.data, out.ctypes.data)
    return out


def test_dot(mode: int, a, b=None, plain: bool = False, exact: bool = True) -> float:
    """exact (reference-order) dot through the library: mode 0 a.b, 1 a.a, 2 (a.*b).*b"""
    init()
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(a if b is None else b, dtype=np.float64)
    return lib().amgd_test_dot(mode, len(a), a.ctypes.data, b.ctypes.data, int(plain), int(exact))


def lmop_mode(mode: int) -> None:
    """interp_lmop path: 0 = row-pull where order-exact (default), 1 = general key/sort walk"""
    lib().amgd_test_lmop_mode(int(mode))


def qf_sparse(mode: int) -> None:
    """huge-support Q factor: 0 dense cooperative, 1 sparse first (default),
    2 sparse with a capacity too small to finish (exercises the dense fallback)"""
    lib().amgd_test_qf_sparse(int(mode))


def qf_coop_lds(m: int) -> None:
    """dense cooperative huge-support factor: supports up to m points stage s1/s2/qk in
    LDS, larger ones read them from global memory (-1: default 8192)"""
    lib().amgd_test_qf_coop_lds(int(m))


def qa_huge(n: int) -> None:
    """Q application: supports above n points run the grid-wide kernels (-1: default 8192)"""
    lib().amgd_test_qa_huge(int(n))


def qf_split(on: int) -> None:
    """huge supports factored per connected component of A on the support (1, the
    default) or as one sequential factor (0); -1: back to the default / AMGD_QF_SPLIT"""
    lib().amgd_test_qf_split(int(on))


def mv_long(n: int) -> None:
    """listed-row products: rows past n entries take the block-per-row exact kernel
    (0: never; -1: default 4096 / AMGD_MV_LONG)"""
    lib().amgd_test_mv_long(int(n))


def fs_long(n: int) -> None:
    """find_support: rows / columns of R past n entries take the grid-wide expand and the
    block-per-column select (0: never; -1: default 4096 / AMGD_FS_LONG)"""
    lib().amgd_test_fs_long(int(n))


def qf_stats() -> dict:
    """huge supports factored sparse / sent to the dense kernel / split into components,
    since the last call"""
    out = (C.c_uint64 * 3)()
    lib().amgd_test_qf_stats(out)
    return {"sparse": int(out[0]), "fallback": int(out[1]), "split": int(out[2])}


ROUTES = ("spmv_pipe", "mv_long", "sg_tiny", "sg_kseq", "sg_wwin", "sg_wwin_sym", "sg_long",
          "cs_inc", "fs_inc", "sg_row", "mv_rw4", "qf_reuse", "lmop_wave", "mv_rw16", "mv_rw64",
          "qf_t512", "qf_t1024", "mv_pair", "fs_amx", "mv_tab", "sg_symreuse", "spat_inc", "sg_drsort")


def route_stats(reset: bool = True) -> dict:
    """how often each default kernel route ran since the last reset (amgd.h AMGD_R_*):
    lane SpMV, outlier-row SpMV, tiny / k-sequential / windowed / wide-symbolic /
    dense-slab / flat SpGEMM, incremental coarsening and find_support sweeps"""
    out = (C.c_uint64 * 32)()
    lib().amgd_test_route_stats(out, int(reset))
    return {k: int(out[i]) for i, k in enumerate(ROUTES)}


def lmop_stats(reset: bool = True) -> dict:
    """interp_lmop path counters since the last reset"""
    out = (C.c_uint64 * 5)()
    lib().amgd_test_lmop_stats(out, int(reset))
    return {"fast": out[0], "general": out[1], "dirty_prefix": out[2], "misses": out[3],
            "pruned": out[4]}


def lmop_prune(n: int) -> None:
    """general walk: supports of at least n points whose factor graph splits into
    components emit same-component contributions only (0: never; -1: default 4096 /
    AMGD_LMOP_PRUNE)"""
    lib().amgd_test_lmop_prune(int(n))


def spgemm_dr_sort(on: int) -> None:
    """SpGEMM rows past the hash bins' capacity by sorting their products (1, default) or by
    the one-block dense-slab kernel (0); -1: as AMGD_DR_SORT says"""
    lib().amgd_test_spgemm_dr_sort(int(on))


def spat_inc(on: int) -> None:
    """the constraint operator's pattern grown from the previous iteration's (1, default) or
    formed whole every iteration (0); -1: as AMGD_SPAT_INC says"""
    lib().amgd_test_spat_inc(int(on))


def spat_stats() -> dict:
    out = (C.c_uint64 * 3)()
    lib().amgd_test_spat_stats(out)
    return {"incremental": out[0], "whole": out[1], "same": out[2]}


def spgemm_sym(mode: int) -> None:
    """the next one-GPU SpGEMM: 1 keeps its symbolic phase, 2 takes the kept one when the
    operand patterns match (else runs in full), -1 drops a kept state (tests)"""
    lib().amgd_test_spgemm_sym(int(mode))


def spgemm_sym_stats() -> dict:
    L = lib()
    k, r = C.c_uint64(), C.c_uint64()
    L.amgd_test_spgemm_sym_stats(C.byref(k), C.byref(r))
    return {"kept": k.value, "reused": r.value}


def spgemm_win(w: int) -> None:
    """wide output rows: 0 = LDS hash kernels only, 1024..16384 = every wide row through the
    wave-private windowed kernel (k_sg_wwin) whatever the column count, -1 = automatic"""
    lib().amgd_test_spgemm_win(int(w))


def qf_reuse(on: int) -> None:
    """Q factors of supports unchanged since the previous interpolation iteration: 1 copy
    (default), 0 refactor every support, -1 default / AMGD_QF_REUSE.  Same bits."""
    lib().amgd_test_qf_reuse(int(on))


def lmop_wave(n: int) -> None:
    """interp_lmop general walk: chunks holding a support of >= n points replay sp_add's
    walk one wavefront per (c, k) with 64 columns searched at once (default 64), 0 one
    thread per (c, k) always, -1 default / AMGD_LMOP_WAVE.  Same landings."""
    lib().amgd_test_lmop_wave(int(n))


def sg_pattern(on: int) -> None:
    """constraint pattern W_skel*W_skel': 1 pattern-only product (default), 0 the full
    product (values discarded by interp_lmop), -1 default.  Same bits."""
    lib().amgd_test_sg_pattern(int(on))


def lmop_small(n: int) -> None:
    """interp_lmop row pull: S rows of <= 32 entries one thread each (n > 0) or on the
    wavefront kernel (0); -1: back to the env (AMGD_LMOP_SMALL)"""
    lib().amgd_test_lmop_small(int(n))


def spgemm_flat(on: bool) -> None:
    """SpGEMM kernels: True = flat enumeration only, False = automatic (k-sequential for long B rows)"""
    lib().amgd_test_spgemm_flat(int(on))
