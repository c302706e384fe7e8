"""Parity of the HIP AMG setup, through the drop-in C ABI (amg_setup.h), against
  * the reference's own outputs (tests/golden/*.npz, made from the compiled
    reference by tests/golden/make_golden.py), and
  * the CPU oracle (oracle/, pinned bit-exactly to the reference) on larger
    grids the reference's O(n^2) mxm cannot reach in test time.

Bar (DESIGN.md "Parity"): level sizes, C/F masks, idc/idf and every CSR
pattern identical; W/AfP/Af/A values within 1e-12 relative to each matrix's
largest entry (north_star); Chebyshev D / rho within 1e-9.  With the default
reference-order dots the hierarchy is in fact bit-identical, which
test_gpu_bitexact_vs_reference_fixture holds it to.
"""
import os

import numpy as np
import pytest

from conftest import GOLD, golden_cases
import omp_amg_amd as oa
from omp_amg_amd import abi, parity, problems

pytestmark = pytest.mark.gpu
RTOL = 1e-12


@pytest.mark.parametrize("case", golden_cases())
def test_gpu_matches_reference_fixture(case):
    z = np.load(os.path.join(GOLD, case + ".npz"))
    ref = parity.from_npz(z)
    h = abi.run_setup(oa.lib(), z["in_Ai"], z["in_Aj"], z["in_Av"])
    bad = parity.compare(ref, h, exact=False, rtol=RTOL)
    assert not bad, bad


@pytest.mark.parametrize("case", golden_cases())
def test_gpu_bitexact_vs_reference_fixture(case):
    """every double of the hierarchy equal to the reference's, bit for bit"""
    z = np.load(os.path.join(GOLD, case + ".npz"))
    ref = parity.from_npz(z)
    h = abi.run_setup(oa.lib(), z["in_Ai"], z["in_Aj"], z["in_Av"])
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad


@pytest.mark.parametrize("mode", [(1 << 40, -1), (0, 64), (0, 16)], ids=["wave", "rw64", "rw16"])
@pytest.mark.parametrize("case", ["p27_8", "sem_e3_N2", "p7_14", "aniso_12"])
def test_gpu_bitexact_spmv_kernel_forced(case, mode):
    """every SpMV with long rows (whole-matrix and listed rows) through the wave-per-row
    kernel, or through the lane kernel with 64 / 16 rows per wavefront (small fixtures
    pick 4 by default): hierarchy still bit-exact"""
    z = np.load(os.path.join(GOLD, case + ".npz"))
    ref = parity.from_npz(z)
    oa.spmv_sl_min(mode[0])
    oa.spmv_rw(mode[1])
    try:
        h = abi.run_setup(oa.lib(), z["in_Ai"], z["in_Aj"], z["in_Av"])
    finally:
        oa.spmv_sl_min(-1)
        oa.spmv_rw(-1)
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad


@pytest.mark.parametrize("gen", [
    ("p7_20", lambda: problems.poisson3d(20)),
    ("p7_24x20x16", lambda: problems.poisson3d(16, mx=24, my=20)),
    ("aniso_16", lambda: problems.poisson3d(16, eps=1e-3)),
    ("p27_12", lambda: problems.poisson3d(12, 27)),
    ("sem_e3_N4", lambda: problems.sem_laplacian(3, 3, 3, 4, seed=2, jitter=0.3)),
], ids=lambda g: g[0])
def test_gpu_matches_oracle_larger(oracle_lib, gen):
    Ai, Aj, Av = gen[1]()
    ref = abi.run_setup(oracle_lib, Ai, Aj, Av)
    h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    bad = parity.compare(ref, h, exact=False, rtol=RTOL)
    assert not bad, bad


def test_export_files_match_oracle(oracle_lib, tmp_path):
    """amg_export writes the Nek5000 AMG files (amg_setup.c:405): same bytes for
    ids / levels / row lengths; values within tolerance."""
    import ctypes as C
    Ai, Aj, Av = problems.load_amgdmp(GOLD)
    outs = {}
    for name, L in (("gpu", oa.lib()), ("oracle", oracle_lib)):
        d = tmp_path / name
        d.mkdir()
        cwd = os.getcwd()
        os.chdir(d)
        try:
            libc = C.CDLL(None)
            libc.malloc.restype = C.c_void_p
            raw = libc.malloc(C.sizeof(abi.AmgSetupData))
            C.memset(raw, 0, C.sizeof(abi.AmgSetupData))
            dp = C.cast(raw, C.POINTER(abi.AmgSetupData))
            abi.srand(1)
            u64 = C.POINTER(abi.amg_uint)
            ai = np.ascontiguousarray(Ai, dtype=np.uint64)
            aj = np.ascontiguousarray(Aj, dtype=np.uint64)
            av = np.ascontiguousarray(Av)
            with abi.quiet_stdout():
                L.amg_setup(len(av), ai.ctypes.data_as(u64), aj.ctypes.data_as(u64),
                            av.ctypes.data_as(C.POINTER(C.c_double)), dp)
                L.amg_export.argtypes = [C.POINTER(abi.AmgSetupData)]
                L.amg_export(dp)
            L.free_data(C.pointer(dp))
        finally:
            os.chdir(cwd)
        outs[name] = {f: np.fromfile(d / f) for f in ("amg.dat", "amg_W.dat", "amg_AfP.dat", "amg_Aff.dat")}
    for f in outs["gpu"]:
        g, o = outs["gpu"][f], outs["oracle"][f]
        assert g.shape == o.shape, f
        np.testing.assert_allclose(g, o, rtol=1e-9, atol=1e-12, err_msg=f)


# incremental coarsening sweeps (amgd_coarsen.hip): forced on at every size, the
# hierarchy must stay bit-identical to the reference's / the oracle's
@pytest.mark.parametrize("case", golden_cases())
def test_gpu_incremental_coarsen_bitexact_fixture(case, monkeypatch):
    monkeypatch.setenv("AMGD_CS_MIN_ROWS", "0")
    z = np.load(os.path.join(GOLD, case + ".npz"))
    ref = parity.from_npz(z)
    h = abi.run_setup(oa.lib(), z["in_Ai"], z["in_Aj"], z["in_Av"])
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad


@pytest.mark.parametrize("gen", [
    ("p7_20", lambda: problems.poisson3d(20)),
    ("aniso_16", lambda: problems.poisson3d(16, eps=1e-3)),
    ("p27_12", lambda: problems.poisson3d(12, 27)),
    ("sem_e3_N4", lambda: problems.sem_laplacian(3, 3, 3, 4, seed=2, jitter=0.3)),
], ids=lambda g: g[0])
def test_gpu_incremental_coarsen_vs_oracle(oracle_lib, gen, monkeypatch):
    monkeypatch.setenv("AMGD_CS_MIN_ROWS", "0")
    Ai, Aj, Av = gen[1]()
    ref = abi.run_setup(oracle_lib, Ai, Aj, Av)
    h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    bad = parity.compare(ref, h, exact=False, rtol=RTOL)
    assert not bad, bad


@pytest.mark.parametrize("m,stencil,min_rows,list_nnz", [
    (48, 7, None, None), (48, 7, None, "0"), (18, 27, "0", None), (18, 27, "0", "1000")])
def test_gpu_incremental_coarsen_matches_full_sweeps(m, stencil, min_rows, list_nnz,
                                                     monkeypatch):
    """default (incremental) vs AMGD_CS_INC=0 (every sweep over all rows):
    identical hierarchies, bit for bit (48^3 is above the default threshold);
    list_nnz "0" forces the block-filter mode, "1000" the row-list mode"""
    Ai, Aj, Av = problems.poisson3d(m, stencil)
    if min_rows is not None:
        monkeypatch.setenv("AMGD_CS_MIN_ROWS", min_rows)
    if list_nnz is not None:
        monkeypatch.setenv("AMGD_CS_LIST_NNZ", list_nnz)
    h_inc = abi.run_setup(oa.lib(), Ai, Aj, Av)
    monkeypatch.setenv("AMGD_CS_INC", "0")
    h_full = abi.run_setup(oa.lib(), Ai, Aj, Av)
    bad = parity.compare(h_full, h_inc, exact=True)
    assert not bad, bad


# incremental find_support sweeps (amgd_setup.c find_support): forced at every size,
# and off, the hierarchy must stay bit-identical to the reference's / the oracle's.
# "long8": rows / columns of R past 8 entries through the grid-wide expand, the
# block-per-column select and the block-per-row exact products (default: 4096)
@pytest.mark.parametrize("mode", ["2", "0", "2long8"], ids=["fs_inc_always", "fs_inc_off", "long8"])
@pytest.mark.parametrize("case", ["p7_12", "p27_8", "sem_e3_N2", "aniso_12", "amgdmp", "p2d9_24"])
def test_gpu_fs_incremental_bitexact_fixture(case, mode, monkeypatch):
    monkeypatch.setenv("AMGD_FS_INC", mode[0])
    z = np.load(os.path.join(GOLD, case + ".npz"))
    ref = parity.from_npz(z)
    if mode.endswith("long8"):
        oa.fs_long(8)
        oa.mv_long(8)
    try:
        h = abi.run_setup(oa.lib(), z["in_Ai"], z["in_Aj"], z["in_Av"])
    finally:
        oa.fs_long(-1)
        oa.mv_long(-1)
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad


# lmop: every support takes the general walk, supports of >= 8 points pruned to the
# components of their factor graph -- against the reference's fixtures
# (the pruned walk one wavefront per k at every support size, or one thread per k)
@pytest.mark.parametrize("wave", [1, 0], ids=["wave", "thread"])
@pytest.mark.parametrize("case", ["p7_12", "aniso_12", "sem_e3_N2"])
def test_gpu_lmop_pruned_bitexact_fixture(case, wave):
    z = np.load(os.path.join(GOLD, case + ".npz"))
    ref = parity.from_npz(z)
    oa.lmop_mode(1)
    oa.lmop_prune(8)
    oa.lmop_wave(wave)
    oa.lmop_stats(reset=True)
    try:
        h = abi.run_setup(oa.lib(), z["in_Ai"], z["in_Aj"], z["in_Av"])
    finally:
        oa.lmop_mode(0)
        oa.lmop_prune(-1)
        oa.lmop_wave(-1)
    assert oa.lmop_stats(reset=True)["pruned"] > 0
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad


# lmop: every support takes the general walk, sp_add's walk replayed one wavefront per
# (c, k) at every support size (and one thread per (c, k)) -- against the fixtures; the
# 27-point and anisotropic ones land contributions past their rows
@pytest.mark.parametrize("wave", [1, 0], ids=["wave", "thread"])
@pytest.mark.parametrize("case", ["p7_12", "p27_7", "p27_8", "aniso_12", "sem_e3_N2", "amgdmp"])
def test_gpu_lmop_walk_wave_bitexact_fixture(case, wave):
    z = np.load(os.path.join(GOLD, case + ".npz"))
    ref = parity.from_npz(z)
    oa.lmop_mode(1)
    oa.lmop_prune(0)
    oa.lmop_wave(wave)
    oa.route_stats(reset=True)
    try:
        h = abi.run_setup(oa.lib(), z["in_Ai"], z["in_Aj"], z["in_Av"])
    finally:
        oa.lmop_mode(0)
        oa.lmop_prune(-1)
        oa.lmop_wave(-1)
    assert (oa.route_stats(reset=True)["lmop_wave"] > 0) == bool(wave)
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad


@pytest.mark.parametrize("gen", [("p7_32", "1", lambda: problems.poisson3d(32)),
                                 ("aniso_16", "2", lambda: problems.poisson3d(16, eps=1e-3)),
                                 ("p27_16", "2", lambda: problems.poisson3d(16, 27))],
                         ids=lambda g: g[0])
def test_gpu_fs_incremental_matches_full(gen, monkeypatch):
    """incremental sweeps (default: from 4096 F rows; "2": at every size) vs
    AMGD_FS_INC=0: identical hierarchies (aniso 24^3 is not used: the reference's own
    loop does not terminate on it -- the oracle runs past 120 s as well)"""
    Ai, Aj, Av = gen[2]()
    monkeypatch.setenv("AMGD_FS_INC", gen[1])
    h_inc = abi.run_setup(oa.lib(), Ai, Aj, Av)
    monkeypatch.setenv("AMGD_FS_INC", "0")
    h_full = abi.run_setup(oa.lib(), Ai, Aj, Av)
    bad = parity.compare(h_full, h_inc, exact=True)
    assert not bad, bad


@pytest.mark.parametrize("gen", [("p7_24", lambda: problems.poisson3d(24)),
                                 ("p27_14", lambda: problems.poisson3d(14, 27)),
                                 ("sem_e3_N4", lambda: problems.sem_laplacian(3, 3, 3, 4, seed=2, jitter=0.3))],
                         ids=lambda g: g[0])
def test_gpu_qfactor_reuse_matches_refactor(gen):
    """Q factors of supports the skeleton expansion left unchanged are copied from the
    previous interpolation iteration: hierarchy bit-identical to refactoring every
    support (AMGD_QF_REUSE=0), and the copy path is taken"""
    import ctypes as C
    Ai, Aj, Av = gen[1]()
    L = oa.lib()
    L.amgd_test_qf_reuse_stats.argtypes = [C.POINTER(C.c_uint64)]
    st = (C.c_uint64 * 2)()
    L.amgd_test_qf_reuse_stats(st)
    h_re = abi.run_setup(L, Ai, Aj, Av)
    L.amgd_test_qf_reuse_stats(st)
    assert st[0] > 0, "no factor was reused"
    L.amgd_test_qf_reuse.argtypes = [C.c_int]
    L.amgd_test_qf_reuse(0)
    try:
        h_full = abi.run_setup(L, Ai, Aj, Av)
    finally:
        L.amgd_test_qf_reuse(-1)
    bad = parity.compare(h_full, h_re, exact=True)
    assert not bad, bad


@pytest.mark.parametrize("gen", [("p7_32", lambda: problems.poisson3d(32)),
                                 ("aniso_16", lambda: problems.poisson3d(16, eps=1e-3)),
                                 ("p27_16", lambda: problems.poisson3d(16, 27)),
                                 ("sem_e4_N4", lambda: problems.sem_laplacian(4, 4, 4, 4, seed=5, jitter=0.3))],
                         ids=lambda g: g[0])
@pytest.mark.parametrize("inc", ["1", "0", "2"], ids=["inc_default", "inc_off", "inc_all"])
def test_gpu_lane_spmv_forced_matches_default(gen, inc, monkeypatch):
    """the long-row pipelined SpMV (k_spmv_pipe) forced at every size, with find_support's
    incremental sweeps at their default / off / at every size, vs the default routing:
    identical hierarchies"""
    Ai, Aj, Av = gen[1]()
    monkeypatch.setenv("AMGD_FS_INC", inc)
    h_d = abi.run_setup(oa.lib(), Ai, Aj, Av)
    oa.spmv_sl_min(0)
    try:
        oa.route_stats(reset=True)
        h_f = abi.run_setup(oa.lib(), Ai, Aj, Av)
        assert oa.route_stats(reset=True)["spmv_pipe"] > 0
    finally:
        oa.spmv_sl_min(-1)
    bad = parity.compare(h_d, h_f, exact=True)
    assert not bad, bad
