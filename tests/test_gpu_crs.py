"""The gslib coarse-solver entry (crs.h crs_setup / crs_free, reference amg.c:475)
through the C ABI, and the setup's out-of-HBM error path.

crs_setup takes a LOCAL matrix: n dofs with global ids id[0..n) (1-based; 0 = not a
dof, its entries dropped like the reference's amg_dump, amg.c:1065) and entries in
local indices.  The kept hierarchy (exported by amgd_crs_export) must be the one
amg_setup builds on the same matrix keyed by global id -- bit for bit, and equal to
the reference's own fixture where one exists.
"""
import os

import numpy as np
import pytest

from conftest import GOLD
import omp_amg_amd as oa
from omp_amg_amd import abi, parity, problems

pytestmark = pytest.mark.gpu

# crs_test.c:18-30: the 4 x 4 singular Laplacian of a square, all 16 entries (4 zeros)
CRS_A = np.array([2, -1, -1, 0, -1, 2, 0, -1, -1, 0, 2, -1, 0, -1, -1, 2], dtype=np.float64)
CRS_I = np.repeat(np.arange(4), 4)
CRS_J = np.tile(np.arange(4), 4)


def _global_coo(ids, Ai, Aj, Av):
    """the matrix crs_setup hands to the setup: entries keyed by global id - 1,
    id-0 dofs and exact zeros dropped, entry order kept"""
    ids = np.asarray(ids, dtype=np.int64)
    I, J = ids[np.asarray(Ai)], ids[np.asarray(Aj)]
    keep = (I != 0) & (J != 0) & (np.asarray(Av) != 0)
    return I[keep] - 1, J[keep] - 1, np.asarray(Av)[keep]


@pytest.mark.parametrize("xid", [[1, 2, 3, 4], [3, 1, 4, 2]], ids=["crs_test_ids", "permuted"])
def test_crs_setup_crs_test_matrix(oracle_lib, xid):
    """crs_test.c:78 -- crs_setup(4, xid, 16, Ai, Aj, A, 1, comm) -- then crs_free"""
    L = oa.lib()
    oa.init()
    hd = abi.crs_setup(L, 4, xid, CRS_I, CRS_J, CRS_A, null_space=1)
    assert hd is not None, oa.lib().amgd_error()
    try:
        h = abi.crs_export(L, hd)
    finally:
        L.crs_free(hd)
    I, J, V = _global_coo(xid, CRS_I, CRS_J, CRS_A)
    ref = abi.run_setup(oracle_lib, I, J, V)
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad
    assert h.nlevels >= 2 and int(h.levels[0].n) == 4


def test_crs_setup_amgdmp_permuted_ids():
    """the reference's bundled matrix presented as a local matrix with scrambled ids,
    shuffled entries and two extra id-0 dofs: the kept hierarchy is the reference's"""
    z = np.load(os.path.join(GOLD, "amgdmp.npz"))
    ref = parity.from_npz(z)
    Ai, Aj, Av = z["in_Ai"].astype(np.int64), z["in_Aj"].astype(np.int64), z["in_Av"]
    n = int(Ai.max()) + 1
    rng = np.random.default_rng(7)
    perm = rng.permutation(n)                    # local dof k has global id perm[k] + 1
    inv = np.empty(n, dtype=np.int64)
    inv[perm] = np.arange(n)
    ids = np.concatenate([perm + 1, [0, 0]])     # local dofs n, n+1: not dofs (id 0)
    li, lj = inv[Ai], inv[Aj]
    # id-0 couplings (dropped), then the real entries in their assembled order (the
    # order fixes the duplicate-summation order; amgdmp has no duplicates)
    ei = np.concatenate([[n, 0, n + 1], li])
    ej = np.concatenate([[0, n, n + 1], lj])
    ev = np.concatenate([[-1.0, -1.0, 5.0], Av])
    oa.init()
    L = oa.lib()
    hd = abi.crs_setup(L, n + 2, ids, ei, ej, ev, null_space=1)
    assert hd is not None
    try:
        h = abi.crs_export(L, hd)
    finally:
        L.crs_free(hd)
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad


def test_crs_setup_rejects_foreign_comm():
    """np > 1 without the library communicator of the same ranks: NULL, not a hang"""
    oa.init()
    hd = abi.crs_setup(oa.lib(), 4, [1, 2, 3, 4], CRS_I, CRS_J, CRS_A, rank=0, np_=2)
    assert hd is None


def test_out_of_hbm_returns_error_and_recovers():
    """an HBM cap far below the setup's need: amgd_setup_device returns -2 with the
    reason in amgd_error() (no abort / core dump), every block the failed setup held
    is released, and the next setup is bit-exact again"""
    import ctypes as C
    oa.init()
    L = oa.lib()
    L.amgd_test_hbm_cap.argtypes = [C.c_uint64]
    L.amgd_test_pool_inuse.restype = C.c_uint64
    Ai, Aj, Av = problems.poisson3d(12)
    ds = oa.DeviceSetup(Ai, Aj, Av)
    try:
        before = L.amgd_test_pool_inuse()
        L.amgd_test_hbm_cap(before + (2 << 20))
        with pytest.raises(RuntimeError, match="out of HBM"):
            ds.run()
        L.amgd_test_hbm_cap(0)
        assert L.amgd_test_pool_inuse() == before
        # amg_setup (void) leaves nlevels = 0 behind on the same failure
        L.amgd_test_hbm_cap(before + (2 << 20))
        h0 = abi.run_setup(L, Ai, Aj, Av)
        L.amgd_test_hbm_cap(0)
        assert h0.nlevels == 0
        assert L.amgd_test_pool_inuse() == before
    finally:
        L.amgd_test_hbm_cap(0)
    ds.run()
    z = np.load(os.path.join(GOLD, "p7_12.npz"))
    bad = parity.compare(parity.from_npz(z), ds.export(), exact=True)
    ds.close()
    assert not bad, bad


@pytest.mark.parametrize("frac", [0.25, 0.5, 0.75, 0.9])
@pytest.mark.parametrize("gen", [("p7_24", lambda: problems.poisson3d(24)),
                                 ("p27_12", lambda: problems.poisson3d(12, 27))],
                         ids=lambda g: g[0])
def test_out_of_hbm_mid_setup_recovers(gen, frac):
    """the HBM cap set to a fraction of the setup's measured peak, so the failure lands
    deep inside the setup (interpolation's products, Q factors with reuse, the pattern-only
    constraint product, RAP) rather than at its first allocation: -2 with the reason, every
    block released (pool in use back to its value before), and the next setup bit-exact
    with an uncapped one (per-call state -- SpGEMM pattern mode, Q-factor reuse
    pointers -- is reset after the unwind)"""
    import ctypes as C
    oa.init()
    L = oa.lib()
    L.amgd_test_hbm_cap.argtypes = [C.c_uint64]
    L.amgd_test_pool_inuse.restype = C.c_uint64
    Ai, Aj, Av = gen[1]()
    ds = oa.DeviceSetup(Ai, Aj, Av)
    try:
        ds.run()
        ref = ds.export()
        peak = oa.stats()["peak_bytes"]          # this setup's peak (reset at its start)
        L.amgd_hier_free(C.byref(ds.h))
        before = L.amgd_test_pool_inuse()
        assert peak > before
        L.amgd_test_hbm_cap(before + int((peak - before) * frac))
        with pytest.raises(RuntimeError, match="out of HBM"):
            ds.run()
        L.amgd_test_hbm_cap(0)
        assert L.amgd_test_pool_inuse() == before
        ds.run()
        bad = parity.compare(ref, ds.export(), exact=True)
        assert not bad, bad
    finally:
        L.amgd_test_hbm_cap(0)
        ds.close()


def test_crs_setup_rejects_bad_local_index():
    """a local index >= n: NULL with the reason in amgd_error(), not a silent drop"""
    oa.init()
    Ai = CRS_I.copy()
    Ai[5] = 4
    hd = abi.crs_setup(oa.lib(), 4, [1, 2, 3, 4], Ai, CRS_J, CRS_A)
    assert hd is None
    assert b"local index" in oa.lib().amgd_error()


def test_amg_setup_rejects_index_past_32_bits():
    """amg_setup (no status in amg_setup.h:5) with an index past the device CSR's 32-bit
    range: nlevels = 0 and the reason in amgd_error(), then a valid call works"""
    oa.init()
    Ai = np.asarray(CRS_I, np.uint64).copy()
    Ai[3] = 1 << 32
    h = abi.run_setup(oa.lib(), Ai, CRS_J, CRS_A)
    assert h.nlevels == 0
    assert b"32-bit" in oa.lib().amgd_error()
    h = abi.run_setup(oa.lib(), CRS_I, CRS_J, CRS_A)
    assert h.nlevels > 0
