"""Row-sharded setup (amgd_comm.hip, DESIGN.md "Multi-GPU") on one MI355X.

  * sim transport: one process computes every shard in turn -- the work split,
    the shard-range kernels and the assembly into the global CSR / Q buffers are
    exercised with N = 2, 3, 8 shards and every op sharded (min work 0); the
    hierarchy must stay bit-identical to the reference fixtures.
  * host transport: 2 and 3 processes on the same GPU, gloo-staged allgatherv
    (tests/shard_worker.py) -- the same collectives the RCCL transport issues.
  * RCCL: a one-rank communicator initialises and frees (the multi-rank RCCL path
    needs one GPU per rank; it runs in bench.py --gpus N).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch  # noqa: F401  -- pages torch in at collection (the workers import it too)

from conftest import GOLD, ROOT
import omp_amg_amd as oa
from omp_amg_amd import abi, parity, problems, shard

pytestmark = pytest.mark.gpu
CASES = ["p7_12", "p27_8", "sem_e3_N2", "aniso_12", "amgdmp"]


def _case(name):
    path = os.path.join(GOLD, name + ".npz")
    if not os.path.exists(path):
        pytest.skip(f"no fixture {name}")
    z = np.load(path)
    return parity.from_npz(z), z["in_Ai"], z["in_Aj"], z["in_Av"]


@pytest.fixture
def sim():
    oa.init()

    def on(n):
        shard.init_sim(n)
        shard.set_min_work(0.0)
    yield on
    shard.set_min_work(1.0)
    shard.free()


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("case", CASES)
def test_sim_shards_bitexact_fixture(sim, case, n):
    ref, Ai, Aj, Av = _case(case)
    sim(n)
    h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    bad = parity.compare(ref, h, exact=True)
    assert not bad, bad


@pytest.mark.parametrize("gen", [("p7_32", lambda: problems.poisson3d(32)),
                                 ("p27_16", lambda: problems.poisson3d(16, 27)),
                                 ("sem_e4_N3", lambda: problems.sem_laplacian(4, 4, 3, 3, seed=3, jitter=0.2))],
                         ids=lambda g: g[0])
def test_sim_shards_match_one_gpu(sim, gen):
    Ai, Aj, Av = gen[1]()
    h1 = abi.run_setup(oa.lib(), Ai, Aj, Av)
    sim(5)
    h5 = abi.run_setup(oa.lib(), Ai, Aj, Av)
    bad = parity.compare(h1, h5, exact=True)
    assert not bad, bad


def test_sim_default_thresholds_48():
    """default work thresholds: a 48^3 setup shards its larger products only"""
    oa.init()
    Ai, Aj, Av = problems.poisson3d(48)
    h1 = abi.run_setup(oa.lib(), Ai, Aj, Av)
    shard.init_sim(4)
    try:
        h4 = abi.run_setup(oa.lib(), Ai, Aj, Av)
    finally:
        shard.free()
    bad = parity.compare(h1, h4, exact=True)
    assert not bad, bad


def test_sim_sharded_spgemm_kernel(sim):
    """X = A*B through the sharded dispatcher vs one GPU, random ragged operands
    (empty rows, a dense row, rows that cancel exactly)"""
    rng = np.random.default_rng(7)

    def rand_csr(rn, cn, dens):
        M = (rng.random((rn, cn)) < dens) * rng.integers(-3, 4, size=(rn, cn)).astype(float)
        M[rn // 3] = 0.0
        M[rn // 2, :] = rng.integers(1, 3, size=cn)
        ro = np.concatenate([[0], np.cumsum((M != 0).sum(1))])
        r, c = np.nonzero(M)
        return abi.Csr(rn, cn, ro, c, M[r, c])
    A, B = rand_csr(300, 200, 0.05), rand_csr(200, 250, 0.08)
    X1 = oa.test_csr_op(0, A, B)
    sim(3)
    X3 = oa.test_csr_op(0, A, B)
    assert np.array_equal(X1.row_off, X3.row_off)
    assert np.array_equal(X1.col, X3.col)
    assert np.array_equal(X1.a.view(np.uint64), X3.a.view(np.uint64))


@pytest.mark.parametrize("n", [2, 3, 7])
def test_sim_sharded_spmv_kernel(sim, n):
    """whole-matrix long-row SpMV split by nnz over n shards (lane kernel on each row
    range, allgatherv of z) vs one GPU, bit for bit: ragged rows (empty, short, one of
    5000 entries), plain / y-scaled / row-sum forms"""
    rng = np.random.default_rng(11 + n)
    rn, cn = 3000, 2500
    lens = rng.integers(0, 80, size=rn)
    lens[::97] = 0
    lens[1234] = 2400
    lens[2999] = 2500
    ro = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    col = np.concatenate([np.sort(rng.choice(cn, size=l, replace=False)) for l in lens]).astype(np.uint32)
    a = rng.standard_normal(int(ro[-1])) * np.exp2(rng.integers(-30, 30, size=int(ro[-1])))
    A = abi.Csr(rn, cn, ro, col, a)
    x = rng.standard_normal(cn)
    y = rng.standard_normal(rn)
    oa.spmv_sl_min(0)
    try:
        z1 = oa.test_spmv(A, x)
        zy1 = oa.test_spmv(A, x, alpha=0.5, y=y, beta=-2.0)
        zs1 = oa.test_spmv_f(A)
        c0 = oa.lib().amgd_test_spmv_shard_calls()
        sim(n)
        z = oa.test_spmv(A, x)
        zy = oa.test_spmv(A, x, alpha=0.5, y=y, beta=-2.0)
        zs = oa.test_spmv_f(A)
        assert oa.lib().amgd_test_spmv_shard_calls() - c0 == 3
    finally:
        oa.spmv_sl_min(-1)
    for u, v in ((z1, z), (zy1, zy), (zs1, zs)):
        assert np.array_equal(u.view(np.uint64), v.view(np.uint64))


@pytest.mark.parametrize("gen", [("sem_e4_N3", lambda: problems.sem_laplacian(4, 4, 3, 3, seed=3, jitter=0.2)),
                                 ("p27_20", lambda: problems.poisson3d(20, 27))],
                         ids=lambda g: g[0])
def test_sim_sharded_spmv_setup(sim, gen):
    """full setup with every long-row whole-matrix SpMV sharded (lane kernel forced at
    every size, min work 0) vs one GPU: the hierarchy is bit-identical"""
    Ai, Aj, Av = gen[1]()
    oa.spmv_sl_min(0)
    try:
        h1 = abi.run_setup(oa.lib(), Ai, Aj, Av)
        c0 = oa.lib().amgd_test_spmv_shard_calls()
        sim(4)
        h4 = abi.run_setup(oa.lib(), Ai, Aj, Av)
        assert oa.lib().amgd_test_spmv_shard_calls() > c0
    finally:
        oa.spmv_sl_min(-1)
    bad = parity.compare(h1, h4, exact=True)
    assert not bad, bad


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("size,case,crs", [(2, "gold:p7_12", ""), (2, "gold:sem_e3_N2", ""),
                                           (3, "gold:p27_8", ""), (2, "p27:14", ""),
                                           (2, "gold:amgdmp", "1"), (3, "gold:p7_12", "1")],
                         ids=["p7_12x2", "sem_e3_N2x2", "p27_8x3", "p27_14x2", "crs_amgdmp_x2",
                              "crs_p7_12x3"])
def test_host_transport_processes(size, case, crs):
    """crs="1": crs_setup(comm = {rank, size}) with each rank passing its own block of
    rows; the gathered, sharded hierarchy is the reference's fixture bit for bit"""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(size),
               SHARD_CASE=case, SHARD_CRS=crs, PYTHONPATH=ROOT)
    ps = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "shard_worker.py")],
                           env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True) for r in range(size)]
    outs = []
    for p in ps:
        try:
            o, e = p.communicate(timeout=110)
        except subprocess.TimeoutExpired:
            for q in ps:
                q.kill()
            raise
        outs.append((p.returncode, o, e[-2000:]))
    for rc, o, e in outs:
        assert rc == 0, (o, e)
        d = json.loads(o.strip().splitlines()[-1])
        assert not d["bad"] and d["calls"] > 0, d


def test_rccl_one_rank_init():
    """librccl loads, a one-rank communicator initialises on the library stream and frees"""
    oa.init()
    import ctypes as C
    L = oa.lib()
    uid = C.create_string_buffer(128)
    assert L.amgd_comm_rccl_uid(uid) == 0
    assert L.amgd_comm_init_rccl(0, 1, uid.raw) == 0
    try:
        assert L.amgd_comm_size() == 1
        Ai, Aj, Av = problems.poisson3d(8)
        h = abi.run_setup(L, Ai, Aj, Av)
        assert h.nlevels > 1
    finally:
        shard.free()
