"""The row-partitioned multi-GPU setup (north_star: rows sharded over the
GPUs, halo rows exchanged before each product).  N processes share the test box's one GPU
over the host transport (tests/part_worker.py); each passes only its slice of the
entries, holds only its row blocks of every matrix, and the gathered hierarchy must equal
the reference's fixture or the oracle digest bit for bit -- the one-GPU parity contract."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(size, case, crs="", timeout=110, extra_env=None):
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(size),
               PART_CASE=case, PART_CRS=crs, PYTHONPATH=ROOT, AMGD_ARENA_GB="8", **(extra_env or {}))
    ps = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "part_worker.py")],
                           env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True) for r in range(size)]
    outs = []
    for p in ps:
        try:
            o, e = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in ps:
                q.kill()
            raise
        outs.append((p.returncode, o, e[-3000:]))
    res = []
    if any(rc != 0 for rc, _, _ in outs):
        # every rank's tail: the first failing rank is usually not rank 0
        raise AssertionError("\n".join(f"--- rank {r} rc={rc}\n{o[-1500:]}\n{e}" for r, (rc, o, e) in enumerate(outs)))
    for rc, o, e in outs:
        assert rc == 0, (o[-2000:], e)
        d = json.loads(o.strip().splitlines()[-1])
        assert not d["bad"] and d["calls"] > 0 and d["leak_bytes"] == 0, d
        res.append(d)
    return res


@pytest.mark.parametrize("size,case", [(2, "gold:p7_12"), (3, "gold:p27_8"), (2, "gold:sem_e3_N2"),
                                       (2, "gold:amgdmp"), (4, "gold:aniso_12"), (3, "gold:p7_16x6x5"),
                                       (2, "gold:sem_e2_N5")],
                         ids=lambda v: str(v).replace("gold:", ""))
def test_partitioned_matches_reference_fixture(size, case):
    """each rank passes 1/size of the entries; the partitioned hierarchy (row blocks of
    every level, halo products, distributed transposes) is the reference's fixture"""
    _run(size, case)


@pytest.mark.parametrize("size,case", [(3, "digest:p7_48"), (2, "digest:p27_20"), (3, "digest:sem_e4_N7"),
                                       (2, "digest:aniso_20"), (4, "digest:p7_64")],
                         ids=lambda v: str(v).replace("digest:", ""))
@pytest.mark.parametrize("inc", ["1", "0"], ids=["inc", "full_sweeps"])
def test_partitioned_matches_digest(size, case, inc):
    """larger grids: the gathered partitioned hierarchy hashes to the stored oracle /
    reference digest (every array of every level); incremental coarsening / find_support
    sweeps across the ranks (default) and full sweeps"""
    _run(size, case, timeout=240, extra_env={"AMGD_CS_INC": inc, "AMGD_FS_INC": inc})


@pytest.mark.parametrize("case", ["gold:amgdmp", "gold:p27_8", "digest:p7_48"],
                         ids=lambda v: v.split(":")[1])
def test_partitioned_eight_ranks(case):
    """8 ranks -- the north_star's GPU count -- on small fixtures (coarse levels leave
    ranks with no rows: empty blocks, empty halos, empty segments in every exchange) and
    on the 7-point 48^3 digest (110 k rows, 13.8 k per rank)"""
    _run(8, case, timeout=240)


def test_partitioned_crs_setup():
    """crs_setup(comm = {rank, 3}) in partitioned mode: each rank's local rows go straight
    to the partitioned setup (no gather of the matrix); the reference fixture bit for bit"""
    _run(3, "gold:p7_12", crs="1")


@pytest.mark.parametrize("case", ["p7_48", "p27_20", "sem_e4_N7"])
def test_partitioned_one_rank_rccl(case):
    """the partitioned driver with a one-rank RCCL communicator (every partitioned
    operation on a single block: views, halo builder, transpose assembly, selections) in
    this process: the stored digest"""
    import ctypes as C
    import omp_amg_amd as oa
    from omp_amg_amd import abi, shard
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_digests as md
    d = json.load(open(md.OUT))["cases"][case]
    Ai, Aj, Av = md.generate(d["gen"])
    oa.init()
    L = oa.lib()
    uid = C.create_string_buffer(128)
    assert L.amgd_comm_rccl_uid(uid) == 0
    assert L.amgd_comm_init_rccl(0, 1, uid.raw) == 0
    try:
        L.amgd_comm_set_partitioned(1)
        assert L.amgd_comm_partitioned() == 1
        h = abi.run_setup(L, Ai, Aj, Av)
    finally:
        shard.free()
    got = md.hierarchy_digest(h)
    bad = sorted(k for k in set(got) | set(d["arrays"]) if got.get(k) != d["arrays"].get(k))
    assert not bad, bad[:8]
