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

# heavy variants whose paths the default suite already covers at another size or rank count
# (kept for full runs: AMGD_TESTS_EXTENDED=1); the round-end GPU suite must stay well inside
# the driver's time limit (round 6: 892 s for the whole suite with them)
EXT = pytest.mark.skipif(os.environ.get("AMGD_TESTS_EXTENDED", "0") != "1",
                         reason="extended variant (AMGD_TESTS_EXTENDED=1)")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(size, case, crs="", extra_env=None):
    port = _free_port()
    # every partitioned test runs with the collective-consistency guard on
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(size),
               PART_CASE=case, PART_CRS=crs, PYTHONPATH=ROOT, AMGD_COMM_CHECK="1",
               # PART_ARENA_GB: each rank's arena (0: every block from hipMalloc, the mode a
               # rank falls into when the GPU has too little free memory for an arena)
               AMGD_ARENA_GB=os.environ.get("PART_ARENA_GB", "8"),
               **(extra_env or {}))
    return [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "part_worker.py")],
                             env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             text=True) for r in range(size)]


def _run(size, case, crs="", timeout=110, extra_env=None):
    ps = _spawn(size, case, crs, extra_env)
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
        # the whole last line of each rank: the full list of differing arrays and, for digest
        # cases, the first differing row of each against the one-GPU setup (part_worker.py)
        raise AssertionError("\n".join(f"--- rank {r} rc={rc}\n{o[-30000:]}\n{e}" for r, (rc, o, e) in enumerate(outs)))
    for rc, o, e in outs:
        assert rc == 0, (o[-2000:], e)
        d = json.loads(o.strip().splitlines()[-1])
        assert not d["bad"] and d["calls"] > 0 and d["leak_bytes"] == 0, d
        res.append(d)
    print(size, case, json.dumps({k: res[0].get(k) for k in ("calls", "lmop_gathered", "lmop_prefix",
                                                              "eager_calls", "eager_second", "levels")}))
    return res


@pytest.mark.parametrize("size,case", [(2, "gold:p7_12"), (3, "gold:p27_8"), (2, "gold:sem_e3_N2"),
                                       (2, "gold:amgdmp"), (4, "gold:aniso_12"), (3, "gold:p7_16x6x5"),
                                       (2, "gold:sem_e2_N5")],
                         ids=lambda v: str(v).replace("gold:", ""))
def test_partitioned_matches_reference_fixture(size, case):
    """each rank passes 1/size of the entries; the partitioned hierarchy (row blocks of
    every level, halo products, distributed transposes) is the reference's fixture"""
    _run(size, case)


_DIGEST_CASES = [(3, "digest:p7_48"), (2, "digest:p27_20"), (3, "digest:sem_e4_N7"), (2, "digest:aniso_20"),
                 (4, "digest:p7_64")]


@pytest.mark.parametrize("size,case,inc",
                         [pytest.param(s, c, i, id=f"{'inc' if i == '1' else 'full_sweeps'}-{s}-{c[7:]}",
                                       marks=[EXT] if i == "0" and s >= 3 and c.startswith("digest:p7") else [])
                          for i in ("1", "0") for s, c in _DIGEST_CASES])
def test_partitioned_matches_digest(size, case, inc):
    """larger grids: the gathered partitioned hierarchy hashes to the stored oracle /
    reference digest (every array of every level); incremental coarsening / find_support
    sweeps across the ranks (default) and full sweeps (the 7-point 48^3 / 64^3 full-sweep
    variants on 3-4 ranks are extended-only: full sweeps stay covered on 2 ranks here and
    the 8-rank 27-point case)"""
    _run(size, case, timeout=170, extra_env={"AMGD_CS_INC": inc, "AMGD_FS_INC": inc})


@pytest.mark.parametrize("case", ["gold:amgdmp", pytest.param("gold:p27_8", marks=EXT),
                                  pytest.param("digest:p7_48", marks=EXT), "digest:p27_20"],
                         ids=lambda v: v.split(":")[1])
def test_partitioned_eight_ranks(case):
    """8 ranks -- the north_star's GPU count -- on small fixtures (coarse levels leave
    ranks with no rows: empty blocks, empty halos, empty segments in every exchange), on
    the 7-point 48^3 digest (110 k rows, 13.8 k per rank) and on the 27-point 20^3 digest
    (configs[3]'s stencil: the densified levels, interp_lmop's dirty points past clean
    ones -- the reference-checked hierarchy)"""
    _run(8, case, timeout=240)


@pytest.mark.parametrize("force", ["lmop_gather", "eager_slot"])
def test_partitioned_forced_rare_paths(force):
    """the r05t1 case (4 ranks, incremental sweeps, 7-point 64^3) with a rare path forced
    at every call: interp_lmop redone on gathered data (its fallback when a view walk
    spills or a clean contribution misses: 0 calls at 128^3 by default), or an 8-byte eager
    slot, so every variable-length exchange (BFS hops, find_support expansions and
    selections) that moves more than 8 bytes takes the exact second round -- the stored
    digest either way, with the forced path counted on every rank"""
    env = {"AMGD_CS_INC": "1", "AMGD_FS_INC": "1"}
    env.update({"PART_LMOP_GATHER": "1"} if force == "lmop_gather" else {"PART_EAGER_SLOT": "8"})
    res = _run(4, "digest:p7_64", timeout=240, extra_env=env)
    for d in res:
        if force == "lmop_gather":
            assert d["lmop_gathered"] > 0, d
        else:
            assert d["eager_second"] > 0 and 2 * d["eager_second"] > d["eager_calls"], d


def test_partitioned_crs_setup():
    """crs_setup(comm = {rank, 3}) in partitioned mode: each rank's local rows go straight
    to the partitioned setup (no gather of the matrix); the reference fixture bit for bit"""
    _run(3, "gold:p7_12", crs="1")


def test_crs_setup_defaults_to_partitioned():
    """crs_setup(comm = {rank, 2}) with no mode chosen runs the partitioned setup (each
    rank's rows stay on it; the matrix is never gathered): the reference fixture"""
    _run(2, "gold:p7_12", crs="1", extra_env={"PART_DEFAULT": "1"})


def _gpus():
    import torch
    return torch.cuda.device_count()          # counts devices without initialising one


@pytest.mark.skipif(_gpus() < 2, reason="needs >= 2 GPUs (one rank per GPU over RCCL)")
@pytest.mark.parametrize("case", ["digest:p7_48", "gold:aniso_12"])
def test_partitioned_two_ranks_rccl(case):
    """the partitioned driver over the library's RCCL communicator with two ranks on two
    GPUs (xGMI send/recv groups for every halo fetch, transpose and route; the host
    transport of the other tests stages them through gloo): bit-identical to the
    one-GPU digest / reference fixture, with the collective guard on"""
    _run(2, case, timeout=170, extra_env={"PART_TRANSPORT": "rccl"})


def test_amg_setup_under_partitioned_comm():
    """amg_setup with a 2-process partitioned communicator: each process passes the whole
    matrix (the reference's meaning) and gets the one-GPU hierarchy with no exchange;
    then the partitioned setup of the same ranks matches it bit for bit"""
    _run(2, "gold:amgdmp", extra_env={"PART_AMG_SETUP": "1"})


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


@pytest.mark.parametrize("what", ["kind", "size"])
def test_collective_guard_aborts_every_rank(what):
    """AMGD_COMM_CHECK=1: rank 1 enters an alltoallv where rank 0 enters an allgatherv
    (a rank-local skip, round 4's r04e fault), or expects 32 bytes where rank 0 sends 64:
    both ranks abort, naming the mismatch, instead of corrupting or hanging"""
    ps = _spawn(2, "gold:p7_4", extra_env={"PART_GUARD": what})
    outs = []
    for p in ps:
        try:
            o, e = p.communicate(timeout=90)
        except subprocess.TimeoutExpired:
            for q in ps:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    for r, (rc, o, e) in enumerate(outs):
        assert rc != 0, f"rank {r} did not abort: {o[-500:]}"
        assert "COLLECTIVE MISMATCH" in e, f"rank {r}: {e[-1500:]}"
        assert "no abort" not in o


def test_out_of_hbm_on_one_rank_unwinds_all():
    """rank 1 of 2 runs out of HBM mid-setup: with the guard every rank's setup returns
    -2 (the failure travels in the guard record), no device bytes stay held, and the
    ranks' next setup is the reference fixture bit for bit"""
    res = _run(2, "gold:p7_12", extra_env={"PART_OOM": "0.5"})
    assert all("out of HBM" in d.get("error", "") or "failed" in d.get("error", "") for d in res), res
