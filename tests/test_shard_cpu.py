"""Multi-rank host logic of the row sharding (omp_amg_amd/shard.py) on the CPU:
the host-staged allgatherv transport over a world_size-2 gloo group, driven
through the same ctypes callback type the library calls (amgd_comm.hip), with
host buffers standing in for device buffers.  Ranges of unequal and zero length,
several buffers per call, as the sharded SpGEMM issues them (ro, col, a)."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from omp_amg_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        mv = lambda dst, src, n: C.memmove(dst, src, n)  # noqa: E731
        cb = shard.ALLGATHERV_FN(shard.host_allgatherv(None, mv, mv))
        # three buffers with the layouts of a sharded CSR: shard ranges of unequal
        # lengths, one empty range, a buffer where one rank owns everything
        lens = [[5, 0, 7][:size], [3, 9, 1][:size], [0, 16, 0][:size]]
        bufs, offs, want = [], [], []
        rng = np.random.default_rng(1234)
        for L in lens:
            full = rng.integers(0, 256, size=sum(L), dtype=np.uint8)
            o = np.concatenate([[0], np.cumsum(L)]).astype(np.uint64)
            mine = np.zeros_like(full)
            mine[o[rank]:o[rank + 1]] = full[o[rank]:o[rank + 1]]
            bufs.append(mine)
            offs.extend(o.tolist())
            want.append(full)
        ptrs = (C.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
        off_arr = (C.c_uint64 * len(offs))(*offs)
        rc = cb(None, len(bufs), ptrs, off_arr, rank, size)
        ok = rc == 0 and all(np.array_equal(b, w) for b, w in zip(bufs, want))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size", [2, 3])
def test_host_allgatherv_gloo(size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res
    assert all(p.exitcode == 0 for p in ps)


def test_comm_symbols_exported():
    """the multi-GPU entry points of include/omp_amg_amd.h are exported (no GPU call)"""
    from omp_amg_amd import lib
    L = lib()
    for name in ("amgd_comm_rccl_uid", "amgd_comm_init_rccl", "amgd_comm_init_host",
                 "amgd_comm_init_sim", "amgd_comm_free", "amgd_comm_size", "amgd_comm_rank",
                 "amgd_comm_set_min_work", "amgd_comm_stats", "amgd_comm_stats_reset"):
        assert hasattr(L, name), name
    assert L.amgd_comm_init_sim(0) != 0          # argument check, no device touched
    assert L.amgd_comm_init_host(2, 2, None, None) != 0
