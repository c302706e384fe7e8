"""Multi-GPU row sharding of the setup (amgd_comm.hip, DESIGN.md "Multi-GPU").

Every rank runs the setup on the same matrix with its HIP device; the library
splits the row-independent heavy kernels (SpGEMMs, Q factors) by work across the
ranks and completes each result with an in-place allgatherv.  Three transports:

  init_rccl(rank, size, group)  RCCL over xGMI (production; the unique id is
                                broadcast over the torch.distributed control group)
  init_host(rank, size, group)  allgatherv staged through host memory over a
                                torch.distributed (gloo) group: tests with several
                                processes on ONE GPU, where RCCL refuses to run
  init_sim(n)                   one process computes all n shards in turn (tests)

`free()` returns to one GPU.  Python here is plumbing for the C ABI, not a compute path.
"""
from __future__ import annotations

import ctypes as C
import traceback

import numpy as np

ALLGATHERV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_void_p),
                            C.POINTER(C.c_uint64), C.c_int, C.c_int)
_keep = []          # callbacks must outlive the library's use of them


def _lib():
    from . import lib
    return lib()


def host_allgatherv(group, download, upload):
    """allgatherv callback over a torch.distributed group, staged through host memory.

    download(host_addr, dev_addr, n) / upload(dev_addr, host_addr, n) move bytes
    between the device buffer and host (amgd_dev_download/upload on a GPU; memmove
    in the CPU tests).  Ranges are padded to the longest for gloo's all_gather."""
    import torch
    import torch.distributed as dist

    def fn(user, nbuf, bufs, offs, rank, size):
        try:
            for b in range(nbuf):
                o = [int(offs[b * (size + 1) + s]) for s in range(size + 1)]
                lens = [o[s + 1] - o[s] for s in range(size)]
                mx = max(lens)
                if mx == 0:
                    continue
                mine = np.zeros(mx, dtype=np.uint8)
                base = bufs[b]
                if lens[rank]:
                    download(mine.ctypes.data, base + o[rank], lens[rank])
                outs = [torch.empty(mx, dtype=torch.uint8) for _ in range(size)]
                dist.all_gather(outs, torch.from_numpy(mine), group=group)
                for s in range(size):
                    if s != rank and lens[s]:
                        h = outs[s].numpy()
                        upload(base + o[s], h.ctypes.data, lens[s])
            return 0
        except Exception:  # noqa: BLE001 -- reported, then the library aborts loudly
            traceback.print_exc()
            return 1
    return fn


def init_host(rank: int, size: int, group=None) -> None:
    L = _lib()
    dl = lambda h, d, n: L.amgd_dev_download(C.c_void_p(h), C.c_void_p(d), n)  # noqa: E731
    ul = lambda d, h, n: L.amgd_dev_upload(C.c_void_p(d), C.c_void_p(h), n)    # noqa: E731
    cb = ALLGATHERV_FN(host_allgatherv(group, dl, ul))
    _keep.append(cb)
    if L.amgd_comm_init_host(rank, size, C.cast(cb, C.c_void_p), None) != 0:
        raise RuntimeError("amgd_comm_init_host failed")


def init_rccl(rank: int, size: int, group=None) -> None:
    """RCCL communicator of the library (its own, on the library stream); the
    unique id travels over the torch.distributed control group (size 1: none needed)."""
    L = _lib()
    uid = C.create_string_buffer(128)
    if rank == 0 and L.amgd_comm_rccl_uid(uid) != 0:
        raise RuntimeError("amgd_comm_rccl_uid failed (librccl missing?)")
    box = [bytes(uid.raw)]
    if size > 1:
        import torch.distributed as dist
        dist.broadcast_object_list(box, src=0, group=group)
    # RCCL prints its version banner on stdout at communicator creation: keep stdout for
    # the caller's own output (bench.py's one JSON line) by sending fd 1 to stderr meanwhile
    import os
    import sys
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        rc = L.amgd_comm_init_rccl(rank, size, box[0])
        C.CDLL(None).fflush(None)
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    if rc != 0:
        raise RuntimeError(f"amgd_comm_init_rccl failed rc={rc}")


def init_sim(n: int) -> None:
    if _lib().amgd_comm_init_sim(int(n)) != 0:
        raise RuntimeError("amgd_comm_init_sim failed")


def free() -> None:
    _lib().amgd_comm_free()


def set_min_work(scale: float) -> None:
    """scale of the per-op minimum work for sharding (0: shard every op; 1: default)"""
    _lib().amgd_comm_set_min_work(float(scale))


def stats(reset: bool = False) -> dict:
    L = _lib()
    c, b, ms = C.c_uint64(), C.c_uint64(), C.c_double()
    L.amgd_comm_stats(C.byref(c), C.byref(b), C.byref(ms))
    if reset:
        L.amgd_comm_stats_reset()
    return {"calls": c.value, "bytes": b.value, "ms": ms.value}
