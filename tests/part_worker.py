"""One rank of the partitioned-setup tests (tests/test_gpu_partition.py).

Launched N times on the same GPU with RANK / WORLD_SIZE / MASTER_PORT set: gloo group,
host-staged transport (RCCL refuses two ranks on one device), partitioned mode.  Each
rank passes only ITS slice of the COO entries (a contiguous 1/N of them, or -- with
PART_CRS -- its block of rows as a crs_setup local matrix); the library routes them to
the row owners, builds the row-partitioned hierarchy, and the exported (gathered)
hierarchy is compared bit for bit with the reference fixture or the stored digest.
Prints one JSON line (per-rank peak HBM bytes and the device bytes left allocated after
the setup returned -- 0 -- included); exit code 0 = pass."""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, "golden"))
import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import omp_amg_amd as oa  # noqa: E402
from omp_amg_amd import abi, parity, shard  # noqa: E402


def main():
    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=size)
    # PART_TRANSPORT=rccl (>= size GPUs): one GPU per rank, the library's RCCL communicator
    # over xGMI -- the send/recv groups of the halo fetches, transposes and routes
    rccl = os.environ.get("PART_TRANSPORT") == "rccl"
    oa.init(rank if rccl else 0)
    L = oa.lib()
    L.amgd_test_pool_inuse.restype = C.c_uint64
    before = L.amgd_test_pool_inuse()
    case = os.environ["PART_CASE"]
    out = {"rank": rank, "case": case, "size": size}
    ref = digest = None
    if case.startswith("gold:"):
        z = np.load(os.path.join(HERE, "golden", case[5:] + ".npz"))
        ref = parity.from_npz(z)
        Ai, Aj, Av = z["in_Ai"], z["in_Aj"], z["in_Av"]
    else:
        import make_digests as md
        digest = json.load(open(md.OUT))["cases"][case[7:]]
        Ai, Aj, Av = md.generate(digest["gen"])
    if rccl:
        shard.init_rccl(rank, size)
    else:
        shard.init_host(rank, size)
    if not os.environ.get("PART_DEFAULT"):     # PART_DEFAULT: crs_setup's own default (partitioned)
        oa.lib().amgd_comm_set_partitioned(1)
    # forced rare paths (tests): every interp_lmop on gathered data; a fixed eager slot
    L.amgd_test_part_force.argtypes = [C.c_int, C.c_int64]
    L.amgd_test_part_force(int(os.environ.get("PART_LMOP_GATHER", "0")),
                           int(os.environ.get("PART_EAGER_SLOT", "0")))
    shard.stats(reset=True)
    Ai64, Aj64, Av = np.asarray(Ai, np.int64), np.asarray(Aj, np.int64), np.asarray(Av)
    guard = os.environ.get("PART_GUARD")
    if guard:
        # the collective guard (AMGD_COMM_CHECK=1 in the env) must abort every rank on a
        # kind / size disagreement: rank 1 enters a different collective (kind) or
        # expects other byte counts (size) than rank 0 sends
        L.amgd_test_comm.argtypes = [C.c_int, C.c_uint64, C.c_uint64]
        L.amgd_test_comm(1, 64, 64)                         # agreeing alltoallv: passes
        L.amgd_test_comm(0, 64, 0)                          # agreeing allgatherv: passes
        if guard == "kind":
            L.amgd_test_comm(0 if rank == 0 else 1, 64, 64)
        else:
            L.amgd_test_comm(1, 64, 64 if rank == 0 else 32)
        print(json.dumps({"rank": rank, "unexpected": "no abort"}), flush=True)
        sys.exit(0)
    if os.environ.get("PART_OOM"):
        # rank 1 runs out of HBM inside the partitioned setup; with the guard on, every
        # rank's setup unwinds and returns -2 (none aborts), nothing stays allocated, and
        # the next setup of the same ranks is the fixture
        L.amgd_test_hbm_cap.argtypes = [C.c_uint64]
        nz = len(Av)
        k0, k1 = rank * nz // size, (rank + 1) * nz // size
        ds = oa.DeviceSetup(Ai64[k0:k1], Aj64[k0:k1], Av[k0:k1])
        held = L.amgd_test_pool_inuse()
        ds.run()                                  # uncapped: this rank's peak
        peak = int(oa.stats()["peak_bytes"])
        ds.close()
        ds = oa.DeviceSetup(Ai64[k0:k1], Aj64[k0:k1], Av[k0:k1])
        held = L.amgd_test_pool_inuse()
        if rank == 1:                             # a cap at PART_OOM of the way to the peak
            L.amgd_test_hbm_cap(held + int((peak - held) * float(os.environ["PART_OOM"])))
        failed = False
        try:
            ds.run()
        except RuntimeError as e:
            failed = True
            out["error"] = str(e)[:200]
        L.amgd_test_hbm_cap(0)
        assert failed, "the capped setup did not fail on this rank"
        assert L.amgd_test_pool_inuse() == held, (L.amgd_test_pool_inuse(), held)
        ds.run()
        h = ds.export()
        ds.close()
    elif os.environ.get("PART_AMG_SETUP"):
        # amg_setup (amg_setup.h:5) takes the WHOLE matrix on every calling process, also
        # with a partitioned multi-process communicator: no exchange, the one-GPU setup
        h = abi.run_setup(oa.lib(), Ai64, Aj64, Av)
        st = shard.stats()
        assert st["calls"] == 0, st
        shard.stats(reset=True)
        # then the same ranks' partitioned setup still works (nothing left suspended)
        nz = len(Av)
        k0, k1 = rank * nz // size, (rank + 1) * nz // size
        ds = oa.DeviceSetup(Ai64[k0:k1], Aj64[k0:k1], Av[k0:k1])
        ds.run()
        h2 = ds.export()
        ds.close()
        bad2 = parity.compare(h, h2, exact=True)
        assert not bad2, bad2[:5]
    elif os.environ.get("PART_CRS"):
        n = int(max(Ai64.max(), Aj64.max())) + 1
        lo, hi = rank * n // size, (rank + 1) * n // size
        sel = (Ai64 >= lo) & (Ai64 < hi)
        ids = np.arange(1, n + 1, dtype=np.uint64)
        hd = abi.crs_setup(oa.lib(), n, ids, Ai64[sel], Aj64[sel], Av[sel], rank=rank, np_=size)
        assert hd is not None, "crs_setup returned NULL"
        h = abi.crs_export(oa.lib(), hd)
        oa.lib().crs_free(hd)
    else:
        # amgd_setup_device (omp_amg_amd.h): in partitioned mode its COO is this rank's
        # share of the matrix (amg_setup keeps the reference's whole-matrix meaning)
        nz = len(Av)
        k0, k1 = rank * nz // size, (rank + 1) * nz // size
        ds = oa.DeviceSetup(Ai64[k0:k1], Aj64[k0:k1], Av[k0:k1])
        ds.run()
        h = ds.export()
        ds.close()
    st = shard.stats()
    out["peak_bytes"] = int(oa.stats()["peak_bytes"])
    ps = (C.c_uint64 * 4)()
    L.amgd_test_part_stats(ps)
    out["lmop_gathered"], out["lmop_prefix"], out["eager_calls"], out["eager_second"] = (int(v) for v in ps)
    rs = oa.route_stats()
    out["routes"] = {k: v for k, v in rs.items() if v}
    out["leak_bytes"] = int(L.amgd_test_pool_inuse()) - int(before)
    if ref is not None:
        bad = parity.compare(ref, h, exact=True)
    else:
        import make_digests as md
        got = md.hierarchy_digest(h)
        exp = digest["arrays"]
        bad = sorted(k for k in set(got) | set(exp) if got.get(k) != exp.get(k))
        if bad:
            # every differing array with its first differing row / entry against the one-GPU
            # setup of the whole matrix (amg_setup takes the whole matrix and makes no
            # exchange under any communicator; the one-GPU hierarchy is the digest's)
            h1 = abi.run_setup(oa.lib(), Ai64, Aj64, Av)
            ok1 = md.hierarchy_digest(h1) == exp
            out["one_gpu_matches_digest"] = ok1
            out["first_diff"] = parity.first_diff(h1, h)
    out.update(calls=st["calls"], bytes=st["bytes"], bad=bad, levels=h.nlevels)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if not bad and st["calls"] > 0 and out["leak_bytes"] == 0 else 1)


if __name__ == "__main__":
    main()
