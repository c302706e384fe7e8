"""One rank of the multi-process sharded-setup test (tests/test_gpu_shard.py).

Launched N times on the same GPU with RANK / WORLD_SIZE / MASTER_PORT set: gloo
group, host-staged allgatherv transport (RCCL refuses two ranks on one device),
every op sharded (min work 0).  Checks the hierarchy bit for bit against the
reference fixture and, for a generated problem, against the one-GPU run of the
same process.  Prints one JSON line; exit code 0 = pass."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import omp_amg_amd as oa  # noqa: E402
from omp_amg_amd import abi, parity, problems, shard  # noqa: E402


def main():
    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=size)
    oa.init(0)
    case = os.environ["SHARD_CASE"]
    out = {"rank": rank, "case": case}
    if case.startswith("gold:"):
        z = np.load(os.path.join(os.path.dirname(__file__), "golden", case[5:] + ".npz"))
        ref = parity.from_npz(z)
        Ai, Aj, Av = z["in_Ai"], z["in_Aj"], z["in_Av"]
    else:
        m = int(case.split(":")[1])
        Ai, Aj, Av = problems.poisson3d(m, 27 if case.startswith("p27") else 7)
        ref = abi.run_setup(oa.lib(), Ai, Aj, Av)            # one GPU, before sharding
    shard.init_host(rank, size)
    oa.lib().amgd_comm_set_partitioned(0)      # the round-2 replicated mode (crs_setup's default is partitioned)
    shard.set_min_work(0.0)
    shard.stats(reset=True)
    if os.environ.get("SHARD_CRS"):
        # crs_setup (crs.h) with comm = {rank, size}: this rank passes its block of
        # rows as a local matrix (local dof k = global id ids[k]), the library gathers
        # the assembled matrix over its communicator and keeps the hierarchy
        Ai64, Aj64 = np.asarray(Ai, np.int64), np.asarray(Aj, np.int64)
        n = int(max(Ai64.max(), Aj64.max())) + 1
        lo, hi = rank * n // size, (rank + 1) * n // size
        sel = (Ai64 >= lo) & (Ai64 < hi)
        ids = np.arange(1, n + 1, dtype=np.uint64)     # every rank knows every global id
        hd = abi.crs_setup(oa.lib(), n, ids, Ai64[sel], Aj64[sel], np.asarray(Av)[sel],
                           rank=rank, np_=size)
        assert hd is not None, "crs_setup returned NULL"
        h = abi.crs_export(oa.lib(), hd)
        oa.lib().crs_free(hd)
    else:
        h = abi.run_setup(oa.lib(), Ai, Aj, Av)
    st = shard.stats()
    shard.free()
    bad = parity.compare(ref, h, exact=True)
    out.update(calls=st["calls"], bytes=st["bytes"], bad=bad[:5], levels=h.nlevels)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if not bad and st["calls"] > 0 else 1)


if __name__ == "__main__":
    main()
