#!/usr/bin/env python3
"""Per-rank HBM peak of the partitioned setup against the one-GPU setup,
on the test box's single GPU: the one-GPU setup first (its amgd_stats.peak_bytes), then N
processes over the host transport, each generating and passing only its own rows.  The
partitioned hierarchy is checked bit for bit against the one-GPU one (SHA-256 of every
array).  Prints / writes one JSON object.

usage: python tools/part_peak.py <m> <N> [out.json] [--stencil 7]"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def digest(h):
    from omp_amg_amd import parity
    import numpy as np
    out = hashlib.sha256()
    for k, v in sorted(parity.to_npz_dict(h).items()):
        a = np.ascontiguousarray(np.asarray(v))
        out.update(k.encode() + a.dtype.str.encode() + a.tobytes())
    return out.hexdigest()


def one_gpu(m, stencil, export=True):
    import omp_amg_amd as oa
    from omp_amg_amd import problems
    Ai, Aj, Av = problems.poisson3d(m, stencil)
    ds = oa.DeviceSetup(Ai, Aj, Av)
    t0 = time.time()
    st = ds.run()
    secs = time.time() - t0
    h = ds.export() if export else None
    print(json.dumps({"peak_bytes": int(st["peak_bytes"]), "secs": secs, "levels": int(st["nlevels"]),
                      "digest": digest(h) if h else None}), flush=True)


def rank_main(m, stencil, export=True):
    import torch.distributed as dist
    import omp_amg_amd as oa
    from omp_amg_amd import problems, shard
    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=size)
    oa.init(0)
    shard.init_host(rank, size)
    oa.lib().amgd_comm_set_partitioned(1)
    n = m ** 3
    Ai, Aj, Av = problems.poisson3d(m, stencil, rows_range=(rank * n // size, (rank + 1) * n // size))
    ds = oa.DeviceSetup(Ai, Aj, Av)
    shard.stats(reset=True)
    t0 = time.time()
    st = ds.run()
    secs = time.time() - t0
    cm = shard.stats()
    # (--no-export: the gathered hierarchy of a 256^3 setup is ~100 GB of host arrays per
    # process -- more than a box's host memory for three processes)
    h = ds.export() if export else None
    print(json.dumps({"rank": rank, "peak_bytes": int(st["peak_bytes"]), "secs": secs,
                      "comm_calls": cm["calls"], "comm_bytes": cm["bytes"], "comm_ms": cm["ms"],
                      "levels": int(st["nlevels"]), "digest": digest(h) if (h and rank == 0) else None}),
          flush=True)
    ds.close()
    shard.free()
    L = oa.lib()
    L.amgd_test_pool_inuse.restype = __import__("ctypes").c_uint64
    print(json.dumps({"rank": rank, "leak_bytes": int(L.amgd_test_pool_inuse())}), flush=True)
    dist.destroy_process_group()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("m", type=int)
    p.add_argument("N", type=int)
    p.add_argument("out", nargs="?")
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--role", default="driver")
    p.add_argument("--timeout", type=float, default=900)
    p.add_argument("--no-export", action="store_true",
                   help="peaks only: no gathered hierarchy / digest (sizes whose host copy is too big)")
    a = p.parse_args()
    if a.role == "one":
        return one_gpu(a.m, a.stencil, not a.no_export)
    if a.role == "rank":
        return rank_main(a.m, a.stencil, not a.no_export)
    env = dict(os.environ, PYTHONPATH=ROOT)
    xa = ["--no-export"] if a.no_export else []
    r = subprocess.run([sys.executable, "-u", __file__, str(a.m), "1", "--role", "one", "--stencil", str(a.stencil)] + xa,
                       capture_output=True, text=True, timeout=a.timeout, env=env)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    one = json.loads(r.stdout.strip().splitlines()[-1])
    one["phase_peaks"] = [l for l in r.stderr.splitlines() if l[:3].strip().isdigit() or l.startswith("lvl")
                          or "peak" in l][-24:]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # arena per process: a third of the GPU each is plenty below 128^3
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(a.N),
               AMGD_ARENA_GB=os.environ.get("AMGD_ARENA_GB", str(max(8, 200 // a.N))))
    ps = [subprocess.Popen([sys.executable, "-u", __file__, str(a.m), str(a.N), "--role", "rank",
                            "--stencil", str(a.stencil)] + xa, env=dict(env, RANK=str(r)),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(a.N)]
    t_start = time.time()
    while any(q.poll() is None for q in ps):           # heartbeat: long runs print progress
        time.sleep(30)
        print(f"[part_peak] {time.time() - t_start:.0f} s, {sum(q.poll() is None for q in ps)} ranks running",
              flush=True)
        if time.time() - t_start > a.timeout:
            break
    ranks = []
    for q in ps:
        o, e = q.communicate(timeout=a.timeout)
        if q.returncode:
            for x in ps:
                x.kill()
            sys.exit(f"rank failed rc={q.returncode}: {e[-3000:]}")
        d = {}
        for line in o.strip().splitlines():
            if line.startswith("{"):
                d.update(json.loads(line))
        d["phase_peaks"] = [l for l in e.splitlines() if l.startswith("rank")][-60:]
        ranks.append(d)
    peak = max(r["peak_bytes"] for r in ranks)
    res = {"workload": f"3D {a.stencil}-point Poisson {a.m}^3", "ranks": a.N, "one_gpu": one,
           "partitioned": ranks, "max_rank_peak_bytes": peak,
           "max_rank_peak_over_one_gpu": peak / one["peak_bytes"],
           "target_1p5_over_N": 1.5 / a.N,
           "bit_identical": (ranks[0]["digest"] == one["digest"]) if one["digest"] else "not checked (--no-export)",
           "max_rank_leak_bytes": max(r.get("leak_bytes", -1) for r in ranks),
           "transport": "host (gloo, N processes on one GPU)"}
    js = json.dumps(res, indent=1)
    print(js)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
