#!/usr/bin/env python3
"""Benchmark: AMG setup throughput of the MI355X-native setup path.

metric  : "AMG setup rows/sec + RAP SpGEMM nnz/sec at 1/2/4/8 MI355X" (BASELINE.json)
workload: BASELINE.json configs[1] -- 3D 7-point Poisson 256^3 CSR (16.7M rows,
          116M nnz) on one MI355X.  One "step" = one full AMG setup (build_csr,
          coarsening, Chebyshev/Lanczos smoother, energy-minimising interpolation,
          Galerkin RAP for every level) from a device-resident COO matrix to a
          hierarchy resident in HBM.  Inputs are uploaded before the timed region.
value   : whole-job rows/s of the setup.  N>1 (DESIGN.md "Multi-GPU"): one setup of
          the matrix row-PARTITIONED over the N GPUs (--mode part, default): each rank
          generates its own rows and holds only its row blocks of every matrix of the
          hierarchy; products fetch halo rows, transposes exchange row pieces, vectors
          are completed by allgatherv (RCCL send/recv over xGMI); value = rows /
          max-over-ranks seconds, scaling "strong".  --mode shard: the round-2
          replicated hierarchy with sharded kernels; --mode replicas: N independent
          setups (value = N x rows / max time, scaling "weak").
roofline: the dominant kernel by time, the long-row SpMV (k_spmv_pair<false,RW,PER,..>
          for products with x -- k_spmv_pair_amx<RW,PER> in find_support's full sweeps,
          which also tracks each row's first largest product for the fused selection --
          k_spmv_pipe<false,RW,PER,false> for ordered row sums;
          whole-matrix products: find_support's sweeps, PCG, Lanczos), event-timed
          live on the library stream; algorithmic bytes = 12 B per entry + 8 B per
          column (x read once) + 16 B per row; the rate with x gathered
          once per entry and the PMC-measured HBM rate are reported beside it.
rap_roofline: the Galerkin RAP SpGEMM numeric kernels (A_{l+1} = W'AfP + A_cf W + A_cc
          and AfP = Af W; instantiated with RAP=1 so rocprof lists them apart;
          k_sg_kseq for long B-operand rows, k_sg_row for short ones, k_sg_win
          for wide output rows), event-timed likewise; algorithmic bytes = 12 B per
          nnz of each operand and result + 8 B per row;
          tools/rap_from_prof.py sums the same kernels from a rocprofv3 summary.
cpu_baseline: the reference's own serial setup (oracle/_ref/libref_amg.so,
          compiled from /root/reference sources) on a bounded sample, rank 0 only.

Run: python bench.py [--gpus N --steps K --warmup W] [--m 256] [--stencil 7]
     N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--budget-s", type=float, default=450.0,
                   help="wall-time budget of the whole run (s): warmup and timed steps stop early "
                        "when one more step would pass it; `steps`/`warmup` report what ran")
    p.add_argument("--mode", choices=["part", "shard", "replicas"], default=None,
                   help="N>1 (default part): one row-partitioned setup (each rank holds its row "
                        "blocks of every matrix, halo exchange; strong scaling), the round-2 "
                        "replicated-hierarchy sharding, or N independent replicas.  N=1: the "
                        "one-GPU driver unless --mode part is given, which runs the partitioned "
                        "driver on a one-rank RCCL communicator (its N=1 baseline)")
    p.add_argument("--transport", choices=["rccl", "host"], default="rccl",
                   help="shard mode data path: RCCL over xGMI, or host-staged gloo (rehearsal "
                        "of N ranks on fewer GPUs; ranks share devices round-robin)")
    p.add_argument("--edge", "--m", dest="m", type=int, default=256,
                   help="grid edge (configs[1]: 256); spell it --edge under torch.distributed.run")
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--fast-dots", action="store_true",
                   help="tree-ordered global dots instead of reference order (not parity-certified)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-m", type=int, default=20,
                   help="reference CPU sample grid edge (20: a size the reference terminates on)")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--cpu-budget-s", type=float, default=45.0,
                   help="cap on the total time of the CPU baseline (all child runs)")
    p.add_argument("--cpu-child", nargs=2, type=int, default=None, help=argparse.SUPPRESS)
    p.add_argument("--traffic", type=float, default=None,
                   help="long-row SpMV L2->fabric bytes per setup from rocprofv3 PMC passes (profiles/)")
    p.add_argument("--rap-traffic", type=float, default=None,
                   help="RAP SpGEMM L2->fabric bytes per setup from rocprofv3 PMC passes (profiles/)")
    return p.parse_args()


def cpu_child(m, reps):
    """(child process) time the reference serial setup; prints one JSON line"""
    from omp_amg_amd import abi, problems
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_amg.so")
    kind = "reference"
    if not os.path.exists(ref):
        ref = os.path.join(ROOT, "oracle", "build", "liboracle.so")
        kind = "port"
    lib = abi.bind_setup(ctypes.CDLL(ref))
    Ai, Aj, Av = problems.poisson3d(m, 7)
    t0 = time.perf_counter()
    for _ in range(reps):
        h = abi.run_setup(lib, Ai, Aj, Av)
    dt = time.perf_counter() - t0
    print(json.dumps({"kind": kind, "secs": dt, "rows": m ** 3, "reps": reps, "levels": h.nlevels}))


def cpu_baseline(m, reps, budget_s):
    """The reference's own serial setup (oracle/_ref/libref_amg.so, compiled from
    /root/reference by oracle/Makefile) on a bounded sample, in a child process:
    the reference crashes or never terminates on many inputs (DESIGN.md
    "Reference UB"), so it must not be able to take the bench down with it.
    Falls back to the oracle (kind "port") where _ref is absent."""
    import subprocess
    if not (os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_amg.so"))
            or os.path.exists(os.path.join(ROOT, "oracle", "build", "liboracle.so"))):
        return None
    secs, done, fails, d = 0.0, 0, 0, None
    deadline = time.time() + budget_s
    for _ in range(3 * reps):          # each rep in its own process: the reference's heap
        left = deadline - time.time()  # overruns make it crash now and then on 7-point grids
        if done == reps or left < 5:
            break
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child", str(m), "1"],
                               capture_output=True, text=True, timeout=left)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            secs += d["secs"]
            done += 1
        except Exception:  # noqa: BLE001 -- crash / timeout of the reference
            fails += 1
    if done == 0:
        return {"value": None, "unit": "rows/s", "cores": 1, "kind": "reference",
                "sample": f"reference serial setup on 3D 7-point Poisson {m}^3: no run finished within "
                          f"{budget_s:.0f} s ({fails} crashed / timed out)"}
    d["reps"], d["secs"] = done, secs
    return {"value": d["rows"] * d["reps"] / d["secs"], "unit": "rows/s", "cores": 1, "kind": d["kind"],
            "sample": f"3D 7-point Poisson {m}^3 ({d['rows']} rows, {d['levels']} levels) x{d['reps']}, "
                      f"full serial amg_setup, {d['secs']:.2f} s on one host core ({fails} crashed runs discarded; the reference's mxm is "
                      f"O(rows^2) and it does not terminate on many larger grids, so 256^3 is out of its reach)"}


def gpu_sample(m, reps=5):
    """the GPU setup on the CPU baseline's own sample (7-point m^3), so the line holds a
    same-size ratio: rows/s over `reps` device-resident setups after one warm-up"""
    import omp_amg_amd as oa
    from omp_amg_amd import problems
    Ai, Aj, Av = problems.poisson3d(m, 7)
    ds = oa.DeviceSetup(Ai, Aj, Av)
    ds.run()
    t0 = time.perf_counter()
    for _ in range(reps):
        ds.run()
    dt = time.perf_counter() - t0
    ds.close()
    return {"value": m ** 3 * reps / dt, "unit": "rows/s", "secs_per_setup": dt / reps,
            "sample": f"3D 7-point Poisson {m}^3, {reps} device-resident setups on 1 MI355X"}


def pmc_traffic(m, stencil, world):
    """L2->fabric bytes (FETCH_SIZE / WRITE_SIZE: an upper bound on HBM bytes, MALL hits
    included) per setup of the two roofline kernels from the committed rocprofv3
    PMC passes (FETCH_SIZE / WRITE_SIZE, one counter per pass, gfx950 correction;
    tools/gpurun_round.sh), only when they were measured on this same workload (grid,
    stencil, one GPU): (spmv, rap, source) or Nones"""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic_r*.json")))
    for f in reversed(files):
        d = json.load(open(f))
        w = d.get("workload", {"m": 256, "stencil": 7, "world": 1})   # r02 files: 256^3 7-point, 1 GPU
        if (w["m"], w["stencil"], w["world"]) == (m, stencil, world):
            return d["spmv"], d["rap"], os.path.relpath(f, ROOT)
    return None, None, None


def heartbeat(period=30.0):
    """progress line on stderr while a long setup runs (keeps batch runners from
    taking a silent multi-minute setup for a hang)"""
    import threading
    t0 = time.time()
    stop = threading.Event()

    def run():
        while not stop.wait(period):
            print(f"[bench] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()
    return stop


def main():
    args = parse()
    if args.steps < 1:
        sys.exit("bench.py: --steps must be >= 1")
    if args.cpu_child:
        cpu_child(*args.cpu_child)
        return
    t_start = time.time()
    hb = heartbeat()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; for N>1 launch under "
                 f"python -m torch.distributed.run --nproc-per-node {args.gpus} ... bench.py --gpus {args.gpus}")
    dist = None
    device = local
    if world > 1:
        import torch
        import torch.distributed as dist
        if args.transport == "host":
            device = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        # control plane (barriers, the stop decision, max-over-ranks time) on gloo;
        # the data path is the library's own RCCL communicator on its stream
        dist.init_process_group("gloo")

    import omp_amg_amd as oa
    from omp_amg_amd import problems, shard

    oa.lib().amgd_init(device)
    part = args.mode == "part" or (world > 1 and args.mode is None)
    sharded = part or (world > 1 and args.mode == "shard")
    if sharded and args.transport == "host":
        shard.init_host(rank, world)
    elif sharded:
        shard.init_rccl(rank, world)
    rows = args.m ** 3
    if part:
        # every rank generates and uploads only its own rows
        oa.lib().amgd_comm_set_partitioned(1)
        Ai, Aj, Av = problems.poisson3d(args.m, args.stencil,
                                        rows_range=(rank * rows // world, (rank + 1) * rows // world))
    else:
        Ai, Aj, Av = problems.poisson3d(args.m, args.stencil)
    ds = oa.DeviceSetup(Ai, Aj, Av)
    del Ai, Aj, Av

    def barrier():
        if dist is not None:
            import torch
            oa.lib().amgd_dev_sync()
            torch.cuda.synchronize()
            dist.barrier()

    def agree(flag):
        """all ranks take the same continue/stop decision (max over ranks)"""
        if dist is None:
            return flag
        import torch
        t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return bool(t.item() > 0)

    # Wall-time budget: the CPU baseline's cap is reserved up front; a warmup or
    # timed step starts only if the estimate of one step still fits.  Warmup may
    # use at most a quarter of what is left, and at least one timed step always runs.
    reserve = 0.0 if (args.no_cpu_baseline or world > 1) else args.cpu_budget_s + 5.0
    deadline = t_start + args.budget_s - reserve
    t_step = 0.0
    warm = 0
    warm_deadline = time.time() + 0.25 * max(0.0, deadline - time.time())
    # the warmup setups run with the collective-consistency guard on (every collective's
    # kind, call site and sizes checked across the ranks first; a mismatch aborts with both
    # sites instead of hanging RCCL); the timed ones without its extra record exchange
    if world > 1:
        oa.lib().amgd_comm_set_check(1)
    while warm < args.warmup and (warm == 0 or not agree(time.time() + t_step > warm_deadline)):
        t1 = time.perf_counter()
        ds.run(exact_dots=not args.fast_dots)
        t_step = time.perf_counter() - t1
        warm += 1
    if world > 1:
        oa.lib().amgd_comm_set_check(0)
    barrier()
    rap_ms, rap_bytes, rap_nnz, mv_ms, mv_bytes, mv_strict, st = 0.0, 0, 0, 0.0, 0, 0, None
    mv_n, rap_n = 0, 0
    rw_ms, rw_b, rw_n = [0.0] * 3, [0] * 3, [0] * 3
    steps = 0
    if sharded:
        shard.stats(reset=True)
    t0 = time.perf_counter()
    while steps < args.steps:
        if steps > 0 and agree(time.time() + t_step > deadline):
            break
        t1 = time.perf_counter()
        st = ds.run(exact_dots=not args.fast_dots)
        t_step = time.perf_counter() - t1
        steps += 1
        rap_ms += st["rap_kernel_ms"]
        rap_bytes += st["rap_bytes"]
        rap_nnz += st["rap_out_nnz"]
        mv_ms += st["spmv_kernel_ms"]
        mv_bytes += st["spmv_bytes"]
        mv_strict += st["spmv_bytes_strict"]
        mv_n += st["spmv_launches"]
        rap_n += st["rap_launches"]
        for q in range(3):
            rw_ms[q] += st["spmv_rw_ms"][q]
            rw_b[q] += st["spmv_rw_bytes_strict"][q]
            rw_n[q] += st["spmv_rw_launches"][q]
        if rank == 0:
            print(f"[bench] step {steps}: {t_step:.2f} s", file=sys.stderr, flush=True)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt * 1e3 / steps
    copies = 1 if sharded else world
    value = copies * rows * steps / dt
    comm = shard.stats() if sharded else None

    if rank == 0:
        p_mv, p_rap, t_src = pmc_traffic(args.m, args.stencil, world)
        t_mv = p_mv["hbm_bytes"] if p_mv else None          # PMC bytes per setup
        t_rap = p_rap["hbm_bytes"] if p_rap else None
        if args.traffic is not None:
            t_mv, t_src, p_mv = args.traffic, "--traffic", None
        if args.rap_traffic is not None:
            t_rap, p_rap = args.rap_traffic, None
        # per launch (the PMC run's own dispatch counts; this run's launch counts otherwise)
        mv_lps = (p_mv or {}).get("dispatches") or (mv_n / steps if mv_n else None)
        rap_lps = (p_rap or {}).get("dispatches") or (rap_n / steps if rap_n else None)
        achieved = rap_bytes / (rap_ms * 1e-3) / 1e9 if rap_ms > 0 else 0.0
        mv_achieved = mv_strict / (mv_ms * 1e-3) / 1e9 if mv_ms > 0 else 0.0
        mv_gather = mv_bytes / (mv_ms * 1e-3) / 1e9 if mv_ms > 0 else 0.0
        mv_pmc = t_mv * steps / (mv_ms * 1e-3) / 1e9 if (mv_ms > 0 and t_mv) else None
        out = {
            "metric": "AMG setup rows/sec + RAP SpGEMM nnz/sec at 1/2/4/8 MI355X",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warm,
            "steps_requested": args.steps,
            "warmup_requested": args.warmup,
            "budget_s": args.budget_s,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"3D {args.stencil}-point Poisson {args.m}^3 CSR, full AMG setup"
                                   + (" (BASELINE configs[1])" if (args.m, args.stencil) == (256, 7) else ""),
                       "rows": rows, "nnz": int(st["nnz0"]), "levels": int(st["nlevels"]),
                       "parallelism": (f"rows partitioned x{world} (row blocks of every matrix per rank, "
                                       + ("halo rows before each product, RCCL over xGMI)" if args.transport == "rccl"
                                          else "halo rows before each product, host-staged gloo rehearsal)")
                                       if part else
                                       f"rows sharded x{world} (replicated hierarchy, RCCL allgatherv over xGMI)"
                                       if sharded and args.transport == "rccl" else
                                       f"rows sharded x{world} (host-staged gloo rehearsal)" if sharded
                                       else f"replicas x{world}"),
                       "global_dots": "tree" if args.fast_dots else "reference-order"},
            "rap_spgemm_nnz_per_s": copies * rap_nnz / (rap_ms * 1e-3) if rap_ms > 0 else None,
            "phases_ms": {k: round(st[k], 2) for k in ("t_build_ms", "t_coarsen_ms", "t_smoother_ms",
                                                          "t_interp_ms", "t_rap_ms")},
            "roofline": {"bound": "hbm", "achieved": mv_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": mv_achieved / HBM_PEAK_GBS,
                         "traffic": t_mv / mv_lps if (t_mv and mv_lps) else None,
                         "traffic_unit": "L2->fabric bytes per launch (PMC FETCH_SIZE + WRITE_SIZE, calibrated; "
                                         "MALL hits included, so an upper bound on HBM bytes; "
                                         "traffic_per_setup / launches_per_setup)",
                         "traffic_per_setup": t_mv,
                         "traffic_source": t_src,
                         "launches_per_setup": mv_n / steps,
                         "algorithmic_bytes_per_launch": mv_strict / mv_n if mv_n else None,
                         "kernel": "k_spmv_pair<false,RW,PER,..> (products with x; k_spmv_pair_amx in find_support's "
                                   "full sweeps, + the fused selection's row maxima) / "
                                   "k_spmv_pipe<false,RW,PER,false> (row sums): whole-matrix "
                                   "long-row SpMV (ordered row sums; "
                                   "find_support sweeps, PCG, Lanczos), the setup's dominant kernel by time, "
                                   "HIP-event timed",
                         "algorithmic_bytes_per_setup": mv_strict / steps,
                         "algorithmic_bytes_def": "12 B per entry (u32 col + f64 a) + 8 B per column (x once) "
                                                  "+ 16 B per row (row offsets, z)",
                         "kernel_ms_per_setup": mv_ms / steps,
                         "by_shape": {f"RW{rw}": {"ms_per_setup": rw_ms[q] / steps,
                                                  "launches_per_setup": rw_n[q] / steps,
                                                  "algorithmic_bytes_per_setup": rw_b[q] / steps,
                                                  "achieved_gbs": (rw_b[q] / (rw_ms[q] * 1e-3) / 1e9
                                                                   if rw_ms[q] > 0 else None)}
                                      for q, rw in enumerate((4, 16, 64))},
                         "pmc_rate_gbs": mv_pmc,
                         "pmc_frac": mv_pmc / HBM_PEAK_GBS if mv_pmc else None,
                         "pmc_over_algorithmic": t_mv * steps / mv_strict if (t_mv and mv_strict) else None,
                         "extra_per_entry_gather": {"bytes_per_setup": mv_bytes / steps, "achieved": mv_gather,
                                                    "note": "x gathered once per entry (8 B/entry): an upper "
                                                            "bound on gather traffic, not the roofline"}},
            "rap_roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": t_rap / rap_lps if (t_rap and rap_lps) else None,
                         "traffic_unit": "L2->fabric bytes per launch (PMC FETCH_SIZE + WRITE_SIZE, calibrated; MALL hits "
                                         "included: an upper bound on HBM bytes; traffic_per_setup / launches)",
                         "traffic_per_setup": t_rap,
                         "traffic_source": t_src,
                         "traffic_over_algorithmic": t_rap * steps / rap_bytes if (t_rap and rap_bytes) else None,
                         "launches_per_setup": rap_n / steps,
                         "kernel": "k_sg_kseq<NT,LG,1,1> + k_sg_row<NT,LG,1,1> + k_sg_wwin<W,1,1> + k_sg_win<W,1> + k_spgemm_long<1,1>: numeric "
                                   "passes of the RAP SpGEMMs (Af*W, W'*AfP, Acf*W; the first and last via their "
                                   "exact transposed products where those run faster) of every level, HIP-event timed",
                         "algorithmic_bytes_per_setup": rap_bytes / steps,
                         "kernel_ms_per_setup": rap_ms / steps},
        }
        if part:
            out["peak_hbm_bytes_rank0"] = int(st["peak_bytes"])
        if comm is not None:
            out["comm_rank0_per_step"] = {"allgatherv_calls": comm["calls"] / steps,
                                          "bytes": comm["bytes"] / steps, "ms": comm["ms"] / steps}
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_m, args.cpu_reps, args.cpu_budget_s)
            if out["cpu_baseline"] is not None:
                out["cpu_baseline"]["gpu_same_sample"] = gpu_sample(args.cpu_m)
        print(json.dumps(out), flush=True)
    ds.close()
    if sharded:
        shard.free()
    # (no amgd_shutdown here: the process exits and the driver reclaims everything;
    # tearing the HIP stream down before exit crashes rocprofv3's own finalisation)
    hb.set()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
