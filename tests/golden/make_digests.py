#!/usr/bin/env python3
"""Digest fixtures for parity at sizes where the library's DEFAULT kernel routing
engages (run here, on the CPU; not on the GPU box).

A full .npz of a 10^5-row hierarchy is tens of MB, so these fixtures keep, per
case, the generator call that makes the input, a SHA-256 of that input, and a
SHA-256 of every array of the expected hierarchy (`parity.to_npz_dict` layout:
level sizes, C/F masks, ids, every CSR row_off / col / a, D, m, rho).  Equal
digests mean bit-identical hierarchies; a mismatch names the level and field.

Sources (field "source"):
  * "reference" -- the reference itself (oracle/_ref/libref_amg.so, compiled from
    /root/reference); its mxm is O(rows^2), so only up to ~10^4 rows;
  * "oracle"    -- the CPU restatement (oracle/build/liboracle.so), which
    tests/test_oracle_golden.py pins bit for bit to the reference's own outputs
    on every .npz fixture; it reaches 10^5 rows in minutes.

A case whose oracle run reports a reference-undefined event (the reference's loop
would never terminate) is recorded under "excluded" with the reason.

usage: python tests/golden/make_digests.py [case ...]   (after `make -C oracle all ref`)
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from omp_amg_amd import abi, parity, problems  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
OUT = os.path.join(GOLD, "digests.json")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_amg.so")
ORA_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")

# name -> (source, generator kwargs).  Sizes chosen so the default routing of
# amgd_setup.c engages with no forcing switch: incremental coarsening (>= 65536
# rows), incremental find_support (>= 4096 F rows), lane SpMV (>= 4096 rows of
# mean >= 32), windowed SpGEMM (>= 2048 distinct output columns), SEM order 7.
CASES = {
    "p7_48": ("oracle", {"kind": "poisson3d", "m": 48}),
    "p7_64": ("oracle", {"kind": "poisson3d", "m": 64}),
    "p7_96": ("oracle", {"kind": "poisson3d", "m": 96}),
    "p7_128": ("oracle", {"kind": "poisson3d", "m": 128}),
    # (the smallest box on which the 64-rows-per-wavefront long-row SpMV runs by default,
    # 7-point 256 x 256 x 192 -- tools/route_probe.py, profiles/r05/route_probe_r05g.jsonl --
    # is out of the oracle's reach here: past 54 GB of host memory after 2 h, stopped at the
    # container's 64 GB; that kernel shape is pinned by test_gpu_matches_digest_rw64_forced)
    "aniso_20": ("oracle", {"kind": "poisson3d", "m": 20, "eps": 1e-3}),
    "aniso_24": ("oracle", {"kind": "poisson3d", "m": 24, "eps": 1e-3}),
    "aniso_32": ("oracle", {"kind": "poisson3d", "m": 32, "eps": 1e-3}),
    "aniso_40": ("oracle", {"kind": "poisson3d", "m": 40, "eps": 1e-3}),
    "aniso_48": ("oracle", {"kind": "poisson3d", "m": 48, "eps": 1e-3}),
    "p27_20": ("oracle", {"kind": "poisson3d", "m": 20, "stencil": 27}),
    "p27_24": ("oracle", {"kind": "poisson3d", "m": 24, "stencil": 27}),
    "p27_28": ("oracle", {"kind": "poisson3d", "m": 28, "stencil": 27}),
    "p27_32": ("oracle", {"kind": "poisson3d", "m": 32, "stencil": 27}),
    "sem_e3_N7": ("reference", {"kind": "sem", "e": 3, "N": 7, "seed": 1, "jitter": 0.3}),
    "sem_e4_N7": ("oracle", {"kind": "sem", "e": 4, "N": 7, "seed": 1, "jitter": 0.3}),
    "sem_e5_N7": ("oracle", {"kind": "sem", "e": 5, "N": 7, "seed": 3, "jitter": 0.3}),
}


def generate(g: dict):
    if g["kind"] == "poisson3d":
        return problems.poisson3d(g["m"], g.get("stencil", 7), eps=g.get("eps", 1.0), mx=g.get("mx"),
                                  my=g.get("my"))
    if g["kind"] == "sem":
        e = g["e"]
        return problems.sem_laplacian(e, e, e, g["N"], seed=g["seed"], jitter=g["jitter"])
    raise ValueError(g)


def input_digest(Ai, Aj, Av) -> str:
    h = hashlib.sha256()
    for a, dt in ((Ai, np.uint32), (Aj, np.uint32), (Av, np.float64)):
        h.update(np.ascontiguousarray(a, dtype=dt).tobytes())
    return h.hexdigest()


def hierarchy_digest(h: abi.Hierarchy) -> dict:
    """key -> sha256 of that array's bytes (dtypes fixed by parity.to_npz_dict)"""
    out = {}
    for k, v in sorted(parity.to_npz_dict(h).items()):
        a = np.ascontiguousarray(np.asarray(v))
        out[k] = hashlib.sha256(a.dtype.str.encode() + a.tobytes()).hexdigest()[:32]
    return out


def summary(h: abi.Hierarchy) -> dict:
    return {"levels": h.nlevels, "n": [int(l.n) for l in h.levels],
            "nnz": [int(l.nnz) for l in h.levels],
            "W_nnz": [int(l.W.nnz) for l in h.levels[:-1]]}


def _run(q, so, gen, want_ub):
    try:
        lib = abi.bind_setup(C.CDLL(so))
        Ai, Aj, Av = generate(gen)
        t0 = time.time()
        h = abi.run_setup(lib, Ai, Aj, Av)
        secs = time.time() - t0
        ub = int(C.CDLL(so).oracle_ub_count()) if want_ub else 0
        q.put(("ok", {"input_sha256": input_digest(Ai, Aj, Av), "arrays": hierarchy_digest(h),
                      "summary": summary(h), "secs": round(secs, 1)}, ub))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e), 0))


def run_case(name, timeout):
    src, gen = CASES[name]
    so = REF_SO if src == "reference" else ORA_SO
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_run, args=(q, so, gen, src == "oracle"))
    p.start()
    import queue
    try:
        st, d, ub = q.get(timeout=timeout)
    except queue.Empty:
        p.kill()
        p.join()
        return name, None, f"{src} timeout after {timeout} s"
    p.join()
    if st != "ok":
        return name, None, f"{src} error {d}"
    if ub:
        return name, None, f"oracle: reference does not terminate (undefined events={ub})"
    d["source"] = src
    d["gen"] = gen
    return name, d, None


def main():
    names = sys.argv[1:] or list(CASES)
    timeout = int(os.environ.get("DIGEST_TIMEOUT", "7200"))
    db = json.load(open(OUT)) if os.path.exists(OUT) else {"cases": {}, "excluded": {}}
    from concurrent.futures import ThreadPoolExecutor, as_completed
    with ThreadPoolExecutor(int(os.environ.get("DIGEST_JOBS", "4"))) as pool:
        futs = [pool.submit(run_case, n, timeout) for n in names]
        for fu in as_completed(futs):
            name, d, why = fu.result()
            db["cases"].pop(name, None)
            db["excluded"].pop(name, None)
            if d is None:
                db["excluded"][name] = why
                print(f"{name:12s} EXCLUDED: {why}", flush=True)
            else:
                db["cases"][name] = d
                print(f"{name:12s} ok {d['summary']['n']} ({d['secs']} s)", flush=True)
            with open(OUT, "w") as f:
                json.dump(db, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
