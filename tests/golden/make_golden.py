#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE ITSELF (run here, not on the GPU box).

For every candidate matrix:
  1. run the reference compiled with AddressSanitizer (oracle/_ref/ref_asan_drv)
     and RECORD whether it is clean -- the reference reads/writes past the end
     of St in sp_add (amg_setup.c:1674) on most Poisson inputs; the in-bounds
     values are unaffected, so such cases are kept when the plain build survives;
  2. run our CPU restatement (oracle/build/liboracle.so) and drop the case if the
     reference would not terminate (oracle_ub_count > 0);
  3. run the reference (oracle/_ref/libref_amg.so) through ctypes and store its
     full hierarchy (inputs + every per-level array) as the fixture;
  4. require the oracle to match it bit for bit.

The fixtures are data (inputs and the reference's outputs), small enough to
commit.  Usage:  python tests/golden/make_golden.py  (after `make -C oracle all ref`)
"""
from __future__ import annotations

import ctypes as C
import json
import multiprocessing as mp
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from omp_amg_amd import abi, parity, problems  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_amg.so")
ASAN = os.path.join(ROOT, "oracle", "_ref", "ref_asan_drv")
ORA_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")


def candidates():
    c = {"amgdmp": lambda: problems.load_amgdmp(os.path.join(GOLD))}
    for m in (4, 7, 9, 10, 11, 12, 13, 14):
        c[f"p7_{m}"] = (lambda m=m: problems.poisson3d(m))
    for (mx, my, mz) in ((12, 10, 8), (16, 6, 5)):
        c[f"p7_{mx}x{my}x{mz}"] = (lambda a=mx, b=my, z=mz: problems.poisson3d(z, mx=a, my=b))
    for m in (6, 8, 10, 12):
        c[f"aniso_{m}"] = (lambda m=m: problems.poisson3d(m, eps=1e-3))
    for m in (4, 5, 6, 7, 8):
        c[f"p27_{m}"] = (lambda m=m: problems.poisson3d(m, 27))
    for m in (8, 12, 16, 20, 24, 32, 40):
        c[f"p2d5_{m}"] = (lambda m=m: problems.poisson2d(m))
    for m in (8, 12, 16, 24):
        c[f"p2d9_{m}"] = (lambda m=m: problems.poisson2d(m, 9))
    # configs[2] is order N = 7: e2 N7 (13^3 = 2197 rows), e3 N7 (20^3 = 8000 rows)
    for (e, N) in ((2, 3), (2, 4), (3, 2), (3, 3), (2, 5), (2, 6), (2, 7), (3, 7)):
        c[f"sem_e{e}_N{N}"] = (lambda e=e, N=N: problems.sem_laplacian(e, e, e, N, seed=1, jitter=0.3))
    return c


def _run(q, so, Ai, Aj, Av, want_ub):
    try:
        lib = abi.bind_setup(C.CDLL(so))
        h = abi.run_setup(lib, Ai, Aj, Av)
        ub = (int(C.CDLL(so).oracle_ub_count()), int(C.CDLL(so).oracle_overflow_count())) if want_ub else (0, 0)
        q.put(("ok", parity.to_npz_dict(h), ub))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e), (0, 0)))


def run_isolated(so, Ai, Aj, Av, timeout=int(os.environ.get("GOLDEN_TIMEOUT", "120")), want_ub=False):
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_run, args=(q, so, Ai, Aj, Av, want_ub))
    p.start()
    import queue
    try:
        st, d, ub = q.get(timeout=timeout)      # drain before join (pipe back-pressure)
    except queue.Empty:
        p.kill()
        p.join()
        return None, "timeout" if p.exitcode is None or p.exitcode < 0 else f"exit {p.exitcode}", (0, 0)
    p.join()
    return (d if st == "ok" else None), st, ub


def asan_clean(Ai, Aj, Av, timeout=180):
    with tempfile.NamedTemporaryFile(suffix=".coo", delete=False) as f:
        nz = np.array([len(Av)], dtype=np.uint64)
        f.write(nz.tobytes())
        f.write(np.asarray(Ai, dtype=np.uint64).tobytes())
        f.write(np.asarray(Aj, dtype=np.uint64).tobytes())
        f.write(np.asarray(Av, dtype=np.float64).tobytes())
        path = f.name
    try:
        r = subprocess.run([ASAN, path], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           timeout=timeout, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
        return r.returncode == 0, (r.stderr.decode(errors="replace").splitlines() or [""])[0][:200]
    except subprocess.TimeoutExpired:
        return False, "timeout (reference does not terminate)"
    finally:
        os.unlink(path)


def main():
    only = set(sys.argv[1:])
    manifest = {"kept": {}, "excluded": {}}
    mpath = os.path.join(GOLD, "MANIFEST.json")
    if only and os.path.exists(mpath):       # partial run: update the existing manifest
        manifest = json.load(open(mpath))
        for k in ("kept", "excluded"):
            for name in only:
                manifest[k].pop(name, None)
    for name, gen in candidates().items():
        if only and name not in only:
            continue
        Ai, Aj, Av = gen()
        asan_ok, why = asan_clean(Ai, Aj, Av)
        od, st, (ub, ovf) = run_isolated(ORA_SO, Ai, Aj, Av, want_ub=True)
        if od is None or ub:
            manifest["excluded"][name] = f"oracle {st}: reference does not terminate (stall events={ub})"
            print(f"{name:14s} EXCLUDED (oracle {st}, stall={ub})", flush=True)
            continue
        rd, st, _ = run_isolated(REF_SO, Ai, Aj, Av)
        if rd is None:
            manifest["excluded"][name] = f"reference {st}"
            print(f"{name:14s} EXCLUDED (reference {st})", flush=True)
            continue
        bad = parity.compare(parity.from_npz(rd), parity.from_npz(od), exact=True)
        if bad:
            manifest["excluded"][name] = "ORACLE MISMATCH: " + "; ".join(bad[:4])
            print(f"{name:14s} ORACLE MISMATCH {bad[:4]}", flush=True)
            continue
        out = dict(rd)
        out["in_Ai"] = np.asarray(Ai, dtype=np.uint32)
        out["in_Aj"] = np.asarray(Aj, dtype=np.uint32)
        out["in_Av"] = np.asarray(Av, dtype=np.float64)
        np.savez_compressed(os.path.join(GOLD, f"{name}.npz"), **out)
        nl = int(rd["nlevels"])
        manifest["kept"][name] = {"rows": int(rd["L0_n"]), "nnz": int(rd["L0_nnz"]), "levels": nl,
                                  "reference_asan_clean": asan_ok, "asan": why if not asan_ok else "",
                                  "sp_add_end_overflows": ovf}
        print(f"{name:14s} kept  rows={int(rd['L0_n'])} levels={nl}", flush=True)
    if True:
        with open(mpath, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
