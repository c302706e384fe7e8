#!/usr/bin/env python3
"""A/B of kernel-choice settings on one device-resident problem (GPU box): for each
setting, one setup (after a warm-up of the first), its time, the RAP / SpMV kernel
times, and a SHA-256 digest of the exported hierarchy -- every setting must give the
same digest (bit-identical hierarchy).

usage: python tools/ab_setup.py <m> [--stencil 7] [--reps 1] SETTING...
SETTING: name=value for the omp_amg_amd test hooks, e.g. wt=0 wt=4 wt=8 win=1024
         (several hooks in one setting: wt=4,win=1024); "default" = no hook
"""
import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import omp_amg_amd as oa  # noqa: E402
from omp_amg_amd import parity, problems  # noqa: E402

HOOKS = {"win": oa.spgemm_win, "rw": oa.spmv_rw, "qfr": oa.qf_reuse, "pat": oa.sg_pattern,
         "lw": oa.lmop_wave, "lsm": oa.lmop_small, "pair": oa.spmv_pair, "rwb": oa.spmv_rw_bounds, "poll": oa.d2h_poll, "qat": oa.qa_tile, "slm": oa.spmv_sl_min, "amx": oa.fs_amx, "spat": oa.spat_inc, "drs": oa.spgemm_dr_sort, "dsp": oa.dot_split, "dsm": oa.dot_spec_min}


def digest(h):
    d = hashlib.sha256()
    for k, v in sorted(parity.to_npz_dict(h).items()):
        a = np.ascontiguousarray(np.asarray(v))
        d.update(k.encode() + a.dtype.str.encode() + a.tobytes())
    return d.hexdigest()[:24]


def apply(setting, reset=False):
    if setting == "default":
        return
    for kv in setting.split(","):
        k, v = kv.split("=")
        HOOKS[k](-1 if reset else int(v))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("m", type=int)
    p.add_argument("settings", nargs="+")
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--eps", type=float, default=1.0)
    p.add_argument("--reps", type=int, default=1)
    p.add_argument("--no-digest", action="store_true")
    a = p.parse_args()
    Ai, Aj, Av = problems.poisson3d(a.m, a.stencil, eps=a.eps)
    ds = oa.DeviceSetup(Ai, Aj, Av)
    del Ai, Aj, Av
    apply(a.settings[0])
    ds.run()                                     # warm-up (arena, code objects)
    apply(a.settings[0], reset=True)
    ref = None
    for s in a.settings:
        apply(s)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            st = ds.run()
            ts.append(time.perf_counter() - t0)
            print(f"# {s}: {ts[-1]:.3f} s", file=sys.stderr, flush=True)   # progress (a run
            # that prints nothing for minutes is taken for a hang)
        apply(s, reset=True)
        if not a.no_digest:
            print(f"# {s}: digest ...", file=sys.stderr, flush=True)
        dg = None if a.no_digest else digest(ds.export())
        ref = ref or dg
        print(json.dumps({"setting": s, "secs": [round(t, 3) for t in ts], "rap_kernel_ms": round(st["rap_kernel_ms"], 1),
                          "spmv_kernel_ms": round(st["spmv_kernel_ms"], 1), "levels": st["nlevels"],
                          "digest": dg, "same": dg == ref}), flush=True)
    ds.close()


if __name__ == "__main__":
    main()
