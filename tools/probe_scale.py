"""Scaling probe: time the device setup on growing 3D Poisson grids, exact and
fast dots, with per-phase breakdown.  Usage: python tools/probe_scale.py 32 64 96"""
import json
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import omp_amg_amd as oa
from omp_amg_amd import problems

import threading
_t0 = time.time()


def _beat():
    while True:
        time.sleep(30)
        print(f"[probe] {time.time() - _t0:.0f} s", file=sys.stderr, flush=True)


threading.Thread(target=_beat, daemon=True).start()
modes = [True]
if "--fast-only" in sys.argv:
    modes = [False]
if "--both" in sys.argv:
    modes = [True, False]
sizes = [int(a) for a in sys.argv[1:] if a.isdigit()]
stencil = 27 if "--27" in sys.argv else 7
for m in sizes:
    t0 = time.time()
    Ai, Aj, Av = problems.poisson3d(m, stencil)
    ds = oa.DeviceSetup(Ai, Aj, Av)
    gen = time.time() - t0
    for exact in modes:
        st = ds.run(exact_dots=exact)
        keep = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in st.items()}
        print(json.dumps({"m": m, "rows": m ** 3, "exact": exact, "gen_s": round(gen, 1), **keep}), flush=True)
    ds.close()
# no amgd_shutdown at exit: tearing the HIP stream down first crashes rocprofv3's finalisation

