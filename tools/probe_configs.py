"""Full-size runs of BASELINE.json's other single-GPU configs: one device setup each,
per-phase times from the library (AMGD_PHASES=1 adds the per-level table on stderr).

  python tools/probe_configs.py aniso256    # configs[4]: anisotropic 3D Poisson 256^3, eps = 1e-3
  python tools/probe_configs.py sem10k      # configs[2]: SEM Laplacian, 22x22x21 = 10164 hexes, N = 7
  python tools/probe_configs.py p27_128     # 27-point Poisson 128^3 (the configs[3] stencil, one GPU)
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import omp_amg_amd as oa  # noqa: E402
from omp_amg_amd import problems  # noqa: E402

_t0 = time.time()


def _beat():
    while True:
        time.sleep(30)
        print(f"[probe] {time.time() - _t0:.0f} s", file=sys.stderr, flush=True)


if os.environ.get("PROBE_BEAT", "1") != "0":      # off under rocprofv3 (a live thread at exit)
    threading.Thread(target=_beat, daemon=True).start()

CONFIGS = {
    "aniso256": ("anisotropic 3D 7-point Poisson 256^3, eps=1e-3 (BASELINE configs[4])",
                 lambda: problems.poisson3d(256, 7, eps=1e-3)),
    "aniso128": ("anisotropic 3D 7-point Poisson 128^3, eps=1e-3",
                 lambda: problems.poisson3d(128, 7, eps=1e-3)),
    "sem10k": ("SEM Laplacian, 22x22x21 = 10164 hexes, N=7 (BASELINE configs[2])",
               lambda: problems.sem_laplacian(22, 22, 21, 7)),
    "sem1k": ("SEM Laplacian, 10x10x10 hexes, N=7",
              lambda: problems.sem_laplacian(10, 10, 10, 7)),
    "p27_32": ("3D 27-point Poisson 32^3", lambda: problems.poisson3d(32, 27)),
    "p27_48": ("3D 27-point Poisson 48^3", lambda: problems.poisson3d(48, 27)),
    "p27_56": ("3D 27-point Poisson 56^3", lambda: problems.poisson3d(56, 27)),
    "p27_64": ("3D 27-point Poisson 64^3", lambda: problems.poisson3d(64, 27)),
    "p27_80": ("3D 27-point Poisson 80^3", lambda: problems.poisson3d(80, 27)),
    "p27_96": ("3D 27-point Poisson 96^3", lambda: problems.poisson3d(96, 27)),
    "p27_128": ("3D 27-point Poisson 128^3", lambda: problems.poisson3d(128, 27)),
    "p27_256": ("3D 27-point Poisson 256^3", lambda: problems.poisson3d(256, 27)),
    "p7_256": ("3D 7-point Poisson 256^3 (BASELINE configs[1])", lambda: problems.poisson3d(256, 7)),
}

reps = int(os.environ.get("PROBE_REPS", "1"))
for name in [a for a in sys.argv[1:] if a in CONFIGS]:
    desc, gen = CONFIGS[name]
    t0 = time.time()
    Ai, Aj, Av = gen()
    rows = int(Ai.max()) + 1
    ds = oa.DeviceSetup(Ai, Aj, Av)
    gen_s = time.time() - t0
    del Ai, Aj, Av
    for r in range(reps):
        t1 = time.perf_counter()
        try:
            st = ds.run()
        except RuntimeError as e:                  # out of HBM: recorded, the probe goes on
            print(json.dumps({"config": name, "workload": desc, "rows": rows, "error": str(e)}), flush=True)
            break
        dt = time.perf_counter() - t1
        keep = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in st.items()}
        print(json.dumps({"config": name, "workload": desc, "rows": rows, "rep": r, "setup_s": round(dt, 3),
                          "rows_per_s": rows / dt, "gen_s": round(gen_s, 1),
                          "rap_gbs": st["rap_bytes"] / max(st["rap_kernel_ms"], 1e-9) / 1e6, **keep}), flush=True)
    ds.close()
# no amgd_shutdown at exit (rocprofv3 finalisation, see bench.py)
