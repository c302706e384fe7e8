#!/usr/bin/env python3
"""Which default kernel routes a 7-point box takes (omp_amg_amd.route_stats), with the
setup time and level sizes: finds the smallest grid on which a given route (mv_rw64,
qf_t512, qf_t1024, ...) fires with no forcing switch.

usage: python tools/route_probe.py MXxMYxMZ [...]      e.g. 256x256x128 192x192x192
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import omp_amg_amd as oa  # noqa: E402
from omp_amg_amd import problems  # noqa: E402


def main():
    for box in sys.argv[1:]:
        mx, my, mz = (int(v) for v in box.lower().split("x"))
        Ai, Aj, Av = problems.poisson3d(mz, 7, mx=mx, my=my)
        ds = oa.DeviceSetup(Ai, Aj, Av)
        del Ai, Aj, Av
        oa.route_stats(reset=True)
        t0 = time.perf_counter()
        st = ds.run()
        dt = time.perf_counter() - t0
        r = oa.route_stats(reset=True)
        ds.close()
        print(json.dumps({"box": box, "rows": mx * my * mz, "secs": round(dt, 2),
                          "levels": st["nlevels"], "peak_gb": round(st["peak_bytes"] / 2**30, 2),
                          "routes": r}), flush=True)


if __name__ == "__main__":
    main()
