#!/usr/bin/env python3
"""Interpolation-loop trace of the CPU oracle (TEST INFRASTRUCTURE, run here) or of the
HIP library (--lib omp_amg_amd/libomp_amg_amd.so, on the GPU box) for one synthetic
problem, with a wall-clock stamp per line.

The oracle prints, per interpolation iteration, " <nnz(W_skel)> nzs, <n> cols > gamma,
worst = <sqrt(max r)>" (ORACLE_VERBOSE, oracle/amg_oracle.c, the reference's own
printout at amg_setup.c:803); the GPU library prints the same line under
AMGD_VERBOSE=1 (amgd_setup.c interpolation()).  tools/trace_diff.py compares the two.

usage: python tools/oracle_trace.py <stencil> <m> <out.txt> [--eps E] [--timeout S] [--lib SO]
       (--lib omp_amg_amd/libomp_amg_amd.so on the GPU box: the same trace from the HIP path)
"""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(stencil, m, eps, lib):
    sys.path.insert(0, ROOT)
    import ctypes
    from omp_amg_amd import abi, problems
    Ai, Aj, Av = problems.poisson3d(m, stencil, eps=eps)
    L = abi.bind_setup(ctypes.CDLL(lib))
    t0 = time.time()
    h = abi.run_setup(L, Ai, Aj, Av, quiet=False)
    sys.stdout.flush()
    print(f"DONE levels={h.nlevels} sizes={[int(l.n) for l in h.levels]} secs={time.time() - t0:.1f}",
          flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("stencil", type=int)
    p.add_argument("m", type=int)
    p.add_argument("out")
    p.add_argument("--eps", type=float, default=1.0)
    p.add_argument("--timeout", type=float, default=4 * 3600)
    p.add_argument("--lib", default=os.path.join(ROOT, "oracle", "build", "liboracle.so"))
    p.add_argument("--child", action="store_true")
    a = p.parse_args()
    if a.child:
        child(a.stencil, a.m, a.eps, a.lib)
        return
    env = dict(os.environ, ORACLE_VERBOSE="1", AMGD_VERBOSE="1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, os.path.abspath(__file__), str(a.stencil), str(a.m), a.out,
           "--eps", str(a.eps), "--lib", a.lib, "--child"]
    t0 = time.time()
    import threading
    with open(a.out, "w") as f:
        f.write(f"# {os.path.basename(a.lib)} {a.stencil}-point m={a.m} eps={a.eps}\n")
        pr = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)

        def copy():
            for line in pr.stdout:
                f.write(f"[{time.time() - t0:9.1f}s] {line}")
                f.flush()
        th = threading.Thread(target=copy, daemon=True)
        th.start()
        try:
            pr.wait(timeout=a.timeout)
        except subprocess.TimeoutExpired:
            pr.kill()
            pr.wait()
            f.write(f"# TIMEOUT after {a.timeout:.0f} s (killed)\n")
        th.join(5)
        f.write(f"# exit {pr.returncode} after {time.time() - t0:.1f} s\n")

if __name__ == "__main__":
    main()
