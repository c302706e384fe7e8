"""debug: one setup of a small problem with the incremental find_support sweeps"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import omp_amg_amd as oa
from omp_amg_amd import abi, problems, parity
m = int(sys.argv[1]) if len(sys.argv) > 1 else 32
Ai, Aj, Av = problems.poisson3d(m, eps=float(sys.argv[2])) if len(sys.argv) > 2 else problems.poisson3d(m)
t = time.time()
os.environ["AMGD_FS_INC"] = "0"
h0 = abi.run_setup(oa.lib(), Ai, Aj, Av)
print("full", time.time() - t, flush=True)
os.environ["AMGD_FS_INC"] = "1"
t = time.time()
h1 = abi.run_setup(oa.lib(), Ai, Aj, Av)
print("inc", time.time() - t, flush=True)
print(parity.compare(h0, h1, exact=True)[:5])
