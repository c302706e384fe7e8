# r03 session f: phase table + SpGEMM / Q-factor call log of one 256^3 setup, then a
# 3-rep A/B of the Q-factor reuse and the pattern-only constraint product
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03f
export PYTHONPATH=$PWD
AMGD_SGLOG=1 AMGD_PHASES=1 timeout -k 10 300 python3 tools/probe_scale.py 256 > gpurun_out/r03f/sglog256.txt 2>&1 || exit 1
grep -A12 "phase ms" gpurun_out/r03f/sglog256.txt | tail -3
timeout -k 10 600 python3 tools/ab_setup.py 256 default qfr=0 pat=0 default --reps 3 --no-digest > gpurun_out/r03f/ab256.txt 2>&1 || { tail -5 gpurun_out/r03f/ab256.txt; exit 1; }
cat gpurun_out/r03f/ab256.txt
