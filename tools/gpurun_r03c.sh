# r03 session c: A/B of the tiled windowed SpGEMM at 256^3 (bit-identical hierarchies,
# times), SpGEMM call log + phase table, then a kernel profile of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03c
export PYTHONPATH=$PWD
timeout -k 10 500 python3 tools/ab_setup.py 256 wt=0 wt=4 wt=8 wt=4,win=1024 > gpurun_out/r03c/ab_wt256.txt 2>&1 || { cat gpurun_out/r03c/ab_wt256.txt | tail -20; exit 1; }
cat gpurun_out/r03c/ab_wt256.txt
AMGD_SGLOG=1 AMGD_PHASES=1 timeout -k 10 300 python3 tools/probe_scale.py 256 > gpurun_out/r03c/sglog256.txt 2>&1 || exit 1
tail -n 30 gpurun_out/r03c/sglog256.txt
