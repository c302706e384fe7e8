# r03 session d: one 256^3 setup with the SpGEMM call log + phase table (tree with the
# R-transpose reuse), the same setup's hierarchy digest vs the previous tree's, and a
# kernel profile of the bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03d
export PYTHONPATH=$PWD
timeout -k 10 200 python3 tools/ab_setup.py 256 default > gpurun_out/r03d/digest256.txt 2>&1 || { tail -5 gpurun_out/r03d/digest256.txt; exit 1; }
cat gpurun_out/r03d/digest256.txt
AMGD_SGLOG=1 AMGD_PHASES=1 timeout -k 10 300 python3 tools/probe_scale.py 256 > gpurun_out/r03d/sglog256.txt 2>&1 || exit 1
tail -n 16 gpurun_out/r03d/sglog256.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03d/prof -o bench --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r03d/prof_line.json 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r03d/prof -name "*kernel_trace.csv" -delete
tail -n 1 $GRAFT_REPO_ROOT/gpurun_out/r03d/prof_line.json
