# r03 session c: SpGEMM call log + phase table of one 256^3 setup, then a kernel profile
# of the bench (baseline of this round's kernel work)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03c
export PYTHONPATH=$PWD
AMGD_SGLOG=1 AMGD_PHASES=1 timeout -k 10 300 python3 tools/probe_scale.py 256 > gpurun_out/r03c/sglog256.txt 2>&1 || exit 1
tail -n 30 gpurun_out/r03c/sglog256.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03c/prof -o bench --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r03c/prof_line.json 2>&1 || exit 1
rm -f $GRAFT_REPO_ROOT/gpurun_out/r03c/prof/*kernel_trace.csv
tail -n 2 $GRAFT_REPO_ROOT/gpurun_out/r03c/prof_line.json
