# rocprofv3 --kernel-trace --stats of one bench setup (after one warm-up) on this tree
# usage: bash tools/gpurun_prof.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/prof_$1
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $D/prof_line.json 2>&1 || exit 1
find $D -name "*kernel_trace.csv" -delete
tail -n 1 $D/prof_line.json | cut -c1-300
