# one GPU call: full parity suite, the driver's bench command and a rocprofv3 kernel
# summary of a short bench run, all on the same tree (PMC traffic: tools/gpurun_pmc.sh).
# usage: bash tools/gpurun_round.sh <tag>    (SKIP_TESTS=1: bench + profile only)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r04}
D=$GRAFT_REPO_ROOT/gpurun_out/$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1140 python3 -u -m pytest tests -m gpu -x -q --durations=15 --timeout 300 --timeout-method thread > $D/gputests.log 2>&1 || { tail -30 $D/gputests.log; exit 1; }
tail -2 $D/gputests.log
fi
[ -n "$TESTS_ONLY" ] && exit 0
t0=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err || { echo bench failed; tail -20 $D/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
cat $D/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $D/prof_line.json 2>&1 || exit 1
find $D -name "*kernel_trace.csv" -delete
tail -n 1 $D/prof_line.json
