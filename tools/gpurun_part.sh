# one GPU call: the partitioned tests first (no -x: every case reports), then the rest
# of the GPU suite (-x), then an optional short bench line
# usage: bash tools/gpurun_part.sh <tag>   (SKIP_SUITE=1, NOBENCH=1, PKSEL=<-k filter for the partition tests>)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r04}
D=$GRAFT_REPO_ROOT/gpurun_out/$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 ${PLIM:-700} python3 -u -m pytest tests/test_gpu_partition.py -m gpu -v --timeout 300 --timeout-method thread ${PKSEL:+-k "$PKSEL"} > $D/parttests.log 2>&1; prc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $D/parttests.log | tail -30
[ $prc -ne 0 ] && { grep -E "Error|error|assert|Abort|abort|fault" $D/parttests.log | head -40; }
[ $prc -gt 1 ] && exit $prc
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 ${TLIM:-900} python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread --deselect tests/test_gpu_partition.py > $D/gputests.log 2>&1 || { tail -40 $D/gputests.log; exit 1; }
tail -3 $D/gputests.log
fi
[ -n "$NOBENCH" ] && exit $prc
timeout -k 10 300 python3 bench.py --gpus 1 --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo bench failed; tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
exit $prc
