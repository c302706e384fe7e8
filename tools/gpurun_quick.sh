# one GPU call: the GPU suite (optionally a -k filter) + a short bench line on the same tree
# usage: bash tools/gpurun_quick.sh <tag>   (KSEL=... pytest -k filter; NOBENCH=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r04}
D=$GRAFT_REPO_ROOT/gpurun_out/$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 ${TLIM:-900} python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 150 --timeout-method thread ${KSEL:+-k "$KSEL"} > $D/gputests.log 2>&1 || { tail -40 $D/gputests.log; exit 1; }
tail -3 $D/gputests.log
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python3 bench.py --gpus 1 --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo bench failed; tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
