# GPU session: new SpMV tests + full gpu suite, then the driver's bench command under its 600 s limit
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${1:-r02a}
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/gputests_$TAG.log
[ $rc -eq 0 ] || exit $rc
t0=$(date +%s); timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
echo "bench wall=$(( $(date +%s) - t0 )) s"; cat gpurun_out/bench_$TAG.json; grep -E "step" gpurun_out/bench_$TAG.err
exit $rc
