# driver's bench command under its 600 s limit, then a find_support sweep log at 256^3
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${1:-r02b}
t0=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
echo "bench rc=$rc wall=$(( $(date +%s) - t0 )) s"
cat gpurun_out/bench_$TAG.json; grep -E "step" gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
AMGD_FSLOG=1 AMGD_PHASES=1 timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/fslog_$TAG.out 2> gpurun_out/fslog_$TAG.err
echo "probe rc=$?"
