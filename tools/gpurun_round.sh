# one GPU session: parity tests, the bench line, a rocprof kernel summary of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${1:-r01}
timeout -k 10 900 python3 -m pytest tests -m gpu -q > gpurun_out/gputests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/gputests_$TAG.log
timeout -k 10 900 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
rm -rf gpurun_out/prof_$TAG; mkdir -p gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG/bench_line.json 2>&1; echo "prof rc=$?"
rm -f $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG/bench_kernel_trace.csv
exit $rc
