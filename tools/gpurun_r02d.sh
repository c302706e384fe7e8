# full GPU suite, then 256^3 setup timing (default), with the lane-0 SpMV sums for A/B, and an MVLOG pass
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${TAG:-r02d}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_$TAG.log; grep -E "FAILED|Error" gpurun_out/gputests_$TAG.log | head; [ $rc -eq 0 ] || exit $rc
AMGD_PHASES=1 timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/p256_$TAG.out 2> gpurun_out/p256_$TAG.err; rc=$?; echo "bn rc=$rc"; cat gpurun_out/p256_$TAG.out; [ $rc -eq 0 ] || exit $rc
AMGD_SL_MIN_ROWS=1099511627776 timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/p256w_$TAG.out 2>&1; echo "bn wave-only rc=$?"; cat gpurun_out/p256w_$TAG.out | grep rows
AMGD_MVLOG=1 timeout -k 10 300 python3 tools/probe_scale.py 256 > gpurun_out/mvlog_$TAG.out 2> gpurun_out/mvlog_$TAG.err; echo "mvlog rc=$?"
