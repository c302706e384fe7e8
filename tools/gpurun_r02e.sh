# SpMV kernel tests, parity subset, then 256^3 timing + per-shape SpMV log with the RW lane kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${TAG:-r02e}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "spmv or bitexact" > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_$TAG.log; grep -E "FAILED|Error" gpurun_out/gputests_$TAG.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/p256_$TAG.out 2> gpurun_out/p256_$TAG.err; rc=$?; cat gpurun_out/p256_$TAG.out; [ $rc -eq 0 ] || exit $rc
AMGD_MVLOG=1 timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/mv_rw2.out 2> gpurun_out/mv_rw2.err; echo "mvlog rc=$?"
