# GPU tests selected by -k "$KSEL" (kernels + parity files), then a 256^3 timing probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${TAG:-kt}
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "$KSEL" > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_$TAG.log; grep -E "FAILED|Error" gpurun_out/gputests_$TAG.log | head; [ $rc -eq 0 ] || exit $rc
${PROBE_ENV:+env $PROBE_ENV} timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/p256_$TAG.out 2> gpurun_out/p256_$TAG.err; rc=$?; cat gpurun_out/p256_$TAG.out; exit $rc
