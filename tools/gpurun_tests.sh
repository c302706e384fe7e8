# GPU tests (optionally a -k filter / file list), then optional config probes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${TAG:-r02}
timeout -k 10 ${TLIM:-600} python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 150 --timeout-method thread ${KSEL:+-k "$KSEL"} > gpurun_out/gputests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gputests_$TAG.log | tail -40
exit $rc
