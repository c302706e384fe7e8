# selected GPU tests ($1 = pytest -k expression), then the per-call log at edge $2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$1" > gpurun_out/gputests_k.log 2>&1 || { tail -40 gpurun_out/gputests_k.log; exit 1; }
tail -3 gpurun_out/gputests_k.log
[ -z "$2" ] && exit 0
M=$2
AMGD_SGLOG=1 AMGD_VERBOSE=1 timeout -k 10 600 python3 -u tools/probe_scale.py $M > gpurun_out/sglog$M.log 2>&1; rc=$?
tail -2 gpurun_out/sglog$M.log
exit $rc
