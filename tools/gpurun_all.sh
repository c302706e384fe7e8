# full GPU test suite (log under gpurun_out/), then the phase profile at edge $1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_all.log 2>&1 || { tail -30 gpurun_out/gputests_all.log; exit 1; }
tail -2 gpurun_out/gputests_all.log
bash tools/gpurun_phenv.sh ${1:-256} AMGD_CLOG=1
