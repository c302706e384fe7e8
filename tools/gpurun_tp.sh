# GPU parity tests, then a per-level phase profile of one setup at edge $1 (default 256)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=${1:-256}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
AMGD_PHASES=1 timeout -k 10 600 python3 -u tools/probe_scale.py $M > gpurun_out/phases$M.log 2>&1; rc=$?
tail -16 gpurun_out/phases$M.log
exit $rc
