# parity tests + a verbose 256^3 setup (per-level sizes, per-call SpGEMM/Q-factor logs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=${1:-256}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
AMGD_VERBOSE=1 AMGD_SGLOG=1 timeout -k 10 600 python3 -u tools/probe_scale.py $M > gpurun_out/diag$M.log 2>&1; rc=$?
tail -5 gpurun_out/diag$M.log
exit $rc
