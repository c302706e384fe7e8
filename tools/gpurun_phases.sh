# per-level phase profile of one setup (AMGD_PHASES=1); args: grid edge, extra probe flags
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=${1:-256}
AMGD_PHASES=1 timeout -k 10 600 python3 -u tools/probe_scale.py $M $2 > gpurun_out/phases$M.log 2>&1; rc=$?
tail -22 gpurun_out/phases$M.log
exit $rc
