# SpGEMM / Q-factor per-call log of one setup at edge $1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=${1:-256}
AMGD_SGLOG=1 AMGD_VERBOSE=1 timeout -k 10 600 python3 -u tools/probe_scale.py $M > gpurun_out/sglog$M.log 2>&1; rc=$?
tail -3 gpurun_out/sglog$M.log
exit $rc
