# verbose + phase profile of one setup at edge $1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=${1:-256}
AMGD_VERBOSE=1 AMGD_PHASES=1 timeout -k 10 600 python3 -u tools/probe_scale.py $M > gpurun_out/phv$M.log 2>&1; rc=$?
tail -16 gpurun_out/phv$M.log
exit $rc
