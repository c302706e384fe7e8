# per-call logs of one setup at edge $1 under each environment setting given after it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=$1; shift
n=0
for E in "$@"; do
  n=$((n+1))
  env $E AMGD_SGLOG=1 AMGD_VERBOSE=1 timeout -k 10 600 python3 -u tools/probe_scale.py $M > gpurun_out/envcmp$n.log 2>&1 || { echo "run $n ($E) failed"; tail -5 gpurun_out/envcmp$n.log; exit 1; }
  echo "$E: $(tail -1 gpurun_out/envcmp$n.log | cut -c1-120)"
done
