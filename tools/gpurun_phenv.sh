# phase profiles of one setup at edge $1 under each environment setting given after it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=$1; shift
n=0
for E in "$@"; do
  n=$((n+1))
  env $E AMGD_PHASES=1 timeout -k 10 600 python3 -u tools/probe_scale.py $M > gpurun_out/phenv$n.log 2>&1 || { echo "run $n ($E) failed"; tail -5 gpurun_out/phenv$n.log; exit 1; }
  echo "$E"; grep -A12 "^lvl" gpurun_out/phenv$n.log | grep "^sum\|^lvl"; tail -1 gpurun_out/phenv$n.log | cut -c1-100
done
