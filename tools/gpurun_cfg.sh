# full-size probes of BASELINE configs[2] / configs[4] (one setup each, phase table on stderr)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${TAG:-r02}
for c in "$@"; do
  lim=${LIM:-300}
  AMGD_PHASES=1 timeout -k 10 $lim python3 -u tools/probe_configs.py $c > gpurun_out/cfg_${c}_$TAG.json 2> gpurun_out/cfg_${c}_$TAG.err
  rc=$?
  echo "$c rc=$rc"; cat gpurun_out/cfg_${c}_$TAG.json
  [ $rc -eq 0 ] || exit $rc
done
