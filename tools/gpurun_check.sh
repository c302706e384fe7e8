# quick GPU check after a change: selected GPU tests, a short bench, optional config probes
# env: KSEL (pytest -k), TESTS (files), TAG, STEPS, CFGS (probe_configs names)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${TAG:-chk}
if [ -n "$KSEL$TESTS" ]; then
  timeout -k 10 ${TLIM:-600} python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 150 --timeout-method thread ${KSEL:+-k "$KSEL"} > gpurun_out/gputests_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/gputests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${STEPS:-2}" != 0 ]; then
  AMGD_PHASES=${PHASES:-0} timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps ${STEPS:-2} --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
fi
for c in $CFGS; do
  AMGD_PHASES=1 timeout -k 10 ${LIM:-300} python3 -u tools/probe_configs.py $c > gpurun_out/cfg_${c}_$TAG.json 2> gpurun_out/cfg_${c}_$TAG.err
  rc=$?; echo "$c rc=$rc"; cat gpurun_out/cfg_${c}_$TAG.json; [ $rc -eq 0 ] || exit $rc
done
exit 0
