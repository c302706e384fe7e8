# one GPU call: a pytest subset, then a short 256^3 bench (one-GPU driver) with its line
# usage: bash tools/gpurun_quick.sh <tag> <steps> <pytest args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-quick}; STEPS=${2:-3}; shift 2
D=$GRAFT_REPO_ROOT/gpurun_out/$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
if [ $# -gt 0 ]; then
timeout -k 10 900 python3 -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $D/tests.log | tail -30; exit 1; }
tail -1 $D/tests.log
fi
timeout -k 10 600 python3 bench.py --steps $STEPS --warmup 1 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
tail -n 1 $D/bench.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('ms', round(d['ms_per_step']), 'frac', round(r['frac'],3), 'mv_ms', round(r['kernel_ms_per_setup']), {k: (round(v['ms_per_setup']), round(v['achieved_gbs'] or 0)) for k, v in r['by_shape'].items()}, 'rap_ms', round(d['rap_roofline']['kernel_ms_per_setup']), d['phases_ms'])"
