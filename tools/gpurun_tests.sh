# one GPU call: a subset of the GPU suite (pytest -k / file args), then optional steps
# usage: bash tools/gpurun_tests.sh <tag> <pytest args...>
#   PHASES=1: afterwards one-GPU and partitioned-N=1 setups of 256^3 with AMGD_PHASES=1
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-tests}; shift
D=$GRAFT_REPO_ROOT/gpurun_out/$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
if [ $# -gt 0 ]; then
timeout -k 10 1000 python3 -u -m pytest "$@" -x -v --durations=20 --timeout 400 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $D/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $D/tests.log | tail -2
grep -E "s call" $D/tests.log | head -12
fi
if [ -n "$PHASES" ]; then
for mode in one part; do
  extra=""; [ $mode = part ] && extra="--mode part"
  AMGD_PHASES=1 timeout -k 10 400 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline $extra > $D/bench_$mode.json 2> $D/phases_$mode.log || { tail -20 $D/phases_$mode.log; exit 1; }
  tail -n 1 $D/bench_$mode.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', round(d['ms_per_step']), d['phases_ms'])"
done
fi
if [ -n "$SITES" ]; then
  # collectives per call site of a partitioned setup over the host transport (N ranks, one GPU)
  AMGD_COMM_SITES=1 AMGD_PHASES=1 timeout -k 10 600 python3 -u tools/part_peak.py $SITES $D/part_peak.json > $D/part_peak.log 2>&1 || { tail -20 $D/part_peak.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/part_peak.json'))
print('bit_identical', d['bit_identical'], 'peak ratio', round(d['max_rank_peak_over_one_gpu'],3), 'secs', [round(r['secs'],1) for r in d['partitioned']], 'calls', [r['comm_calls'] for r in d['partitioned']])
for l in d['partitioned'][0]['phase_peaks']:
    if 'site' in l or 'collectives' in l or 'exchanges' in l: print(l)
"
fi
