# per-rank HBM peaks of the partitioned setup (host transport, N processes on one GPU)
# usage: bash tools/gpurun_partpeak.sh <tag> "<m> <N> <stencil>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
D=$GRAFT_REPO_ROOT/gpurun_out/pp_$TAG
mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
for cfg in "$@"; do
  set -- $cfg
  f=$D/part_peak_p$3_$1_n$2.json
  timeout -k 10 1000 python3 -u tools/part_peak.py $1 $2 $f --stencil $3 --timeout 900 $PP_EXTRA > $D/p$3_$1_n$2.log 2>&1 || { echo "FAILED $cfg"; tail -5 $D/p$3_$1_n$2.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$f'))
print('$cfg', 'identical', d['bit_identical'], 'one_gpu_GB', round(d['one_gpu']['peak_bytes']/1e9,2), 'rank_peak_GB', round(d['max_rank_peak_bytes']/1e9,2), 'ratio', round(d['max_rank_peak_over_one_gpu'],3), 'secs', round(d['one_gpu']['secs'],1), [round(r['secs'],1) for r in d['partitioned']][:1], 'levels', d['one_gpu']['levels'])"
done
