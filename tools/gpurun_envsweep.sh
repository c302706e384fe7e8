# one-setup bench per kernel-choice setting (all settings give the same bits)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for kv in "X=0" "AMGD_SG_WIN=4096" "AMGD_SG_WIN=1024" "AMGD_SG_WSYM=65536" "AMGD_SG_WSYM=16384"; do
  env $kv timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/sweep.json 2> gpurun_out/sweep.err || { echo "$kv failed"; tail -5 gpurun_out/sweep.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep.json').read().strip().splitlines()[-1]); print('$kv', round(d['ms_per_step']/1e3,3), 's')"
done
