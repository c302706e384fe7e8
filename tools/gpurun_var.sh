# 256^3 setup timing under several environment variants: VARS="A=1 B=2;A=3" (';'-separated)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
IFS=';' read -ra VS <<< "$VARS"
n=0
for v in "${VS[@]}"; do
  n=$((n+1))
  env $v timeout -k 10 200 python3 tools/probe_scale.py ${M:-256} > gpurun_out/var_$n.out 2> gpurun_out/var_$n.err || { echo "variant $v failed"; tail -5 gpurun_out/var_$n.err; exit 1; }
  echo "[$v] $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/var_$n.out').read().strip().splitlines()[-1]); print(d['t_total_ms'], 'rap', d['rap_kernel_ms'])")"
done
