set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for m in 24 32 48; do
  timeout -k 10 150 python tools/probe_scale.py $m >> gpurun_out/probe2.log 2>&1 || { echo "m=$m failed rc=$?"; break; }
done
cat gpurun_out/probe2.log
