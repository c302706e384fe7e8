set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python bench.py --m 128 --no-cpu-baseline > gpurun_out/bench128.log 2>&1; echo "b128 rc=$?"; tail -2 gpurun_out/bench128.log
timeout -k 10 600 python bench.py --m 256 --cpu-m 20 > gpurun_out/bench256.log 2>&1; echo "b256 rc=$?"; tail -3 gpurun_out/bench256.log
