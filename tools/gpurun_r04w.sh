# 8-rank partitioned tests incl. the 7-point 48^3 digest
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04w
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_partition.py -m gpu -v -k eight_ranks --durations=5 --timeout 300 --timeout-method thread > $D/part8.log 2>&1; r=$?; echo "rc=$r"; grep -E "PASSED|FAILED|passed|failed|call " $D/part8.log | tail -12
