# partition digests (incremental vs full sweeps) with every rank's stderr on failure
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04e
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_partition.py -m gpu -v --timeout 300 --timeout-method thread -k "digest" > $D/parttests.log 2>&1; r=$?; echo "part tests rc=$r"; grep -E "PASSED|FAILED|passed|failed" $D/parttests.log | tail -20
grep -E "omp_amg_amd|rank [0-9] rc|Abort|abort|expects|failed at" $D/parttests.log | head -40
exit 0
