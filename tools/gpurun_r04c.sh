# partition tests (crs fix), per-rank HBM peaks at 128^3 (N = 2, 3), RAP counters at 256^3
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04c
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_partition.py -m gpu -v --timeout 200 --timeout-method thread -k "crs or one_rank" > $D/parttests.log 2>&1; echo "part tests rc=$?"; grep -E "passed|failed" $D/parttests.log | tail -2
timeout -k 10 600 python3 -u tools/part_peak.py 128 2 $D/part_peak_128_n2.json > $D/peak2.log 2>&1; r=$?; echo "peak n2 rc=$r"; tail -5 $D/peak2.log; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python3 -u tools/part_peak.py 128 3 $D/part_peak_128_n3.json > $D/peak3.log 2>&1; r=$?; echo "peak n3 rc=$r"; tail -5 $D/peak3.log; [ $r -eq 0 ] || exit 1
bash tools/gpurun_rapctr.sh r04c 256
