# partition tests + per-rank peaks 128^3 N=2/3 with the own Q factors kept only in the lmop halo view
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04bb
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_partition.py -m gpu -v --timeout 300 --timeout-method thread > $D/parttests.log 2>&1; r=$?; echo "part tests rc=$r"; grep -E "PASSED|FAILED|passed|failed" $D/parttests.log | tail -25
[ $r -eq 0 ] || { grep -E "omp_amg_amd|rank [0-9] rc" $D/parttests.log | head -20; exit 1; }
AMGD_PHASES=1 timeout -k 10 400 python3 -u tools/part_peak.py 128 2 $D/part_peak_128_n2.json > $D/peak2.log 2>&1; r=$?; echo "peak n2 rc=$r"; grep -E "over_one|bit_id|leak" $D/peak2.log; grep -E "rank 0 (L|interp)" $D/peak2.log; [ $r -eq 0 ] || exit 1
AMGD_PHASES=1 timeout -k 10 400 python3 -u tools/part_peak.py 128 3 $D/part_peak_128_n3.json > $D/peak3.log 2>&1; r=$?; echo "peak n3 rc=$r"; grep -E "over_one|bit_id|leak" $D/peak3.log; grep -E "rank 0 (L|interp)" $D/peak3.log; [ $r -eq 0 ] || exit 1
