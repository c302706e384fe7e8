# partition digests (incremental fix), per-rank peak 128^3 N=2 with phase peaks, XCD-order A/B at 256^3
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04f
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_partition.py -m gpu -v --timeout 300 --timeout-method thread -k "digest" > $D/parttests.log 2>&1; r=$?; echo "part tests rc=$r"; grep -E "PASSED|FAILED|passed|failed" $D/parttests.log | tail -12
[ $r -eq 0 ] || { grep -E "omp_amg_amd|rank [0-9] rc" $D/parttests.log | head -20; exit 1; }
AMGD_PHASES=1 timeout -k 10 400 python3 -u tools/part_peak.py 128 2 $D/part_peak_128_n2.json > $D/peak2.log 2>&1; r=$?; echo "peak n2 rc=$r"; grep -E "over_one|bit_id" $D/peak2.log; [ $r -eq 0 ] || exit 1
timeout -k 10 120 python3 -u tools/ab_setup.py 64 default xcd=7 xcd=1 > $D/ab64.log 2>&1; echo "ab64 rc=$?"; cat $D/ab64.log | grep setting
timeout -k 10 420 python3 -u tools/ab_setup.py 256 --no-digest default xcd=1 xcd=7 default xcd=7 xcd=1 > $D/ab256.log 2>&1; echo "ab256 rc=$?"; grep setting $D/ab256.log
