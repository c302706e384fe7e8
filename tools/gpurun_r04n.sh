# per-rank peak 128^3 N=2: exchanges by kind
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04n
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
AMGD_PHASES=1 timeout -k 10 400 python3 -u tools/part_peak.py 128 2 $D/part_peak_128_n2.json > $D/peak2.log 2>&1; r=$?; echo "peak n2 rc=$r"; grep -E "over_one|bit_id|leak" $D/peak2.log; [ $r -eq 0 ] || exit 1
