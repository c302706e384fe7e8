# per-rank peak at 128^3 with 4 and 8 ranks (host transport, one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04aa
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
for N in 4 8; do
  AMGD_PHASES=1 timeout -k 10 700 python3 -u tools/part_peak.py 128 $N $D/part_peak_128_n$N.json --timeout 650 > $D/peak$N.log 2>&1; r=$?; echo "peak n$N rc=$r"; grep -E "over_one|bit_id|max_rank_leak" $D/peak$N.log; [ $r -eq 0 ] || exit 1
done
