# bench.py's partitioned path end to end: 2 and 4 ranks on the box's one GPU over the host transport
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04z
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
for N in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --steps 2 --warmup 1 --transport host --edge 96 > $D/bench_part_n$N.json 2> $D/bench_part_n$N.err; r=$?; echo "N=$N rc=$r"; tail -c 1500 $D/bench_part_n$N.json; [ $r -eq 0 ] || { tail -20 $D/bench_part_n$N.err; exit 1; }
done
for N in 4 8; do
  AMGD_PHASES=1 timeout -k 10 500 python3 -u tools/part_peak.py 128 $N $D/part_peak_128_n$N.json > $D/peak$N.log 2>&1; r=$?; echo "peak n$N rc=$r"; grep -E "over_one|bit_id|max_rank_leak" $D/peak$N.log; [ $r -eq 0 ] || exit 1
done
