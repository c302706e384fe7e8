# multi-process sharded setup (host transport, every op sharded incl. long-row SpMVs) vs
# one GPU, bit for bit, at sizes past the test suite's: tests/shard_worker.py per rank
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD MASTER_ADDR=127.0.0.1
run() {   # $1 = ranks, $2 = case, $3 = port
  local pids=() rc=0
  for r in $(seq 0 $(($1 - 1))); do
    RANK=$r WORLD_SIZE=$1 MASTER_PORT=$3 SHARD_CASE=$2 timeout -k 10 400 python3 -u tests/shard_worker.py > gpurun_out/shardchk_${2/:/_}_$r.json 2> gpurun_out/shardchk_${2/:/_}_$r.err &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || rc=1; done
  cat gpurun_out/shardchk_${2/:/_}_*.json
  return $rc
}
run 2 p7:48 29611 && run 3 p27:20 29612
