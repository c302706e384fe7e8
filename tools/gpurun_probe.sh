# one GPU call of short probes: default routes by box size, the forced RW=64 digests,
# the partitioned driver on a one-rank RCCL communicator at 256^3 (bench --mode part).
# usage: bash tools/gpurun_probe.sh <tag> [boxes...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r05probe}; shift
D=$GRAFT_REPO_ROOT/gpurun_out/$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
BOXES=${@:-256x256x128}
timeout -k 10 300 python3 -u tools/route_probe.py $BOXES > $D/routes.jsonl 2> $D/routes.err || { tail -20 $D/routes.err; exit 1; }
cat $D/routes.jsonl
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_digests.py -k rw64 -x -v -s --timeout 200 --timeout-method thread > $D/rw64.log 2>&1 || { tail -30 $D/rw64.log; exit 1; }
grep -E "PASS|FAIL|p7_" $D/rw64.log | tail -6
if [ -z "$SKIP_PART" ]; then
timeout -k 10 500 python3 bench.py --gpus 1 --mode part --steps 2 --warmup 1 --no-cpu-baseline > $D/bench_part_n1.json 2> $D/bench_part_n1.err || { tail -20 $D/bench_part_n1.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_part_n1.json')); print({k: d[k] for k in ('value','ms_per_step','steps')}, d['phases_ms'], d.get('comm_rank0_per_step'), d.get('peak_hbm_bytes_rank0'))"
fi
