# round 6: SpGEMM / Q-factor log of one configs[1] setup (tier counts, reuse, times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06n}; mkdir -p $D
AMGD_SGLOG=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $D/bench.json 2> $D/sglog.txt || { tail -5 $D/sglog.txt; exit 1; }
grep -c . $D/sglog.txt; tail -n 1 $D/bench.json | cut -c1-200
