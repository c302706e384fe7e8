# round 6: gather-table SpMV -- kernel tests, default-routed digests, bench with / without
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r06e; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -k gather_table tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 500 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/bench_tab.json 2> $D/bench_tab.err || { tail -5 $D/bench_tab.err; exit 1; }
tail -n 1 $D/bench_tab.json | cut -c1-600
AMGD_MV_TAB=0 timeout -k 10 500 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/bench_notab.json 2> $D/bench_notab.err || { tail -5 $D/bench_notab.err; exit 1; }
tail -n 1 $D/bench_notab.json | cut -c1-300
