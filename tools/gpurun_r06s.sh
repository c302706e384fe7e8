# round 6: dense SpGEMM rows by sorting their products -- tests, configs[4], configs[1]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06s}; mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_crs.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
PROBE_BEAT=0 timeout -k 10 300 python3 tools/probe_configs.py aniso256 > $D/aniso.json 2> $D/aniso.err || { tail -5 $D/aniso.err; exit 1; }
tail -n 1 $D/aniso.json | cut -c1-200
timeout -k 10 500 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
tail -n 1 $D/bench.json | cut -c1-300
