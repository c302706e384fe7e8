# round 6: long-column selection / exact-sum paths -- tests, then configs[4] with counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06i}; mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
AMGD_SEGSTAT=1 PROBE_BEAT=0 timeout -k 10 300 python3 tools/probe_configs.py aniso256 > $D/aniso.json 2> $D/aniso.err || { tail -5 $D/aniso.err; exit 1; }
tail -n 1 $D/aniso.json | cut -c1-300; grep segstat $D/aniso.err
