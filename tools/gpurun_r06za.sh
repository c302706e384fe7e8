# round 6: dot speculation threshold (chunks) -- kernel tests, interleaved A/B on configs[1]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06za}; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "exact_dot" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 700 python3 -u tools/ab_setup.py 256 dsm=16 dsm=4 dsm=2 dsm=16 dsm=4 dsm=2 > $D/ab256.txt 2>&1 || { tail -5 $D/ab256.txt; exit 1; }
grep setting $D/ab256.txt
