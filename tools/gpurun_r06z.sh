# round 6: split records in the exact dots -- kernel tests, counters, interleaved A/B on configs[1]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06z}; mkdir -p $D
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "exact_dot or binade_jumps or multichunk_exact or dot" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
AMGD_SEGSTAT=1 timeout -k 10 200 python3 -u tools/ab_setup.py 128 default --no-digest > $D/segstat128.txt 2>&1 || { tail -5 $D/segstat128.txt; exit 1; }
grep -h "segstat\|setting" $D/segstat128.txt
timeout -k 10 500 python3 -u tools/ab_setup.py 256 dsp=0 dsp=1 dsp=0 dsp=1 > $D/ab256.txt 2>&1 || { tail -5 $D/ab256.txt; exit 1; }
grep setting $D/ab256.txt
