# round 6: long-row split records + thresholded incremental constraint pattern: kernel tests,
# digests, A/B on configs[1] / [4]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06v}; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "binade_jumps or multichunk or adversarial_rows or exact_dot or spgemm" > $D/ktests.log 2>&1 || { tail -40 $D/ktests.log; exit 1; }
tail -2 $D/ktests.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $D/dtests.log 2>&1 || { tail -40 $D/dtests.log; exit 1; }
tail -2 $D/dtests.log
AMGD_SEGSTAT=1 PROBE_BEAT=0 timeout -k 10 300 python3 tools/probe_configs.py aniso256 > $D/aniso_stat.json 2> $D/aniso_stat.err || { tail -5 $D/aniso_stat.err; exit 1; }
grep segstat $D/aniso_stat.err
timeout -k 10 500 python3 -u tools/ab_setup.py 256 spat=1 spat=0 --reps 2 > $D/ab256.txt 2>&1 || { tail -5 $D/ab256.txt; exit 1; }
grep setting $D/ab256.txt
