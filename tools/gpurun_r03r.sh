# r03 session r: interp_lmop row pull with short S rows one thread each (k_lmop_pull_small):
# lmop tests (fast path vs general walk, both row kernels), 256^3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03r
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lmop.py -m gpu -x -q --timeout 150 --timeout-method thread > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 1; }
tail -2 $D/t.log
timeout -k 10 500 python3 tools/ab_setup.py 256 --reps 2 default lsm=0 > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
