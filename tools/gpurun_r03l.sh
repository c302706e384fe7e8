# r03 session l: Q factor with a column-packed U copy (coalesced s2 pass): kernel tests,
# 256^3 digest with it on, A/B against the row-packed pass
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03l
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 150 --timeout-method thread -k "qfactor" > gpurun_out/r03l/t.log 2>&1 || { tail -30 gpurun_out/r03l/t.log; exit 1; }
tail -2 gpurun_out/r03l/t.log
timeout -k 10 900 python3 tools/ab_setup.py 256 colc=1 default colc=1 default --reps 2 > gpurun_out/r03l/ab256.txt 2>&1 || { tail -5 gpurun_out/r03l/ab256.txt; exit 1; }
grep setting gpurun_out/r03l/ab256.txt
