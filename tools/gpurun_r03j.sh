# r03 session j: SpMV kernel tests (chunks forced at every row length), lmop wavefront walk
# and Q-reuse tests, 256^3 digest, A/B of the chunk kernel and the lmop wavefront walk
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03j
export PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "spmv or fused or lmop or qfactor" > gpurun_out/r03j/t.log 2>&1 || { tail -30 gpurun_out/r03j/t.log; exit 1; }
tail -2 gpurun_out/r03j/t.log
timeout -k 10 300 python3 tools/ab_setup.py 256 default > gpurun_out/r03j/digest256.txt 2>&1 || { tail -5 gpurun_out/r03j/digest256.txt; exit 1; }
grep setting gpurun_out/r03j/digest256.txt
timeout -k 10 700 python3 tools/ab_setup.py 256 default chunk=0 lw=0 default --reps 2 --no-digest > gpurun_out/r03j/ab256.txt 2>&1 || { tail -5 gpurun_out/r03j/ab256.txt; exit 1; }
grep setting gpurun_out/r03j/ab256.txt
