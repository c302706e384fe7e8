# r03 session i: contiguous-chunk SpMV (k_spmv_chunk) and the fused find_support
# selection -- kernel + parity tests, micro-benchmark against the row-segment kernel,
# 256^3 digest (must equal 52a7958624e27375e91c8707) + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03i
export PYTHONPATH=$PWD
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "spmv or fused" > gpurun_out/r03i/t.log 2>&1 || { tail -30 gpurun_out/r03i/t.log; exit 1; }
tail -2 gpurun_out/r03i/t.log
timeout -k 10 300 python3 -u tools/spmv_bench.py --chunk > gpurun_out/r03i/spmv_bench.txt 2>&1 || { tail -5 gpurun_out/r03i/spmv_bench.txt; exit 1; }
cat gpurun_out/r03i/spmv_bench.txt
timeout -k 10 300 python3 tools/ab_setup.py 256 default > gpurun_out/r03i/digest256.txt 2>&1 || { tail -5 gpurun_out/r03i/digest256.txt; exit 1; }
grep setting gpurun_out/r03i/digest256.txt
timeout -k 10 700 python3 tools/ab_setup.py 256 default chunk=0 fused=0 --reps 2 --no-digest > gpurun_out/r03i/ab256.txt 2>&1 || { tail -5 gpurun_out/r03i/ab256.txt; exit 1; }
grep setting gpurun_out/r03i/ab256.txt
