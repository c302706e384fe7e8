# r03 session e: new kernel tests (pattern-only SpGEMM, column mask, Q-factor reuse),
# 256^3 digest + time per setting (every digest must equal the round's reference
# 52a7958624e27375e91c8707), the full GPU suite, then the 27-point 64^3 trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03e
export PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "pattern or cols_masked or qfactor_reuse" > gpurun_out/r03e/k.log 2>&1 || { tail -30 gpurun_out/r03e/k.log; exit 1; }
tail -2 gpurun_out/r03e/k.log
timeout -k 10 420 python3 tools/ab_setup.py 256 default qfr=0 pat=0 > gpurun_out/r03e/ab256.txt 2>&1 || { tail -5 gpurun_out/r03e/ab256.txt; exit 1; }
cat gpurun_out/r03e/ab256.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03e/gputests.log 2>&1 || { tail -30 gpurun_out/r03e/gputests.log; exit 1; }
tail -3 gpurun_out/r03e/gputests.log
AMGD_TRACE_MAX_S=100 timeout -k 10 200 python3 tools/oracle_trace.py 27 64 gpurun_out/r03e/p27_64_gpu_trace.txt --timeout 170 --lib omp_amg_amd/libomp_amg_amd.so || exit 1
grep -v find_support gpurun_out/r03e/p27_64_gpu_trace.txt | tail -n 6
