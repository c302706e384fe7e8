# r03 session b: digest parity (default routing), crs_setup / OOM / multi-rank crs tests,
# the tiled windowed SpGEMM kernel tests, then the GPU's interpolation trace on
# 27-point 20/24/28/32^3 (the oracle's are in profiles/r03)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03b
export PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_digests.py tests/test_gpu_crs.py tests/test_gpu_shard.py tests/test_gpu_kernels.py -m gpu -x -v -s \
  --timeout 200 --timeout-method thread -k "digest or crs or hbm or host_transport or tiled" > gpurun_out/r03b/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/r03b/tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for m in 20 24 28 32; do
  AMGD_TRACE_MAX_S=80 timeout -k 10 200 python3 tools/oracle_trace.py 27 $m gpurun_out/r03b/p27_${m}_gpu_trace.txt --timeout 170 \
    --lib omp_amg_amd/libomp_amg_amd.so || exit 1
  grep -v find_support gpurun_out/r03b/p27_${m}_gpu_trace.txt | tail -n 4
done
