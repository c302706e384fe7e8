# r03 session a: digest parity (default routing) + SEM N>=5 reference fixtures, then the
# GPU's interpolation trace on 27-point 20/24/28/32^3 (compared with the oracle's in profiles/r03)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
export PYTHONPATH=$PWD
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_digests.py tests/test_gpu_parity.py -m gpu -x -v -s \
  --timeout 200 --timeout-method thread -k "digest or sem_e2_N5 or sem_e2_N6 or sem_e2_N7" > gpurun_out/r03a/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|routes" gpurun_out/r03a/tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for m in 20 24 28 32; do
  AMGD_TRACE_MAX_S=90 timeout -k 10 200 python3 tools/oracle_trace.py 27 $m gpurun_out/r03a/p27_${m}_gpu_trace.txt --timeout 170 \
    --lib omp_amg_amd/libomp_amg_amd.so || exit 1
  grep -v find_support gpurun_out/r03a/p27_${m}_gpu_trace.txt | tail -n 4
done
