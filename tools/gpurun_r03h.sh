# r03 session h: fused find_support selection -- parity tests (kernel routes, fixtures,
# digests), 256^3 digest (must equal 52a7958624e27375e91c8707) and a 3-rep A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03h
export PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or digest or bitexact_spmv or reference_fixture" > gpurun_out/r03h/t.log 2>&1 || { tail -30 gpurun_out/r03h/t.log; exit 1; }
tail -2 gpurun_out/r03h/t.log
timeout -k 10 600 python3 tools/ab_setup.py 256 default fused=0 default --reps 3 > gpurun_out/r03h/ab256.txt 2>&1 || { tail -5 gpurun_out/r03h/ab256.txt; exit 1; }
cat gpurun_out/r03h/ab256.txt
