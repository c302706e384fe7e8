# r03 session h: fused find_support selection -- parity tests, the 256^3 digest (must
# equal 52a7958624e27375e91c8707) and a 3-rep A/B of the fused selection
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03h
export PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused" > gpurun_out/r03h/t.log 2>&1 || { tail -30 gpurun_out/r03h/t.log; exit 1; }
tail -2 gpurun_out/r03h/t.log
timeout -k 10 300 python3 tools/ab_setup.py 256 default > gpurun_out/r03h/digest256.txt 2>&1 || { tail -5 gpurun_out/r03h/digest256.txt; exit 1; }
grep setting gpurun_out/r03h/digest256.txt
timeout -k 10 700 python3 tools/ab_setup.py 256 default fused=0 default --reps 3 --no-digest > gpurun_out/r03h/ab256.txt 2>&1 || { tail -5 gpurun_out/r03h/ab256.txt; exit 1; }
grep setting gpurun_out/r03h/ab256.txt
