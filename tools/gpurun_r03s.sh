# r03 session s: find_support column sums from the w = R' rs pass (k_spmv_pipe SUM2):
# parity (sum2 on / off, incremental sweeps default / off / all), 256^3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03s
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 150 --timeout-method thread -k "sum2 or fused or spmv" > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 1; }
tail -2 $D/t.log
timeout -k 10 500 python3 tools/ab_setup.py 256 --reps 2 default sum2=0 > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
