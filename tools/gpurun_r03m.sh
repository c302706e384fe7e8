# r03 session m: new defaults (k_spmv_pipe 16 per lane, k_sg_wwin for windowed numeric rows
# at 1024 columns, short-row SpMV loads 8 in flight): SpMV / SpGEMM kernel tests, then
# 256^3 A/B of the symbolic wave windows (16384- / 4096-column byte maps) against it
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03m5
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 150 --timeout-method thread -k "spmv or spgemm" > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 1; }
tail -2 $D/t.log
timeout -k 10 700 python3 tools/ab_setup.py 256 --no-digest --reps 2 default ww=11 ww=27 > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
