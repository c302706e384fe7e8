# r03 session o: short-B-row (flat) SpGEMM hash bins through k_sg_wwin (bit 128): kernel
# tests, 256^3 A/B against the default
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03o
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 150 --timeout-method thread -k "wave_windows" > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 1; }
tail -2 $D/t.log
timeout -k 10 500 python3 tools/ab_setup.py 256 --no-digest --reps 2 default ww=155 > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
