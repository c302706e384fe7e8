# bit-map symbolic windows: kernel tests, then A/B at 256^3 with digests
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04p
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k "spgemm" --timeout 120 --timeout-method thread > $D/kern.log 2>&1; r=$?; echo "kernel tests rc=$r"; tail -3 $D/kern.log; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python3 -u tools/ab_setup.py 256 sb=1 sb=0 sb=1 sb=0 ww=2048 sb=1 > $D/ab256.log 2>&1; r=$?; echo "ab rc=$r"; tail -8 $D/ab256.log
