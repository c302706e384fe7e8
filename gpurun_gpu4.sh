set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -q > gpurun_out/parity.log 2>&1; echo "parity rc=$?"
tail -40 gpurun_out/parity.log
