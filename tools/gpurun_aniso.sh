# tests touching the Q factor, then a long diagnostic run of configs[4] (aniso 256^3)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "qfactor or bitexact" > gpurun_out/gputests_qf.log 2>&1
rc=$?; tail -2 gpurun_out/gputests_qf.log; [ $rc -eq 0 ] || exit $rc
AMGD_PHASES=1 AMGD_SGLOG=1 AMGD_FSLOG=1 timeout -k 10 ${LIM:-900} python3 -u tools/probe_configs.py aniso256 > gpurun_out/aniso256_diag.json 2> gpurun_out/aniso256_diag.err
echo "aniso rc=$?"; cat gpurun_out/aniso256_diag.json
exit 0
