# qfactor tests, then a rocprofv3 kernel summary of one config probe ($1, default aniso128)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
C=${1:-aniso128}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 150 --timeout-method thread -k "qfactor" > gpurun_out/gputests_qf2.log 2>&1
rc=$?; tail -2 gpurun_out/gputests_qf2.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_$C; mkdir -p gpurun_out/prof_$C
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_configs.py $C > $GRAFT_REPO_ROOT/gpurun_out/prof_$C/out.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_$C/err.txt
echo "prof rc=$?"
rm -f $GRAFT_REPO_ROOT/gpurun_out/prof_$C/run_kernel_trace.csv
cat $GRAFT_REPO_ROOT/gpurun_out/prof_$C/out.json
