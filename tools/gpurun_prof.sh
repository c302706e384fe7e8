set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=${1:-256}
rm -rf gpurun_out/prof$M; mkdir -p gpurun_out/prof$M
cd /tmp && export TMPDIR=/tmp
AMGD_SGLOG=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof$M -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py $M > $GRAFT_REPO_ROOT/gpurun_out/prof$M.log 2>&1; echo "prof rc=$?"
rm -f $GRAFT_REPO_ROOT/gpurun_out/prof$M/run_kernel_trace.csv
grep '"m"' $GRAFT_REPO_ROOT/gpurun_out/prof$M.log
