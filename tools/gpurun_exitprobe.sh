# does the rocprofv3 exit-time SIGSEGV come from amgd_shutdown?  (probe without it)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp
AMGD_NO_SHUTDOWN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/exitprobe -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py 32 > $GRAFT_REPO_ROOT/gpurun_out/exitprobe.log 2>&1
echo "no-shutdown rc=$?"
