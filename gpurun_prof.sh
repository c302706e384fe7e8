set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof32
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof32 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py 32 > $GRAFT_REPO_ROOT/gpurun_out/prof32.log 2>&1; echo "prof rc=$?"
cd $GRAFT_REPO_ROOT
tail -2 gpurun_out/prof32.log
find gpurun_out/prof32 -name "*stats*" | head
