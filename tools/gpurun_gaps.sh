# GPU idle time between kernels over one 256^3 setup (rocprofv3 --kernel-trace), attributed
# to the kernel pairs around each gap (tools/ktrace_gaps.py); the trace CSV is dropped.
# usage: bash tools/gpurun_gaps.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r05}
D=$GRAFT_REPO_ROOT/gpurun_out/gaps_$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $D/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py 256 > $D/probe.log 2>&1 || { tail -5 $D/probe.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $D/tr -name "*kernel_trace.csv" | head -1)
python3 tools/ktrace_gaps.py $f 1.0 > $D/gaps.txt && head -60 $D/gaps.txt
find $D -name "*kernel_trace.csv" -delete
