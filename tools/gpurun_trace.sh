set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=${1:-128}
rm -rf gpurun_out/trace$M; mkdir -p gpurun_out/trace$M
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/trace$M -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py $M > $GRAFT_REPO_ROOT/gpurun_out/trace$M.log 2>&1; echo "prof rc=$?"
cd $GRAFT_REPO_ROOT && python3 - <<'PY'
import csv, collections, sys
M = sys.argv[1] if len(sys.argv) > 1 else "128"
PY
ls -la gpurun_out/trace$M
grep '"m"' gpurun_out/trace$M.log
