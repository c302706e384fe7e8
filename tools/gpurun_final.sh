# GPU suite on the tree, then the nontemporal-load SpMV comparison (tools/gpurun_ntcmp.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${TAG:-fin}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/gputests_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpurun_ntcmp.sh
