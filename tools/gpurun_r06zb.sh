# round 6 close: the full GPU suite on the final tree (the driver's command, one process)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06zb}; mkdir -p $D
t0=$(date +%s)
timeout -k 10 1140 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gputests.log 2>&1
r=$?
echo "suite rc=$r wall $(( $(date +%s) - t0 )) s" | tee -a $D/gputests.log
tail -3 $D/gputests.log
exit $r
