# one SQ PMC pass (8 counters) over the kernels matching $RX in one setup of size $M
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${TAG:-sq}
CT=${CT:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS}
rm -rf gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc $CT --kernel-include-regex "$RX" -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py ${M:-256} > $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.log 2>&1
rc=$?; echo "pmc rc=$rc"
cd $GRAFT_REPO_ROOT && python3 tools/pmc_sum.py gpurun_out/pmc_$TAG/run_counter_collection.csv | head -60
exit $rc
