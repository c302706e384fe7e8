# Where the long-row SpMV's time goes: texture-address (TA) busy and stall cycles, L1
# (TCP) cache-line accesses per load instruction, L1 TLB (UTCL1) misses -- one rocprofv3
# --pmc pass per group on one 256^3 setup, each its own run.
# usage: bash tools/gpurun_mvctr.sh <tag> [m]
set -o pipefail
TAG=${1:-r05}
M=${2:-256}
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/mvctr_$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
RX=${RX:-'k_spmv_(pair|pipe)<false'}
i=0
for G in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
         "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $G --kernel-include-regex "$RX" -d $D/pass$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py $M > $D/pass$i.log 2>&1
  r=$?; echo "pass $i ($G) rc=$r"; [ $r -eq 0 ] || exit 1
done
cd $GRAFT_REPO_ROOT && python3 tools/mvctr_sum.py $D > $D/summary.txt && cat $D/summary.txt
find $D -name "*counter_collection.csv" -size +30M -delete
