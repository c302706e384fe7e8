# Counters of the RAP SpGEMM numeric kernels (and the long-row SpMV) on one 256^3 setup:
# L2 hit/miss, LDS instructions / bank-conflict cycles, busy / wait cycles -- one rocprofv3
# --pmc pass per group, each its own run (ADVICE/VERDICT r3: product-bound or miss-bound?).
# usage: bash tools/gpurun_rapctr.sh <tag> [m]
set -o pipefail
TAG=${1:-r04}
M=${2:-256}
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/rapctr_$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
RX=${RX:-'k_sg_(row|kseq)<[0-9]+, [0-9]+, 1, 1>|k_sg_wwin<|k_spgemm_long<1, 1>|k_spmv_(pipe|pair)<false'}
i=0
for G in "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $G --kernel-include-regex "$RX" -d $D/pass$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py $M > $D/pass$i.log 2>&1
  r=$?; echo "pass $i ($G) rc=$r"; [ $r -eq 0 ] || exit 1
done
cd $GRAFT_REPO_ROOT && python3 tools/rapctr_sum.py $D > $D/summary.txt && cat $D/summary.txt
find $D -name "*counter_collection.csv" -size +30M -delete
