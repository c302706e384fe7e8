# PMC traffic of the roofline kernels (one counter per pass, separate runs) + the
# counter calibration on the lane SpMV's access pattern, and a kernel-trace summary of
# the bench command on the same tree.  usage: bash tools/gpurun_pmc.sh <tag>
set -o pipefail
TAG=${1:-r03}
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $GRAFT_REPO_ROOT/tools/pmc_calib.py > $D/calib.json 2>&1 || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'k_spmv_(lane|pipe)' -d $D/calib_$C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pmc_calib.py > $D/calib_$C.log 2>&1
  r=$?; echo "calib $C rc=$r"; [ $r -eq 0 ] || exit 1
done
for K in spmv rap; do
  if [ $K = spmv ]; then RX='k_spmv_(pipe|pair)<false|k_spmv_pair_amx'; else RX='k_sg_(row|kseq)<[0-9]+, [0-9]+, 1, 1>|k_sg_win<[0-9]+, 1>|k_sg_wwin<[0-9]+, 1, 1>|k_spgemm_long<1, 1>'; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d $D/traffic_${K}_$C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py 256 > $D/traffic_${K}_$C.log 2>&1
    r=$?; echo "$K $C rc=$r"; [ $r -eq 0 ] || exit 1
  done
done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_traffic_json.py $D $TAG > $D/traffic_$TAG.json && cat $D/traffic_$TAG.json | head -40
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $D/prof_line.json 2>&1 || exit 1
find $D -name "*kernel_trace.csv" -delete
find $D -name "*counter_collection.csv" -size +20M -delete
tail -n 1 $D/prof_line.json
