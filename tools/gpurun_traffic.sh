# RAP SpGEMM HBM traffic for the bench roofline: two PMC passes (FETCH_SIZE, WRITE_SIZE)
# over one 256^3 setup, counters collected only on the RAP numeric kernels (RAP=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
M=${1:-256}
RX='k_sg_(row|kseq)<[0-9]+, [0-9]+, 1, 1>|k_sg_win<[0-9]+, 1>|k_spgemm_long<1, 1>'
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/traffic_$C
  timeout -s KILL 400 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d $GRAFT_REPO_ROOT/gpurun_out/traffic_$C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py $M > $GRAFT_REPO_ROOT/gpurun_out/traffic_$C.log 2>&1
  rc=$?
  echo "$C rc=$rc"
  [ $rc -eq 0 ] || exit 1
  ls $GRAFT_REPO_ROOT/gpurun_out/traffic_$C || exit 1
done
exit 0
