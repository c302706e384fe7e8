# per-shape SpMV kernel comparison at 256^3 (AMGD_MVLOG): lane-0 wave, all-lane, all-wave
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
AMGD_SPMV_BN=0 AMGD_MVLOG=1 timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/mv_def.out 2> gpurun_out/mv_def.err || exit $?
AMGD_SPMV_BN=0 AMGD_MVLOG=1 AMGD_SL_MIN_ROWS=0 timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/mv_lane.out 2> gpurun_out/mv_lane.err || exit $?
AMGD_SPMV_BN=0 AMGD_MVLOG=1 AMGD_SL_MIN_ROWS=1099511627776 timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/mv_wave.out 2> gpurun_out/mv_wave.err || exit $?
cat gpurun_out/mv_def.out gpurun_out/mv_lane.out gpurun_out/mv_wave.out
