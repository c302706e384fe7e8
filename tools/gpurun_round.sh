# one GPU session: full parity suite, the driver's bench command, a rocprofv3 kernel
# summary of a short bench run, and FETCH_SIZE / WRITE_SIZE passes over the SpMV and
# RAP roofline kernels (one counter per pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${1:-r02}
if [ -z "$SKIP_TESTS" ]; then   # SKIP_TESTS=1: the suite already ran green on this tree
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/gputests_$TAG.log
[ $rc -eq 0 ] || exit $rc
fi
t0=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
cat gpurun_out/bench_$TAG.json
rm -rf gpurun_out/prof_$TAG; mkdir -p gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG/bench_line.json 2>&1; echo "prof rc=$?"
rm -f $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG/bench_kernel_trace.csv
for K in spmv rap; do
  if [ $K = spmv ]; then RX='k_spmv_lane<false'; else RX='k_sg_(row|kseq)<[0-9]+, [0-9]+, 1, 1>|k_sg_win<[0-9]+, 1>|k_spgemm_long<1, 1>'; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf $GRAFT_REPO_ROOT/gpurun_out/traffic_${K}_$C
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d $GRAFT_REPO_ROOT/gpurun_out/traffic_${K}_$C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py 256 > $GRAFT_REPO_ROOT/gpurun_out/traffic_${K}_$C.log 2>&1
    r=$?; echo "$K $C rc=$r"; [ $r -eq 0 ] || exit 1
  done
done
exit 0
