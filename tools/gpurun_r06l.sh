# round 6: rocprofv3 kernel summaries of configs[4] and configs[1] on this tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06l}; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
PROBE_BEAT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pa -o a --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_configs.py aniso256 > $D/aniso.json 2> $D/aniso.err
echo "aniso rc=$?"
find /tmp/pa -name "*kernel_stats.csv" -exec cp {} $D/aniso_kernel_stats.csv \;
tail -c 3000 $D/aniso.err > $D/aniso_tail.err; rm -f $D/aniso.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $D/bench.json 2> $D/bench.err
echo "bench rc=$?"
find /tmp/pb -name "*kernel_stats.csv" -exec cp {} $D/bench_kernel_stats.csv \;
tail -c 3000 $D/bench.err > $D/bench_tail.err; rm -f $D/bench.err
ls -la $D
