# round 6 close (dots' split records): kernel summary of the bench command, the driver's bench
# command (fewer steps; SpMV / RAP kernels unchanged since r06y, so its PMC traffic file stands),
# configs[4]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
TAG=${TAG:-r06zc}
D=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $D/prof_line.json 2>&1 || { tail -5 $D/prof_line.json; exit 1; }
find $D -name "*kernel_trace.csv" -delete
tail -n 1 $D/prof_line.json | cut -c1-300
cd $GRAFT_REPO_ROOT
t0=$(date +%s)
timeout -k 10 400 python3 bench.py --gpus 1 --steps 4 --warmup 1 > $D/bench.json 2> $D/bench.err || { echo bench failed; tail -20 $D/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
tail -n 1 $D/bench.json | cut -c1-400
PROBE_BEAT=0 timeout -k 10 300 python3 tools/probe_configs.py aniso256 > $D/aniso.json 2> $D/aniso.err || { tail -5 $D/aniso.err; exit 1; }
tail -n 1 $D/aniso.json | cut -c1-200
