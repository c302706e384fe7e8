# round 6: SpMV gather-locality statistics of a 256^3 setup (AMGD_MVSTAT=1) and a
# rocprofv3 kernel summary of configs[4] (anisotropic 256^3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r06d; mkdir -p $D
AMGD_MVSTAT=1 timeout -k 10 500 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $D/mvstat.json 2> $D/mvstat.err || { tail -5 $D/mvstat.err; exit 1; }
grep mvstat $D/mvstat.err > $D/mvstat.txt; rm -f $D/mvstat.err
cd /tmp && export TMPDIR=/tmp
PROBE_BEAT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_aniso -o aniso --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_configs.py aniso256 > $D/aniso.json 2> $D/aniso.err
rc=$?
find /tmp/prof_aniso -name "*kernel_stats.csv" -exec cp {} $D/aniso_kernel_stats.csv \;
tail -c 20000 $D/aniso.err > $D/aniso_tail.err; rm -f $D/aniso.err
echo "rocprof rc=$rc"; tail -n 2 $D/aniso.json | cut -c1-400
