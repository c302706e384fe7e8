# round 6: gather-table SpMV -- digests with default routing, then rocprof kernel summaries
# of one 256^3 setup with the tables on and off
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r06f; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py::test_spmv_gather_table tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
cd /tmp && export TMPDIR=/tmp
for t in 1 0; do
AMGD_MV_TAB=$t timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_t$t -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $D/prof_t$t.json 2> $D/prof_t$t.err
rc=$?
find /tmp/prof_t$t -name "*kernel_stats.csv" -exec cp {} $D/kstats_t$t.csv \;
tail -c 3000 $D/prof_t$t.err > $D/prof_t$t.tail; rm -f $D/prof_t$t.err
echo "tab=$t rc=$rc"; tail -n 1 $D/prof_t$t.json | cut -c1-200
done
