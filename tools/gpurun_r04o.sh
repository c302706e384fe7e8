# partition tests incl. 8 ranks and p7_64
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04o
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_partition.py -m gpu -v --durations=30 --timeout 300 --timeout-method thread > $D/parttests.log 2>&1; r=$?; echo "part tests rc=$r"; grep -E "PASSED|FAILED|passed|failed" $D/parttests.log | tail -30
[ $r -eq 0 ] || { grep -E "omp_amg_amd|rank [0-9] rc|Error" $D/parttests.log | head -30; exit 1; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_crs.py -m gpu -q --timeout 120 --timeout-method thread > $D/crs.log 2>&1; r=$?; echo "crs tests rc=$r"; tail -3 $D/crs.log; [ $r -eq 0 ] || exit 1
timeout -k 10 400 python3 -u tools/probe_configs.py p27_56 > $D/p27.json 2> $D/p27.err; echo "p27 rc=$?"; cat $D/p27.json | cut -c1-600
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D/kt -o kt -- python3 tools/probe_configs.py p7_256 > $D/kt.log 2>&1; echo "ktrace rc=$?"
f=$(find $D/kt -name "*kernel_trace.csv" | head -1); echo "trace $f"; [ -n "$f" ] && python3 tools/ktrace_gaps.py $f 1.0 > $D/ktgaps.txt && head -8 $D/ktgaps.txt && gzip $f
