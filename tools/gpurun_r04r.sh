# mpm with LDS-staged searches: kernel tests, then kernel stats of one 256^3 setup
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04r
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k "mpm or spgemm" --timeout 120 --timeout-method thread > $D/kern.log 2>&1; r=$?; echo "kernel tests rc=$r"; tail -3 $D/kern.log; [ $r -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o p -- python3 tools/probe_configs.py p7_256 > $D/probe.log 2>&1; r=$?; echo "probe rc=$r"; [ $r -eq 0 ] || exit 1
f=$(find $D/prof -name "*kernel_stats.csv" | head -1); python3 tools/kstats.py $f 40 > $D/top.txt; grep -E "total|mpm|wwin" $D/top.txt; grep -o '"setup_s": [0-9.]*' $D/probe.log || true
find $D/prof -name "*kernel_trace.csv" -delete
