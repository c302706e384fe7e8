# kernel tests of a change, the hierarchy digests of its settings at 128^3 (must be
# identical), and an interleaved 256^3 A/B.  usage: bash tools/gpurun_abq.sh <tag> <pytest -k> SETTING...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; K=$2; shift 2
D=gpurun_out/abq_$TAG
rm -rf $D; mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -k "$K" -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $D/tests.log | tail -30; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python3 tools/ab_setup.py 128 default "$@" > $D/ab128_digest.txt 2> $D/ab128.err || { tail -5 $D/ab128.err; exit 1; }
cat $D/ab128_digest.txt
timeout -k 10 900 python3 tools/ab_setup.py 256 --no-digest default "$@" default "$@" > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
