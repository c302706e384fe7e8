# fused selection, parallel max tracking: default-routed digests, the 128^3 digests with and
# without the fusion, a short 256^3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/amx2_$1
rm -rf $D; mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_digests.py -k "default_routing" -x -q --timeout 150 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $D/tests.log | tail -20; exit 1; }
tail -1 $D/tests.log
timeout -k 10 120 python3 tools/ab_setup.py 128 default amx=0 > $D/ab128_digest.txt 2> $D/ab128.err || { tail -5 $D/ab128.err; exit 1; }
cat $D/ab128_digest.txt
timeout -k 10 200 python3 tools/ab_setup.py 256 --no-digest default amx=0 default > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
