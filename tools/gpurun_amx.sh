# fused find_support selection: digests (default routing) + SpMV kernel tests, the 128^3
# hierarchy digests with the fused and the separate selection, an interleaved 256^3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/amx_$1
rm -rf $D; mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_digests.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $D/tests.log | tail -30; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python3 tools/ab_setup.py 128 default amx=0 > $D/ab128_digest.txt 2> $D/ab128.err || { tail -5 $D/ab128.err; exit 1; }
cat $D/ab128_digest.txt
timeout -k 10 600 python3 tools/ab_setup.py 256 --no-digest default amx=0 default amx=0 > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
