# r03 session s2: no-digest, interleaved A/B (the digest pause between settings lets the
# next setups run ~0.8 s faster, so digest-separated settings are not comparable):
# find_support SUM2 on/off, the thread-per-row lmop pull
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03s2
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 700 python3 tools/ab_setup.py 256 --no-digest --reps 2 sum2=0 default lsm=1 sum2=0 default > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
