# r03 session t: interleaved no-digest A/B: k_spmv_chunk for moderate rows (chunk=1), the
# thread-per-row lmop pull (lsm=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03t
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 700 python3 tools/ab_setup.py 256 --no-digest default lsm=1 chunk=1 default lsm=1 chunk=1 default > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
