# interleaved A/B of kernel-choice settings on one 256^3 problem (tools/ab_setup.py; no
# digest pauses between settings -- they change the GPU's sustained clocks).
# usage: bash tools/gpurun_ab.sh <tag> SETTING...   e.g. default ww=0 default ww=0
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
D=gpurun_out/ab_$TAG
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 1000 python3 tools/ab_setup.py 256 --no-digest "$@" > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
