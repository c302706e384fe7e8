# one PMC pass: tools/gpurun_pmc.sh <tag> <edge> <kernel-regex> <counters...>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=$1; M=$2; RX=$3; shift 3
rm -rf gpurun_out/pmc_$TAG; mkdir -p gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py $M > $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.log 2>&1; rc=$?
echo "pmc rc=$rc"
tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.log
ls $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
exit 0
