# round 6: A/B of the incremental constraint pattern on configs[1] and configs[4]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06r}; mkdir -p $D
timeout -k 10 500 python3 -u tools/ab_setup.py 256 spat=0 spat=1 --reps 2 > $D/ab256.txt 2>&1 || { tail -5 $D/ab256.txt; exit 1; }
tail -8 $D/ab256.txt
