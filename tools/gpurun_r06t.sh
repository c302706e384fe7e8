# round 6: A/B of the sorted dense SpGEMM rows on configs[1] and configs[4]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06t}; mkdir -p $D
timeout -k 10 400 python3 -u tools/ab_setup.py 256 drs=0 drs=1 > $D/ab256.txt 2>&1 || { tail -5 $D/ab256.txt; exit 1; }
grep setting $D/ab256.txt
timeout -k 10 400 python3 -u tools/ab_setup.py 256 drs=0 drs=1 --eps 1e-3 > $D/ab256an.txt 2>&1 || { tail -5 $D/ab256an.txt; exit 1; }
grep setting $D/ab256an.txt
