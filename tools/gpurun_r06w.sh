# round 6: interleaved A/B (no pauses) of the incremental constraint pattern; configs[4] timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06w}; mkdir -p $D
timeout -k 10 500 python3 -u tools/ab_setup.py 256 spat=0 spat=1 spat=0 spat=1 spat=0 spat=1 --no-digest > $D/ab256.txt 2>&1 || { tail -5 $D/ab256.txt; exit 1; }
grep setting $D/ab256.txt
PROBE_BEAT=0 timeout -k 10 300 python3 tools/probe_configs.py aniso256 > $D/aniso.json 2> $D/aniso.err || { tail -5 $D/aniso.err; exit 1; }
tail -n 1 $D/aniso.json | cut -c1-200
