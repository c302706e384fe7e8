# round 6 close: PMC traffic of the roofline kernels + kernel summary (gpurun_pmc.sh), then
# the driver's bench command (fewer steps) reading that traffic file, then configs[4]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
TAG=${TAG:-r06y}
bash tools/gpurun_pmc.sh $TAG || exit 1
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
cp $D/traffic_$TAG.json profiles/r06/traffic_$TAG.json
t0=$(date +%s)
timeout -k 10 400 python3 bench.py --gpus 1 --steps 4 --warmup 1 > $D/bench.json 2> $D/bench.err || { echo bench failed; tail -20 $D/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
tail -n 1 $D/bench.json | cut -c1-400
PROBE_BEAT=0 timeout -k 10 300 python3 tools/probe_configs.py aniso256 > $D/aniso.json 2> $D/aniso.err || { tail -5 $D/aniso.err; exit 1; }
tail -n 1 $D/aniso.json | cut -c1-200
