# bench N=2 rehearsal (host transport, both ranks on the one GPU), configs[2] full size, aniso logs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --transport host --edge 96 --steps 2 --warmup 1 > gpurun_out/bench_n2host.json 2> gpurun_out/bench_n2host.err
rc=$?; echo "bench n2 host rc=$rc"; cat gpurun_out/bench_n2host.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/bench_n2host.err; exit $rc; }
LIM=400 bash tools/gpurun_cfg.sh sem10k || exit $?
AMGD_FSLOG=1 timeout -k 10 200 python3 tools/probe_scale.py 256 > gpurun_out/fslog256.out 2> gpurun_out/fslog256.err; echo "fslog rc=$?"
AMGD_SGLOG=1 timeout -k 10 200 python3 -u tools/probe_configs.py aniso128 > gpurun_out/aniso128_sglog.json 2> gpurun_out/aniso128_sglog.err; echo "sglog rc=$?"
LIM=500 bash tools/gpurun_cfg.sh aniso256
