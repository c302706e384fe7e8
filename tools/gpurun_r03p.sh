# r03 session p: per-level phase profile of a 256^3 setup, and BASELINE configs[2] (SEM
# N=7, 10164 hexes) / configs[4] (anisotropic 256^3) on the r03n kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03p
mkdir -p $D
export PYTHONPATH=$PWD
AMGD_PHASES=1 timeout -k 10 300 python3 -u tools/probe_scale.py 256 > $D/phases256.log 2>&1 || { tail -20 $D/phases256.log; exit 1; }
tail -30 $D/phases256.log
timeout -k 10 200 python3 -u tools/probe_configs.py sem10k > $D/cfg_sem10k.json 2> $D/cfg_sem10k.err || { tail -5 $D/cfg_sem10k.err; exit 1; }
tail -1 $D/cfg_sem10k.json
timeout -k 10 300 python3 -u tools/probe_configs.py aniso256 > $D/cfg_aniso256.json 2> $D/cfg_aniso256.err || { tail -5 $D/cfg_aniso256.err; exit 1; }
tail -1 $D/cfg_aniso256.json
