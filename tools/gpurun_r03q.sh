# r03 session q: configs[4] (anisotropic 256^3) with the round-3 kernels on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03q
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 600 python3 tools/ab_setup.py 256 --eps 1e-3 --no-digest default ww=0 pipe=0 > $D/ab_aniso.txt 2> $D/ab_aniso.err || { tail -5 $D/ab_aniso.err; cat $D/ab_aniso.txt; exit 1; }
cat $D/ab_aniso.txt
