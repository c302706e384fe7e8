# r03 session m: k_spmv_pipe entries per lane per round (12 / 16), with 1024-column
# wave windows for the windowed SpGEMM rows, 256^3 A/B, 2 setups each
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03m4
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 700 python3 tools/ab_setup.py 256 --no-digest --reps 2 pipe=11 pipe=19 pipe=11,ww=9 pipe=19,ww=9 > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
