# r03 session m: wave-window widths: symbolic byte windows 2048 / 4096 columns, numeric
# 512 / 1024 columns; 256^3 A/B, 2 setups each
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r03m6
mkdir -p $D
export PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 150 --timeout-method thread -k "wave_windows" > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 1; }
tail -2 $D/t.log
timeout -k 10 700 python3 tools/ab_setup.py 256 --no-digest --reps 2 ww=27 ww=43 ww=91 ww=75 > $D/ab256.txt 2> $D/ab256.err || { tail -5 $D/ab256.err; cat $D/ab256.txt; exit 1; }
cat $D/ab256.txt
