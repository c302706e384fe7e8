# lane SpMV with / without nontemporal matrix loads: micro-benchmark, then one bench setup with NT
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u tools/spmv_bench.py > gpurun_out/spmv_nt0.txt 2>&1 || exit 1
AMGD_SPMV_NT=1 timeout -k 10 300 python3 -u tools/spmv_bench.py > gpurun_out/spmv_nt1.txt 2>&1 || exit 1
paste -d'\n' gpurun_out/spmv_nt0.txt gpurun_out/spmv_nt1.txt | grep "x=1" | head -24
AMGD_SPMV_NT=1 timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bench_nt1.json 2> gpurun_out/bench_nt1.err || exit 1
cut -c1-420 gpurun_out/bench_nt1.json
