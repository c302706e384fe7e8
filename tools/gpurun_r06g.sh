# round 6: per-product SpMV times (AMGD_MVLOG=1: one synced line per whole-matrix product)
# of one 256^3 setup with the gather tables on and off
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r06g; mkdir -p $D
for t in 1 0; do
AMGD_MV_TAB=$t AMGD_MVLOG=1 timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $D/mv_t$t.json 2> $D/mv_t$t.err || { tail -5 $D/mv_t$t.err; exit 1; }
grep "^spmv" $D/mv_t$t.err | gzip > $D/mv_t$t.txt.gz; rm -f $D/mv_t$t.err
done
ls -la $D
