# kernel stats of one 256^3 setup: default, byte-map symbolic windows, 2048-wide numeric windows
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04t
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
for v in mvxcd default; do
  case $v in default) E="";; sb0) E="AMGD_SG_SYMBITS=0";; ww2048) E="AMGD_SG_WW=2048";; ww512) E="AMGD_SG_WW=512";; per8) E="AMGD_SL_PER4=8";; per4) E="AMGD_SL_PER4=4";; p16_8) E="AMGD_SL_PER16=8";; rw4all) E="AMGD_SL_RW=4";; m16_18) E="AMGD_SL_RW16_MIN=262144";; m16_20) E="AMGD_SL_RW16_MIN=1048576";; p64_8) E="AMGD_SL_PER64=8";; mid8) E="AMGD_SL_MID=8";; sort0) E="AMGD_SG_SORT=0";; sortall) E="AMGD_SG_SORT_ALL=1";; qlsort0) E="AMGD_QF_SORT=0 AMGD_LMOP_SORT=0";; fssort0) E="AMGD_FS_SORT=0";; xcd1) E="AMGD_SG_XCD=1";; p0_32) E="AMGD_SG_WIN_P0=32";; p0_64) E="AMGD_SG_WIN_P0=64";; selsort) E="AMGD_FS_SELSORT=1";; sl512) E="AMGD_SL_MIN_ROWS=512 AMGD_SL_LIST_MIN_ROWS=512";; sl1024) E="AMGD_SL_MIN_ROWS=1024 AMGD_SL_LIST_MIN_ROWS=1024";; mvxcd) E="AMGD_MV_XCD=1";; esac
  ( [ -n "$E" ] && export $E; exec timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/$v -o p -- python3 tools/probe_configs.py p7_256 > $D/$v.log 2>&1 ); r=$?; echo "$v rc=$r"; [ $r -eq 0 ] || exit 1
  f=$(find $D/$v -name "*kernel_stats.csv" | head -1); python3 tools/kstats.py $f 40 > $D/$v.top.txt; grep -E "total|spmv" $D/$v.top.txt; grep -o '"setup_s": [0-9.]*' $D/$v.log || true
  find $D/$v -name "*kernel_trace.csv" -delete
done
