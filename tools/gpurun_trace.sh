# rocprofv3 kernel trace (per-launch durations kept) + SGLOG of one 256^3 setup
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
rm -rf gpurun_out/trace256; mkdir -p gpurun_out/trace256
cd /tmp && export TMPDIR=/tmp
AMGD_SGLOG=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/trace256 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_scale.py 256 > $GRAFT_REPO_ROOT/gpurun_out/trace256.log 2>&1; rc=$?
echo "prof rc=$rc"
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/trace256/run_kernel_trace.csv')))
print(len(rows), 'launches')
with open('gpurun_out/trace256/launches.txt', 'w') as f:
    for r in rows:
        f.write(f"{int(r['End_Timestamp']) - int(r['Start_Timestamp'])} {r['Start_Timestamp']} {r['Kernel_Name'][:90]}\n")
PY
rm -f gpurun_out/trace256/run_kernel_trace.csv
exit $rc
