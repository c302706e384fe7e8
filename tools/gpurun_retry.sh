# gpurun with retries while every GPU slot of the pod is busy (exit code 3 / "slot(s) ... busy")
# usage: bash tools/gpurun_retry.sh <log> <timeout> '<command>'
log=$1; to=$2; shift 2
for i in $(seq 1 15); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  if grep -q "slot(s) on this pod are busy\|no box\|no free box\|backing off\|status=transient" $log; then sleep 90; continue; fi
  exit $rc
done
exit 3
