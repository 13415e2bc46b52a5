#!/bin/bash
# gpurun with waits for the pool: re-submits ONLY when gpurun reports that nothing ran (no box / slot
# free, box lost while being prepared, back-off); any run that started — pass or fail — is final.
#   bash tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|no free box\|slot(s) on this pod are busy" "$LOG" && ! grep -q "status=ok\|status=fail" "$LOG"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
