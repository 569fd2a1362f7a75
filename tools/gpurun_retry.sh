#!/bin/bash
# Submit one gpurun call, resubmitting only when the pool reports an
# infrastructure-side transient failure before anything ran (at most 10 tries).
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; shift 2
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient\|no box or slot free\|backing off" "$log" && ! grep -q "status=ok\|status=fail" "$log"; then
    sleep 60
    continue
  fi
  exit $rc
done
exit $rc
