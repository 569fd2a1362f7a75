#!/bin/bash
# tools/probe_session.sh -- design-experiment GPU session (xvar timings, extra counters).
#   bash tools/probe_session.sh TAG "VARIANTS" ["COUNTER GROUP" ...]
# Every GPU step has its own time limit; a crash / abort / timeout ends the session.
set -u
TAG=$1
VARS=$2
shift 2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_bad() {  # $1 = rc, $2 = step
  echo "[$2] exit $1"
  case $1 in 0) ;; 124|134|137|139) echo "[$2] abnormal: stopping"; exit "$1" ;; *) ;; esac
}
if [ -n "$VARS" ]; then
  timeout -k 10 600 python tools/xvar.py run $VARS > "$OUT/xv_$TAG.txt" 2>&1
  stop_if_bad $? xvar
  cat "$OUT/xv_$TAG.txt"
fi
i=0
for grp in "$@"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/ctr_$TAG/g$i" -o run -- \
    python tools/kernel_probe.py ${PROBE_ARGS:-} > "$OUT/ctr_${TAG}_g$i.log" 2>&1
  stop_if_bad $? "ctr g$i ($grp)"
done
[ $i -gt 0 ] && python tools/counters.py "$OUT/ctr_$TAG" > "$OUT/ctr_$TAG.txt" 2>&1 && cat "$OUT/ctr_$TAG.txt"
exit 0
