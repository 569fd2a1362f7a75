#!/bin/bash
# tools/lds_counters.sh TAG -- LDS / issue counters of the 3D f32 codec kernels (one --pmc pass each)
set -u
TAG=${1:-lds}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/ctr_$TAG
export TMPDIR=/tmp
i=0
for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- \
    python tools/kernel_probe.py ${PROBE_ARGS:-} > /dev/null 2>&1
  rc=$?; echo "[g$i] exit $rc"; [ $rc -ne 0 ] && exit $rc
done
python tools/counters.py "$OUT"
