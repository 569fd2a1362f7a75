#!/bin/bash
# tools/counters_deep.sh TAG [probe args] -- issue / stall / LDS counters of the codec kernels
# (SQ_ACTIVE_INST_VALU2 = quad-cycles with two VALU issued, WAIT_INST_*, LDS FIFO/conflicts,
# instruction fetch), one rocprofv3 --pmc pass per group of <= 8 SQ counters.
# Usage (GPU box, repo root): bash tools/counters_deep.sh r02 --dims 3 --size 256 --rate 8
set -u
TAG=${1:-deep}
shift || true
ARGS=${*:-"--dims 3 --size 256 --rate 8"}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/ctrd_${TAG}
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INSTS_BRANCH" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_CYCLES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- \
    python tools/kernel_probe.py $ARGS > /dev/null 2>&1
  rc=$?; echo "[g$i] exit $rc"; [ $rc -ne 0 ] && exit $rc
done
python tools/counters.py "$OUT"
