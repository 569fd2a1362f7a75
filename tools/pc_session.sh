#!/bin/bash
# tools/pc_session.sh TAG [probe args] -- rocprofv3 stochastic PC sampling of the
# codec kernels (tools/kernel_probe.py), summarised by tools/pcsample.py.
# Every GPU step has its own time limit and the session stops at the first failure.
# Usage (GPU box, repo root): bash tools/pc_session.sh r05 --dims 3 --size 256 --rate 8
set -u
TAG=${1:-pc}
shift || true
ARGS=${*:-"--dims 3 --size 256 --rate 8"}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
UNIT=${PC_UNIT:-cycles}
IVAL=${PC_INTERVAL:-4096}
timeout -k 10 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
  --pc-sampling-unit "$UNIT" --pc-sampling-interval "$IVAL" --kernel-trace \
  --output-format csv -d "$OUT/raw" -o run -- python tools/kernel_probe.py $ARGS --reps ${PC_REPS:-3} > "$OUT/run.log" 2>&1
rc=$?
echo "[pcsample] exit $rc"
if [ $rc -ne 0 ]; then tail -30 "$OUT/run.log"; exit $rc; fi
python tools/pcsample.py "$OUT/raw" --top 60 > "$OUT/summary.txt" 2>&1
echo "[summary] exit $?"
# keep the raw csv small enough to travel back
find "$OUT/raw" -name "*pc_sampling*.csv" -size +20M -exec gzip -f {} \;
head -c 20000 "$OUT/summary.txt"
