#!/bin/bash
# tools/all_counters.sh TAG -- SQ instruction/stall counters and HBM traffic (FETCH_SIZE, WRITE_SIZE)
# of the codec kernels for every BASELINE GPU config, one rocprofv3 --pmc pass per counter group.
# Usage (GPU box, repo root): bash tools/all_counters.sh r02
set -u
TAG=${1:-all}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/ctr_${TAG}
export TMPDIR=/tmp
declare -A CFG
CFG[3d_f32_256_r8]="--dims 3 --size 256 --rate 8"
CFG[3d_f64_256_r16]="--dims 3 --size 256 --rate 16 --dtype float64"
CFG[2d_f32_8192_r2]="--dims 2 --size 8192 --rate 2"
CFG[1d_f32_1M_r8]="--dims 1 --size 1048576 --rate 8"
CFG[3d_f32_1024_r8]="--dims 3 --size 1024 --rate 8 --reps 2"
for name in 3d_f32_256_r8 3d_f64_256_r16 2d_f32_8192_r2 1d_f32_1M_r8 3d_f32_1024_r8; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/$name/g$i" -o run -- \
      python tools/kernel_probe.py ${CFG[$name]} > /dev/null 2>&1
    rc=$?; echo "[$name g$i] exit $rc"; [ $rc -ne 0 ] && exit $rc
  done
  echo "== $name"; python tools/counters.py "$OUT/$name"
done
