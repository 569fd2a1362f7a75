#!/bin/bash
# tools/prio_sweep.sh -- encode+decode step with the plane-loop priority
# schedule forced on (CUZFP_PRIO=1) / off (0) / chosen by the launcher (auto),
# by array size (3D f32 rate 8).  Run on the GPU box from the repo root.
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
for sz in ${SIZES:-192 256 320 384 512 768}; do
  for p in 1 0 auto; do
    if [ "$p" = auto ]; then unset CUZFP_PRIO; else export CUZFP_PRIO=$p; fi
    timeout -k 10 300 python bench.py --size "$sz" --steps 20 --warmup 5 --no-cpu-baseline --no-host-path \
      > "$OUT/prio_${sz}_$p.json" 2>/dev/null || { echo "size $sz prio $p failed"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['encode_ms'], d['decode_ms'], d['max_abs_err'])" \
      "$OUT/prio_${sz}_$p.json" "$sz" "$p"
  done
done
