#!/bin/bash
# tools/r05_prio.sh -- the decoder priority-schedule sweep of round 5 (GPU box):
# 3D f32 (both fields), 2D f32 8192^2 r2, 1D f32 64M r8, 3D f64 r16, each
# variant interleaved twice (tools/xvar.py builds), then the chunked-copy costs.
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
f=$OUT/prio_r05.txt
: > "$f"
run() { timeout -k 10 600 python tools/xvar.py run "$@" >> "$f" 2>&1 || { echo "[xvar $*] failed"; cat "$f"; exit 1; }; }
run --field polynomial,splitmix cur pa3 pa2 pa3t25 pa3t17 pa3t13 cur pa3 pa2 pa3t25 pa3t17 pa3t13
run --dims 2 --size 8192 --rate 2 --field polynomial d2cur d2pa3 d2cur d2pa3
run --dims 1 --size 67108864 --rate 8 --field polynomial d1cur d1pa3 d1cur d1pa3
run --dtype float64 --rate 16 --field polynomial f64cur f64pa3 f64cur f64pa3
grep -v amdgpu.ids "$f"
timeout -k 10 300 python tools/copy_chunks.py > "$OUT/copy_chunks2_r05.txt" 2>&1 || { echo "[copy_chunks] failed"; exit 1; }
grep -v amdgpu.ids "$OUT/copy_chunks2_r05.txt" | tail -12
