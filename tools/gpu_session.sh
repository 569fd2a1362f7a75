#!/bin/bash
# tools/gpu_session.sh -- one GPU-box session: parity tests, bench, rocprofv3.
# Every GPU step has its own time limit; a crash / abort / timeout (exit codes
# other than 0 and pytest's 1 = "tests failed") ends the session at once.
# Usage (from the repo root on the box):  bash tools/gpu_session.sh [tag] [steps...]
set -u
TAG=${1:-run}
shift || true
STEPS=${*:-"pytest bench prof"}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
ok_or_stop() {  # $1 = rc, $2 = step name
  local rc=$1
  echo "[$2] exit $rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[$2] abnormal exit: stopping"; exit "$rc"; fi
}
for s in $STEPS; do
  case $s in
    pytest)
      timeout -k 10 1200 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
      ok_or_stop $? pytest; tail -5 "$OUT/pytest_gpu_$TAG.log" ;;
    quick)
      # the parity subset that exercises every coder path (golden BASELINE streams, fuzz, extremes, random streams)
      timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "golden_baseline or fuzz_vs_oracle or extreme or random_streams or golden_fuzz" > "$OUT/pytest_quick_$TAG.log" 2>&1
      ok_or_stop $? quick; tail -3 "$OUT/pytest_quick_$TAG.log" ;;
    g1024)
      # BASELINE configs[4] parity: the whole 1024^3 array and its slabs against the reference's hashes
      timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "1024" > "$OUT/pytest_1024_$TAG.log" 2>&1
      ok_or_stop $? g1024; tail -3 "$OUT/pytest_1024_$TAG.log" ;;
    stepgap)
      timeout -k 10 300 python tools/step_gap.py > "$OUT/stepgap_$TAG.txt" 2>&1
      ok_or_stop $? stepgap; cat "$OUT/stepgap_$TAG.txt" ;;
    benchq)
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-path > "$OUT/benchq_$TAG.json" 2> "$OUT/benchq_$TAG.err"
      ok_or_stop $? benchq; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('value', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], d['parity'])" "$OUT/benchq_$TAG.json" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
      ok_or_stop $? smoke; tail -2 "$OUT/smoke_$TAG.log" ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
      ok_or_stop $? bench; cat "$OUT/bench_$TAG.json" ;;
    benchsplit)
      timeout -k 10 300 python bench.py --field splitmix --no-cpu-baseline --no-host-path > "$OUT/bench_splitmix_$TAG.json" 2>&1
      ok_or_stop $? benchsplit; cat "$OUT/bench_splitmix_$TAG.json" ;;
    bench64)
      timeout -k 10 300 python bench.py --dtype float64 --rate 16 --no-cpu-baseline --no-host-path > "$OUT/bench_f64_$TAG.json" 2>&1
      ok_or_stop $? bench64; cat "$OUT/bench_f64_$TAG.json" ;;
    prof)
      rm -rf "$OUT/prof_$TAG"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
        python bench.py --steps 20 --no-cpu-baseline --no-host-path > "$OUT/prof_bench_$TAG.json" 2>&1
      ok_or_stop $? prof
      find "$OUT/prof_$TAG" -name "*kernel_stats.csv" -exec head -8 {} \; ;;
    pmc)
      rm -rf "$OUT/pmc_$TAG"
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$TAG/fetch" -o run -- \
        python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > /dev/null 2>&1
      ok_or_stop $? pmc_fetch
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$TAG/write" -o run -- \
        python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > /dev/null 2>&1
      ok_or_stop $? pmc_write ;;
    counters)
      # instruction mix / stall counters of the codec kernels (one --pmc pass per group)
      i=0
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" "SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT"; do
        i=$((i+1))
        timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/ctr_$TAG/g$i" -o run -- \
          python tools/kernel_probe.py ${PROBE_ARGS:-} > /dev/null 2>&1
        ok_or_stop $? counters_g$i
      done ;;
    icache)
      # instruction-cache behaviour of the codec kernels (one --pmc pass, SQ block)
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQC_ICACHE_INPUT_VALID_READYB SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d "$OUT/ic_$TAG" -o run -- \
        python tools/kernel_probe.py ${PROBE_ARGS:-} > /dev/null 2>&1
      ok_or_stop $? icache ;;
    configs)
      # the other BASELINE configs: 2D f32 8192^2 rate 2, 1D f32 1M rate 8 (and 1D 64M)
      timeout -k 10 300 python bench.py --dims 2 --size 8192 --rate 2 --no-cpu-baseline --no-host-path > "$OUT/bench_2d_$TAG.json" 2>&1
      ok_or_stop $? bench2d; tail -1 "$OUT/bench_2d_$TAG.json" | cut -c1-900
      timeout -k 10 300 python bench.py --dims 1 --size 1048576 --rate 8 --no-cpu-baseline --no-host-path > "$OUT/bench_1d_$TAG.json" 2>&1
      ok_or_stop $? bench1d; tail -1 "$OUT/bench_1d_$TAG.json" | cut -c1-900
      timeout -k 10 300 python bench.py --dims 1 --size 67108864 --rate 8 --no-cpu-baseline --no-host-path > "$OUT/bench_1dL_$TAG.json" 2>&1
      ok_or_stop $? bench1dL; tail -1 "$OUT/bench_1dL_$TAG.json" | cut -c1-900 ;;
    sizes)
      # throughput vs problem size (rounds of resident waves): 128^3 .. 512^3
      for sz in 128 192 256 384 512; do
        timeout -k 10 300 python bench.py --size $sz --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > "$OUT/bench_size${sz}_$TAG.json" 2>&1
        ok_or_stop $? size$sz
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print($sz, d['value'], d['encode_ms'], d['decode_ms'])" "$OUT/bench_size${sz}_$TAG.json"
      done ;;
    stamps)
      # per-wave phase timestamps (s_memtime) of the diagnostic build
      timeout -k 10 300 python tools/probe.py stamps --back 4 > "$OUT/stamps_$TAG.log" 2>&1
      ok_or_stop $? stamps
      timeout -k 10 300 python tools/probe.py stamps --back 4 --field splitmix >> "$OUT/stamps_$TAG.log" 2>&1
      ok_or_stop $? stamps_split
      timeout -k 10 300 python tools/probe.py stamps --back 4 --size 512 >> "$OUT/stamps_$TAG.log" 2>&1
      ok_or_stop $? stamps_512; cat "$OUT/stamps_$TAG.log" ;;
    probe)
      # phase costs: product kernels vs no plane coder vs no transpose (tools/probe.py)
      timeout -k 10 600 python tools/probe.py run > "$OUT/probe_$TAG.log" 2>&1
      ok_or_stop $? probe
      timeout -k 10 600 python tools/probe.py run --field splitmix >> "$OUT/probe_$TAG.log" 2>&1
      ok_or_stop $? probe_split; cat "$OUT/probe_$TAG.log" ;;
    *) echo "unknown step $s" ;;
  esac
done
