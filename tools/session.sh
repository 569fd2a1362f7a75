#!/bin/bash
# tools/session.sh TAG STEPS... -- one GPU-box session:
# xvar A/B timing of kernel variants, the launch-overhead probe, GPU tests,
# bench, rocprofv3 stats / counters.  Every GPU step runs under its own time
# limit; a crash / abort / timeout ends the session at once (pytest's exit 1,
# "tests failed", is reported and also ends it).
set -u
TAG=${1:-r06}
shift || true
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_on() {  # $1 = rc, $2 = step name
  echo "[$2] exit $1"
  if [ "$1" -ne 0 ]; then echo "[$2] failed: stopping"; exit "$1"; fi
}
for s in "$@"; do
  case $s in
    xvar:*)  # xvar:v1,v2,...[:field]
      IFS=: read -r _ names field <<< "$s"
      timeout -k 10 600 python tools/xvar.py run --field ${field:-polynomial,splitmix} ${names//,/ } > "$OUT/xvar_${TAG}.txt" 2>&1
      stop_on $? xvar; cat "$OUT/xvar_${TAG}.txt" ;;
    xvar64:*)
      IFS=: read -r _ names <<< "$s"
      timeout -k 10 600 python tools/xvar.py run --dtype float64 --rate 16 ${names//,/ } > "$OUT/xvar64_${TAG}.txt" 2>&1
      stop_on $? xvar64; cat "$OUT/xvar64_${TAG}.txt" ;;
    hostsweep)
      timeout -k 10 300 python tools/host_sweep.py > "$OUT/host_sweep_${TAG}.txt" 2>&1
      stop_on $? hostsweep; cat "$OUT/host_sweep_${TAG}.txt" ;;
    stamps:*)  # stamps:LIB[:field] -- build/probe/LIB, 3D f32 256^3 r8, two launches back to back
      IFS=: read -r _ lib field <<< "$s"
      timeout -k 10 300 python tools/probe.py stamps --lib $lib --field ${field:-polynomial} --back 2 > "$OUT/stamps_${lib}_${TAG}.txt" 2>&1
      stop_on $? stamps; cat "$OUT/stamps_${lib}_${TAG}.txt" ;;
    copychunks)
      timeout -k 10 300 python tools/copy_chunks.py > "$OUT/copy_chunks_${TAG}.txt" 2>&1
      stop_on $? copychunks; cat "$OUT/copy_chunks_${TAG}.txt" ;;
    ranges)
      timeout -k 10 120 python tools/zero_copy.py --ranges > "$OUT/ranges_${TAG}.txt" 2>&1
      stop_on $? ranges; cat "$OUT/ranges_${TAG}.txt" ;;
    hosttrace)
      rm -rf "$OUT/htrace_${TAG}"
      timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/htrace_${TAG}" -o run -- \
        python tools/host_trace.py > "$OUT/htrace_${TAG}.log" 2>&1
      stop_on $? hosttrace
      python tools/host_trace.py --analyse "$OUT/htrace_${TAG}" > "$OUT/htrace_${TAG}.txt" 2>&1; head -80 "$OUT/htrace_${TAG}.txt" ;;
    zerocopy)
      timeout -k 10 300 python tools/zero_copy.py > "$OUT/zero_copy_${TAG}.txt" 2>&1
      stop_on $? zerocopy; cat "$OUT/zero_copy_${TAG}.txt" ;;
    stamps64)
      timeout -k 10 300 python tools/probe.py stamps --lib p9 --dtype float64 --rate 16 --back 2 > "$OUT/stamps64_${TAG}.txt" 2>&1
      stop_on $? stamps64; cat "$OUT/stamps64_${TAG}.txt" ;;
    launch)
      timeout -k 10 300 python tools/launch_overhead.py > "$OUT/launch_${TAG}.txt" 2>&1
      stop_on $? launch; cat "$OUT/launch_${TAG}.txt" ;;
    quick)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
        -k "golden_baseline or fuzz_vs_oracle or extreme or random_streams or golden_fuzz or non_pow2 or sanity or edge_sizes or staged" > "$OUT/pytest_quick_${TAG}.log" 2>&1
      stop_on $? quick; tail -3 "$OUT/pytest_quick_${TAG}.log" ;;
    pytestk:*)  # pytestk:EXPR -- the GPU tests matching EXPR
      IFS=: read -r _ expr <<< "$s"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
        -k "$expr" > "$OUT/pytestk_${TAG}.log" 2>&1
      stop_on $? pytestk; tail -3 "$OUT/pytestk_${TAG}.log" ;;
    pytest)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_${TAG}.log" 2>&1
      stop_on $? pytest; tail -3 "$OUT/pytest_gpu_${TAG}.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_${TAG}.log" 2>&1
      stop_on $? smoke; tail -2 "$OUT/smoke_${TAG}.log" ;;
    bench)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench_${TAG}.json" 2> "$OUT/bench_${TAG}.err"
      stop_on $? bench; tail -c 1500 "$OUT/bench_${TAG}.json" ;;
    bench200)
      timeout -k 10 600 python bench.py --no-cpu-baseline --no-host-path > "$OUT/bench200_${TAG}.json" 2> "$OUT/bench200_${TAG}.err"
      stop_on $? bench200; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('value', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], d['parity'], 'c5', (d.get('config5') or {}).get('value_GBps'))" "$OUT/bench200_${TAG}.json" ;;
    benchcfg)
      timeout -k 10 300 python bench.py --dtype float64 --rate 16 --no-cpu-baseline --no-host-path --no-config5 > "$OUT/bench_f64_${TAG}.json" 2>&1
      stop_on $? bench64; tail -1 "$OUT/bench_f64_${TAG}.json" | cut -c1-700
      timeout -k 10 300 python bench.py --dims 2 --size 8192 --rate 2 --no-cpu-baseline --no-host-path --no-config5 > "$OUT/bench_2d_${TAG}.json" 2>&1
      stop_on $? bench2d; tail -1 "$OUT/bench_2d_${TAG}.json" | cut -c1-700
      timeout -k 10 300 python bench.py --dims 1 --size 1048576 --rate 8 --no-cpu-baseline --no-host-path --no-config5 > "$OUT/bench_1d_${TAG}.json" 2>&1
      stop_on $? bench1d; tail -1 "$OUT/bench_1d_${TAG}.json" | cut -c1-700 ;;
    prof)
      rm -rf "$OUT/prof_${TAG}"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}" -o run -- \
        python bench.py --steps 20 --no-cpu-baseline --no-host-path > "$OUT/prof_bench_${TAG}.json" 2>&1
      stop_on $? prof
      find "$OUT/prof_${TAG}" -name "*kernel_stats.csv" -exec head -6 {} \; ;;
    pmc)
      rm -rf "$OUT/pmc_${TAG}"
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_${TAG}/fetch" -o run -- \
        python tools/kernel_probe.py > /dev/null 2>&1
      stop_on $? pmc_fetch
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_${TAG}/write" -o run -- \
        python tools/kernel_probe.py > /dev/null 2>&1
      stop_on $? pmc_write ;;
    pmccfg)  # PMC traffic of BASELINE configs[2] (3D f64 256^3 r16) and configs[3] (2D f32 8192^2 r2)
      for cfg in "f64:--dtype float64 --rate 16" "2d:--dims 2 --size 8192 --rate 2"; do
        name=${cfg%%:*}; args=${cfg#*:}
        rm -rf "$OUT/pmc_${name}_${TAG}"
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_${name}_${TAG}/fetch" -o run -- \
          python tools/kernel_probe.py $args > /dev/null 2>&1
        stop_on $? pmccfg_${name}_fetch
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_${name}_${TAG}/write" -o run -- \
          python tools/kernel_probe.py $args > /dev/null 2>&1
        stop_on $? pmccfg_${name}_write
      done ;;
    counters)
      i=0
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
                 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
                 "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU2 SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VSKIPPED"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/ctr_${TAG}/g$i" -o run -- \
          python tools/kernel_probe.py ${PROBE_ARGS:-} > /dev/null 2>&1
        stop_on $? counters_g$i
      done
      python tools/counters.py "$OUT/ctr_${TAG}" > "$OUT/ctr_${TAG}.txt" 2>&1; cat "$OUT/ctr_${TAG}.txt" ;;
    *) echo "unknown step $s" ;;
  esac
done
