set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
export TMPDIR=/tmp
for n in 0 2; do
  rm -rf $OUT/ht2_$n
  CUZFP_HOST_DEBUG=1 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/ht2_$n -o run -- \
    python tools/host_trace.py --streams $n > $OUT/ht2_$n.log 2>&1 || { tail -20 $OUT/ht2_$n.log; exit 1; }
  echo "== streams before: $n"; grep "host queues" $OUT/ht2_$n.log | head -12
  python tools/host_trace.py --analyse $OUT/ht2_$n > $OUT/ht2_$n.txt 2>&1; tail -24 $OUT/ht2_$n.txt
done
