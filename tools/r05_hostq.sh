set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
for n in 0 1 2 3 4 5; do
  CUZFP_HOST_DEBUG=1 timeout -k 10 120 python tools/hostpath_probe.py --streams $n > $OUT/hqc_$n.txt 2>&1 || { tail $OUT/hqc_$n.txt; exit 1; }
  echo "== $n before: $(grep -c 'host queues' $OUT/hqc_$n.txt) trials; $(grep fresh $OUT/hqc_$n.txt | cut -c1-140)"
done
