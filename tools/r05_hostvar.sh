set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config5 > $OUT/hv_bench_$i.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_path']; print('bench', d['value'], h['compress_GBps'], h['decompress_GBps'], h['link_GBps'], h['frac_of_link'])" $OUT/hv_bench_$i.json
done
timeout -k 10 300 python tools/host_sweep.py > $OUT/hv_sweep.txt 2>&1 || exit 1
grep -v amdgpu $OUT/hv_sweep.txt | tail -4
