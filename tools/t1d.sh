set -u
for sz in 1048576 4194304; do
  for pr in "" 0 1; do
    CUZFP_PRIO=$pr timeout -k 10 120 python bench.py --dims 1 --size $sz --rate 8 --steps 50 --warmup 10 --no-cpu-baseline --no-host-path 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($sz, 'prio=$pr', d['value'], d['encode_ms'], d['decode_ms'])" || exit 1
  done
done
