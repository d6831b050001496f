#!/bin/bash
# One bench line per config (no CPU baseline / e2e unless asked): scripts/bench_cfgs.sh <tag> <cfg...>
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 300 python bench.py --config "$c" --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/$c.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && echo "$c rc=$rc" && tail -5 "$OUT/$c.log" && exit $rc
  tail -1 "$OUT/$c.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], 'GiB/s', d['stages_ms'], 'frac', d['roofline']['frac'])"
done
