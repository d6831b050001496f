#!/bin/bash
# bench lines of the current tree (device decode only: no CPU baseline, no e2e). usage: r4_lines.sh <tag> "<configs>"
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in $2; do
    echo "== bench_$c ($(date +%T))"
    timeout -k 10 600 python bench.py --config $c --no-cpu-baseline --no-e2e > "$OUT/bench_$c.log" 2>&1 || { echo "bench_$c failed"; tail -5 "$OUT/bench_$c.log"; exit 1; }
    grep '^{' "$OUT/bench_$c.log" > "$OUT/bench_$c.json" || true
    python -c "
import json
d = json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1])
print('$c', d['value'], d.get('stages_ms') or d.get('stages_ms_per_table'))"
done
