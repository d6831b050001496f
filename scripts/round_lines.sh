#!/bin/bash
# Round evidence, the other bench lines (each decode config with its own live PMC traffic).
# usage: scripts/round_lines.sh <tag> "<configs>"
set -u
TAG=$1; CFGS=$2; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in $CFGS; do
    echo "== bench_$c ($(date +%T))"
    timeout -k 10 600 python bench.py --config $c > "$OUT/bench_$c.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench_$c rc=$rc"; tail -5 "$OUT/bench_$c.log"; exit $rc; }
    grep '^{' "$OUT/bench_$c.log" > "$OUT/bench_$c.json" || true
    python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); r=d.get('roofline') or {}; print('$c', d['metric'][:40], d['value'], d.get('stages_ms'), r.get('frac'), r.get('traffic'))"
done
