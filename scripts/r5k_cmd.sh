#!/bin/bash
# Round 5: C4's memory streams on the current tree (timing-only builds), the C4 / C2 / C3 lines with live PMC traffic.
set -u
mkdir -p gpurun_out/r5k
scripts/ab_timing.sh r5k_mem "mem1 mem2 mem3" "c4" 1 || exit 1
for c in c4 c2 c3; do
  timeout -k 10 600 python bench.py --config $c --no-e2e > gpurun_out/r5k/bench_$c.log 2>&1; echo $c rc=$?
  grep '^{' gpurun_out/r5k/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', d['value'], d['stages_ms'], r['frac'], r['traffic'], r.get('traffic_read'), r.get('traffic_write'))"
done
