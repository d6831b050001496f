#!/bin/bash
# e2e (PCIe-inclusive) A/B of the host copy thread count (RIO_COPY_THREADS) on C2, alternating runs
set -u
OUT=gpurun_out/r4e2e; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do
  for t in 8 16 4; do
    RIO_COPY_THREADS=$t timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/e2e_t${t}_$r.log" 2>&1 || { echo "t=$t failed"; tail -3 "$OUT/e2e_t${t}_$r.log"; exit 1; }
    grep '^{' "$OUT/e2e_t${t}_$r.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['e2e']
print('threads=$t', e['GiBps_input'], {k:v['GiBps_input'] for k,v in e['windowed'].items()}, 'file', e['from_file_page_cache_128MiB']['GiBps_input'], 'one_shot', e['one_shot']['GiBps_input'])"
  done
done
