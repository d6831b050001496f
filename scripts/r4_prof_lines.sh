#!/bin/bash
# rocprofv3 kernel-trace summaries of the C3, C4 and c2x bench commands (per-kernel times for the other decode lines)
set -u
OUT=gpurun_out/r4pl; mkdir -p $OUT; export TMPDIR=/tmp
for c in c3 c4 c2x; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- \
      python bench.py --config $c --no-cpu-baseline --no-e2e > $OUT/rocprof_$c.log 2>&1 || { echo "$c failed"; tail -5 $OUT/rocprof_$c.log; exit 1; }
  find $OUT/prof_$c -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_$c.csv \;
  python scripts/kstats.py $OUT/prof_$c $OUT/kernel_launches_$c.json > /dev/null
  grep '^{' $OUT/rocprof_$c.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['stages_ms'])"
  head -4 $OUT/kernel_stats_$c.csv | cut -c1-120
done
