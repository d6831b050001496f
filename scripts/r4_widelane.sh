#!/bin/bash
set -u
OUT=gpurun_out/r4wl; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/test_gpu_wide.py > $OUT/tests_wide.log 2>&1
rc=$?; tail -3 $OUT/tests_wide.log; [ $rc -ne 0 ] && exit $rc
for c in c2x c2 c3 c4; do
  timeout -k 10 400 python bench.py --config $c --no-e2e > $OUT/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $OUT/bench_$c.log; exit 1; }
  grep '^{' $OUT/bench_$c.log > $OUT/bench_$c.json
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['stages_ms'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
done
