#!/bin/bash
set -u
OUT=gpurun_out/r4wl3; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/test_gpu_wide.py -k "span_past" > $OUT/tests_span.log 2>&1
rc=$?; tail -3 $OUT/tests_span.log; [ $rc -ne 0 ] && exit $rc
RIO_COOP_MIN=0 timeout -k 10 400 python bench.py --config c2x --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_c2x_coop.log 2>&1 || exit 1
grep '^{' $OUT/bench_c2x_coop.log > $OUT/bench_c2x_coop.json
python3 -c "
import json; d=json.loads(open('$OUT/bench_c2x_coop.json').read().strip().splitlines()[-1])
print('c2x coop (the pre-round-4 path for files past 4 GiB)', d['value'], d['stages_ms'])"
