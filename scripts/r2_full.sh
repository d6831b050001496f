#!/bin/bash
# full GPU suite, then bench lines (default options: cpu baseline + e2e) for the given configs
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if [ "${2:-tests}" != none ]; then
  echo "== tests ($(date +%T))"
  timeout -k 10 1000 python -u -m pytest ${2:-tests} -m gpu -q --maxfail=20 --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc"; tail -12 "$OUT/tests.log"; if fatal $rc; then exit $rc; fi
fi
for c in ${3:-c2}; do
  echo "== bench $c ($(date +%T))"
  timeout -k 10 600 python bench.py --config $c > "$OUT/bench_$c.log" 2>&1
  rc=$?; echo "rc=$rc"; grep '^{' "$OUT/bench_$c.log" | cut -c1-600 || tail -5 "$OUT/bench_$c.log"
  if fatal $rc; then exit $rc; fi
done
