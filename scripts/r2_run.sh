#!/bin/bash
# One gpurun session for round-2 iteration: GPU tests (optionally a subset), then bench lines.
# usage: scripts/r2_run.sh <tag> "<pytest paths/args>" "<bench configs>"
set -u
TAG=$1; TESTS=${2:-tests}; CFGS=${3:-c2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if [ "$TESTS" != "none" ]; then
  echo "== tests ($(date +%T))"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q --maxfail=25 --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc"; tail -15 "$OUT/tests.log"
  if fatal $rc; then exit $rc; fi
fi
[ "$CFGS" = none ] && { echo done; exit 0; }
for c in $CFGS; do
  echo "== bench $c ($(date +%T))"
  timeout -k 10 300 python bench.py --config $c --no-e2e --no-cpu-baseline > "$OUT/bench_$c.log" 2>&1
  rc=$?; echo "bench $c rc=$rc"; grep '^{' "$OUT/bench_$c.log" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','stages_ms')}, d.get('roofline',{}).get('frac'))" 2>/dev/null || tail -5 "$OUT/bench_$c.log"
  if fatal $rc; then exit $rc; fi
done
echo done
