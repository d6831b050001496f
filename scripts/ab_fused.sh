#!/bin/bash
# The fused walk (look-back placement, RIO_FUSED=1, default) on one box: the whole GPU suite first,
# then interleaved bench lines against the two-launch scan (RIO_FUSED=0).
# usage: scripts/ab_fused.sh <tag> [configs] [skip-tests]
set -u
TAG=$1; CFGS=${2:-"c3 c2"}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "${3:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
  for c in $CFGS; do
    for f in 1 0; do
      RIO_FUSED=$f timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/b_${c}_f${f}_$r.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $c fused=$f rc=$rc"; tail -5 "$OUT/b_${c}_f${f}_$r.log"; exit $rc; }
      grep '^{' "$OUT/b_${c}_f${f}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c fused=$f', d['value'], d['stages_ms'])"
    done
  done
done
