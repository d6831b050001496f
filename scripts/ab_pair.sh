#!/bin/bash
# Two-wave decoder (RIO_SNAPPY_PAIR=1) against the one-wave decoder on one box: parity tests on the
# pair path first, then interleaved bench lines. usage: scripts/ab_pair.sh <tag> [configs] [tests]
set -u
TAG=$1; CFGS=${2:-"c2 c3 c4"}; TESTS=${3:-"tests/test_gpu_parity.py tests/test_gpu_codec_errors.py tests/test_gpu_batch.py"}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ "$TESTS" != "none" ]; then
  RIO_SNAPPY_PAIR=1 timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests_pair.log" 2>&1
  rc=$?; tail -3 "$OUT/tests_pair.log"; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
  for c in $CFGS; do
    for p in 0 1; do
      RIO_SNAPPY_PAIR=$p timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/b_${c}_p${p}_$r.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $c pair=$p rc=$rc"; tail -5 "$OUT/b_${c}_p${p}_$r.log"; exit $rc; }
      grep '^{' "$OUT/b_${c}_p${p}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c pair=$p', d['value'], d['stages_ms'])"
    done
  done
done
