#!/bin/bash
# coop decoder check: parity tests with every snappy file forced onto k_snappy_coop, batch tests, benches
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
echo "== coop-forced tests ($(date +%T))"
RIO_COOP_MIN=${TCOOP:-0} timeout -k 10 900 python -u -m pytest ${2:-tests/test_gpu_parity.py tests/test_gpu_codec_errors.py tests/test_gpu_batch.py} -m gpu -q -x --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 "$OUT/tests.log"; if fatal $rc; then exit $rc; fi
for cm in ${3:-c4:16384 c2:0 c2:16384}; do
  c=${cm%%:*}; m=${cm##*:}
  echo "== bench $c coop_min=$m ($(date +%T))"
  RIO_COOP_MIN=$m timeout -k 10 400 python bench.py --config $c --no-e2e --no-cpu-baseline > "$OUT/bench_${c}_$m.log" 2>&1
  rc=$?; grep '^{' "$OUT/bench_${c}_$m.log" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','stages_ms')}, d['roofline']['frac'])" 2>/dev/null || tail -5 "$OUT/bench_${c}_$m.log"
  if fatal $rc; then exit $rc; fi
done
