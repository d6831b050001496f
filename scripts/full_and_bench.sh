set -u
TAG=${1:-fb}; shift; CFGS=${@:-c2}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for c in $CFGS; do
  timeout -k 10 300 python bench.py --config $c --no-e2e --no-cpu-baseline > $OUT/bench_$c.log 2>&1
  rc=$?; [ $rc -ne 0 ] && tail -5 $OUT/bench_$c.log && exit $rc
  tail -1 $OUT/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d.get('stages_ms'), d.get('roofline',{}) and d['roofline'].get('frac'))"
done
