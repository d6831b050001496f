# The 512-byte lane-walk tier on its own: parity subset (lane walk, wide files, parity), then the c2 / c2x lines.
set -u
OUT=gpurun_out/r5bf; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_walk_lane.py tests/test_gpu_wide.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && exit $rc
for c in c2 c2x; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --no-e2e --traffic none > $OUT/b_$c.log 2>&1 || exit $?
  grep '^{' $OUT/b_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['stages_ms'], d.get('verified'))"
done
