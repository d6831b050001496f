#!/bin/bash
# The windowed e2e path from a page-locked host image (rio_host_register) beside the staged one:
# the stream tests, then bench lines whose e2e object holds both.
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/stream_tests.log 2>&1
rc=$?; tail -2 $OUT/stream_tests.log; [ $rc -ne 0 ] && exit $rc
for c in ${CFGS:-c2 c2 c3}; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $OUT/b_$c.log 2>&1 || exit 1
  grep '^{' $OUT/b_$c.log | tee -a $OUT/lines.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['e2e']; print('$c', d['value'], 'staged128', e['GiBps_input'], {k: v['GiBps_input'] for k, v in e['windowed'].items()}, 'registered', {k: v['GiBps_input'] for k, v in e['registered_host_image'].items()}, 'one_shot', e['one_shot']['GiBps_input'])"
done
