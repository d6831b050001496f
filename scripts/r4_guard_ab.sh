#!/bin/bash
set -u
OUT=gpurun_out/r4gd; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_snappy_align.py tests/test_gpu_batch.py tests/test_gpu_wide.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for c in c2 c3; do
    for v in new head; do
      LIBP=$PWD/go-sstables_amd/librio.so; [ $v = head ] && LIBP=$PWD/go-sstables_amd/librio_head.so
      RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/b_${c}_${v}_$r.log 2>&1 || exit 1
      grep '^{' $OUT/b_${c}_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d['stages_ms'])"
    done
  done
done
