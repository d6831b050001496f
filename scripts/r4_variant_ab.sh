#!/bin/bash
# A variant build (go-sstables_amd/librio_<tag>.so) against the stock library: the decode parity files
# with the variant, then interleaved bench lines. usage: scripts/r4_variant_ab.sh <out-tag> <variant> [configs]
set -u
TAG=$1; V=$2; CFGS=${3:-"c2 c3 c4"}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
VL=$PWD/go-sstables_amd/librio_$V.so
RIO_LIB_PATH=$VL timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_snappy_align.py tests/test_gpu_batch.py tests/test_gpu_codec_errors.py \
    tests/test_gpu_literal.py > $OUT/tests_$V.log 2>&1
rc=$?; tail -2 $OUT/tests_$V.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for c in $CFGS; do
    for v in new $V; do
      LIBP=$PWD/go-sstables_amd/librio.so; [ $v = $V ] && LIBP=$VL
      RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/b_${c}_${v}_$r.log 2>&1 || exit 1
      grep '^{' $OUT/b_${c}_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d['stages_ms'])"
    done
  done
done
