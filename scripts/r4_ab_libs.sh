#!/bin/bash
# Variant libraries (go-sstables_amd/librio_<v>.so, "new" = librio.so) against each other: the GPU suite
# on librio.so first (SUITE=0 skips it), then alternating bench lines, two rounds.
# usage: scripts/r4_ab_libs.sh <out-tag> "<variants>" ["<configs>"]
set -u
TAG=$1; VS=$2; CFGS=${3:-"c3 c2 c4"}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
  for c in $CFGS; do
    for v in $VS; do
      LIBP=$PWD/go-sstables_amd/librio.so; [ $v != new ] && LIBP=$PWD/go-sstables_amd/librio_$v.so
      RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/b_${c}_${v}_$r.log 2>&1 || exit 1
      grep '^{' $OUT/b_${c}_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d['stages_ms'])"
    done
  done
done
