#!/bin/bash
# Framing-only parity subset on variant builds, then interleaved bench lines of librio.so against them.
# usage: [TESTS="tests/a.py tests/b.py"] scripts/ab_parity_quick.sh <out-tag> "<variant-tags>" [configs]
set -u
TAG=$1; VS=$2; CFGS=${3:-"c3 c2 c4"}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in $VS; do
  RIO_LIB_PATH=$PWD/go-sstables_amd/librio_$v.so timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py \
      tests/test_gpu_batch.py tests/test_gpu_wide.py} -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests_$v.log" 2>&1
  rc=$?; echo "parity $v rc=$rc: $(tail -1 "$OUT/tests_$v.log")"; [ $rc -ne 0 ] && exit $rc
done
bash scripts/ab_quick.sh "$TAG" "$VS" "$CFGS"
