#!/bin/bash
# Parity subset on the current librio.so, then interleaved bench lines of librio.so against another build.
# usage: scripts/ab_libs2.sh <tag> <other-lib-tag> [configs]   (other = go-sstables_amd/librio_<tag>.so)
set -u
# OTHER: one or more lib tags, space-separated
TAG=$1; OTHER=$2; CFGS=${3:-"c2 c3 c4"}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_codec_errors.py \
    tests/test_gpu_literal.py tests/test_gpu_reader_api.py tests/test_gpu_snappy_align.py tests/test_gpu_wide.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for c in $CFGS; do
    for v in new $OTHER; do
      if [ $v = new ]; then LIBP=$PWD/go-sstables_amd/librio.so; else LIBP=$PWD/go-sstables_amd/librio_$v.so; fi
      RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none > "$OUT/b_${c}_${v}_$r.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $c $v rc=$rc"; tail -5 "$OUT/b_${c}_${v}_$r.log"; exit $rc; }
      grep '^{' "$OUT/b_${c}_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d['stages_ms'])"
    done
  done
done
exit 0
