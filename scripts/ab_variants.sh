#!/bin/bash
# Decoder variants (librio_<tag>.so built by `make variant`) against the product library on one box:
# the Snappy parity tests on each variant, then interleaved bench lines.
# usage: scripts/ab_variants.sh <out-tag> "<configs>" <rounds> <lib-tag...>   (lib-tag "base" = librio.so)
set -u
TAG=$1; CFGS=$2; R=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
TESTS=${AB_TESTS:-"tests/test_gpu_parity.py tests/test_gpu_codec_errors.py"}
for v in "$@"; do
  [ "$v" = base ] && continue
  RIO_LIB_PATH=$PWD/go-sstables_amd/librio_$v.so timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests_$v.log" 2>&1
  rc=$?; echo "tests $v rc=$rc $(tail -1 $OUT/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for r in $(seq 1 $R); do
  for c in $CFGS; do
    for v in "$@"; do
      if [ "$v" = base ]; then LIBP=$PWD/go-sstables_amd/librio.so; else LIBP=$PWD/go-sstables_amd/librio_$v.so; fi
      RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/b_${c}_${v}_$r.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $c $v rc=$rc"; tail -5 "$OUT/b_${c}_${v}_$r.log"; exit $rc; }
      grep '^{' "$OUT/b_${c}_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d['stages_ms'])"
    done
  done
done
