#!/bin/bash
# Timing-only A/B (no parity: for experiment builds whose output is knowingly wrong, e.g. RIO_EXP_*):
# interleaved bench lines of librio.so and librio_<tag>.so builds, two rounds.
# usage: scripts/ab_time.sh <out-tag> "<lib-tags>" [configs]
set -u
TAG=$1; LIBS=$2; CFGS=${3:-"c2 c3 c4"}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do
  for c in $CFGS; do
    for v in base $LIBS; do
      if [ $v = base ]; then LIBP=$PWD/go-sstables_amd/librio.so; else LIBP=$PWD/go-sstables_amd/librio_$v.so; fi
      RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none > "$OUT/b_${c}_${v}_$r.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $c $v rc=$rc"; tail -5 "$OUT/b_${c}_${v}_$r.log"; exit $rc; }
      grep '^{' "$OUT/b_${c}_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d['stages_ms'])"
    done
  done
done
exit 0
