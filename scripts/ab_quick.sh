#!/bin/bash
# usage: abwalk.sh <tag> "<variants>" "<configs>" : interleaved bench lines (no parity), walk-focused
set -u
TAG=$1; VS=$2; CFGS=$3; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for c in $CFGS; do for v in base $VS; do
  LIBP=$PWD/go-sstables_amd/librio.so; [ $v != base ] && LIBP=$PWD/go-sstables_amd/librio_$v.so
  RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none > "$OUT/b_${c}_${v}_$r.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench $c $v rc=$rc"; tail -5 "$OUT/b_${c}_${v}_$r.log"; exit $rc; }
  grep '^{' "$OUT/b_${c}_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d['stages_ms'], d.get('verified'))"
done; done; done
