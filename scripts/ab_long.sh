#!/bin/bash
# usage: scripts/ab_long.sh <tag> "<variants>" "<configs>" [steps] : like ab_quick.sh with many steps per line (the
# MALL-flushed pass averages over as many cold steps), three rounds
set -u
TAG=$1; VS=$2; CFGS=$3; ST=${4:-100}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3; do for c in $CFGS; do for v in base $VS; do
  LIBP=$PWD/go-sstables_amd/librio.so; [ $v != base ] && LIBP=$PWD/go-sstables_amd/librio_$v.so
  RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config $c --steps $ST --warmup 3 --no-cpu-baseline --no-e2e --traffic none > "$OUT/b_${c}_${v}_$r.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench $c $v rc=$rc"; tail -5 "$OUT/b_${c}_${v}_$r.log"; exit $rc; }
  grep '^{' "$OUT/b_${c}_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d.get('stages_ms'))"
done; done; done
