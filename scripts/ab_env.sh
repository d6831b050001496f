#!/bin/bash
# usage: scripts/ab_env.sh <tag> "<configs>" "ENV=a" "ENV=b" ... : interleaved bench lines of librio.so under each
# environment setting (no parity), two rounds
set -u
TAG=$1; CFGS=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do for c in $CFGS; do i=0; for e in "$@"; do i=$((i+1))
  env $e timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --traffic none > "$OUT/b_${c}_${i}_$r.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench $c [$e] rc=$rc"; tail -5 "$OUT/b_${c}_${i}_$r.log"; exit $rc; }
  grep '^{' "$OUT/b_${c}_${i}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c [$e]', d['value'], d.get('stages_ms'))"
done; done; done
