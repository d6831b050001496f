#!/bin/bash
# One-box A/B of environment knobs on bench lines, interleaved, two rounds.
# usage: scripts/ab_env.sh <tag> "<configs>" "<env settings A>" "<env settings B>" [...]
#   e.g. scripts/ab_env.sh r3g "c2 c3" "RIO_FUSED=0" "RIO_FUSED=1"
set -u
TAG=$1; CFGS=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 ${R:-2}); do
  for c in $CFGS; do
    v=0
    for e in "$@"; do
      v=$((v + 1))
      env $e timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none \
          > "$OUT/b_${c}_v${v}_$r.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $c [$e] rc=$rc"; tail -5 "$OUT/b_${c}_v${v}_$r.log"; exit $rc; }
      grep '^{' "$OUT/b_${c}_v${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c [$e]', d['value'], d['stages_ms'])"
    done
  done
done
