#!/bin/bash
# k_walk_lanes (RIO_WALK_LANES=1): the full GPU suite with it, then c2 / c3 / c1 / c4 lines
# of both walks. usage: scripts/r4_walk.sh <tag>
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step suite_lanes 1000 env RIO_WALK_LANES=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests
for v in 1 0 1 0; do
    for c in ${LINES:-c2 c3}; do
        step bench_${c}_lanes$v 300 env RIO_WALK_LANES=$v python bench.py --config $c --no-cpu-baseline --no-e2e
        grep '^{' "$OUT/bench_${c}_lanes$v.log" | python -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$c lanes=$v', d['value'], d['stages_ms'])"
    done
done
echo done
