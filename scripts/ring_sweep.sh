#!/bin/bash
# Decode-kernel variant sweep: bench C2/C3 for each RIO_RING value. usage: scripts/ring_sweep.sh <tag> <rings...>
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for r in "$@"; do
  for c in c2 c3; do
    echo "== ring $r $c"
    RIO_RING=$r timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/r${r}_$c.log" 2>&1
    rc=$?; echo "rc=$rc"; tail -1 "$OUT/r${r}_$c.log" | cut -c1-400
    if fatal $rc; then exit $rc; fi
  done
done
