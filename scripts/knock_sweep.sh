#!/bin/bash
# Decode-kernel knock-out attribution (diagnostic): bench C2 for each RIO_KNOCK value. usage: scripts/knock_sweep.sh <tag> <knocks...>
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for k in "$@"; do
  echo "== knock $k"
  RIO_KNOCK=$k timeout -k 10 300 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/k$k.log" 2>&1
  rc=$?; echo "rc=$rc"; tail -1 "$OUT/k$k.log" | grep -o "\"kernel_ms\": [0-9.]*" ; tail -1 "$OUT/k$k.log" | grep -o '"value": [0-9.]*'
  if fatal $rc; then exit $rc; fi
done
