#!/bin/bash
# Framing chunk size (RIO_CHUNK_BYTES) against the walk stage, per config. usage: scripts/chunk_env_sweep.sh "<cfgs>" "<sizes>"
set -u
for c in $1; do
  for k in $2; do
    out=$(RIO_CHUNK_BYTES=$k timeout -k 10 180 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none 2>&1 | grep '^{')
    echo "$c $k $(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['stages_ms'], d['value'])")"
  done
done
