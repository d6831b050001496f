#!/bin/bash
# Interleaved A/B of decoder variants on one bench config: each library (RIO_LIB_PATH) runs the bench
# `rounds` times in alternation; prints decode-stage ms per run. usage: scripts/ab_libs.sh <cfg> <rounds> lib...
set -u
CFG=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for lib in "$@"; do
    if [ "$lib" = "main" ]; then unset RIO_LIB_PATH; else export RIO_LIB_PATH=$PWD/go-sstables_amd/librio_$lib.so; fi
    out=$(timeout -k 10 180 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-e2e 2>&1 | grep '^{')
    rc=$?
    if [ $rc -ne 0 ]; then echo "$lib failed"; exit 1; fi
    echo "$lib $(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['stages_ms'], d['value'])")"
  done
done
