#!/bin/bash
# A/B timing of experiment builds: one bench line per library (no profiler).
# usage: scripts/ab_bench.sh <tag> <config> <lib-tag...>   (lib-tag "base" = librio.so)
set -u
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then LIBP=$PWD/go-sstables_amd/librio.so; else LIBP=$PWD/go-sstables_amd/librio_$v.so; fi
  RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config "$CFG" --steps ${AB_STEPS:-10} --warmup 2 --no-cpu-baseline --no-e2e --traffic none > "$OUT/$v.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && echo "$v rc=$rc" && tail -5 "$OUT/$v.log" && exit $rc
  tail -1 "$OUT/$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['stages_ms'])"
done
