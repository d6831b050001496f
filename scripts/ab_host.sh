#!/bin/bash
# A/B of host-runtime builds on one box: WAL replay and the C2 end-to-end lines, alternating.
# usage: scripts/ab_host.sh <tag> <lib-tag...>   (lib-tag "base" = librio.so)
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then LIBP=$PWD/go-sstables_amd/librio.so; else LIBP=$PWD/go-sstables_amd/librio_$v.so; fi
    RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config wal --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/wal_$v.$rep.log" 2>&1 || exit 1
    RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c2_$v.$rep.log" 2>&1 || exit 1
    python3 - "$OUT/wal_$v.$rep.log" "$OUT/c2_$v.$rep.log" "$v" <<'PY'
import json, sys
w = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
e = c["e2e"]
print(sys.argv[3], "wal", w["value"], w["variants_GiBps"], "e2e", e["GiBps_input"],
      {k: v["GiBps_input"] for k, v in e.get("windowed", {}).items()})
PY
  done
done
