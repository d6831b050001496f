#!/bin/bash
# A/B experiment builds (csrc/Makefile `variant`): bench + FETCH_SIZE pass per library.
# usage: scripts/variant_sweep.sh <tag> <config> <lib-tag...>   (lib-tag "base" = librio.so)
set -u
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then LIBP=$PWD/go-sstables_amd/librio.so; else LIBP=$PWD/go-sstables_amd/librio_$v.so; fi
  echo "== $v"
  RIO_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config "$CFG" --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/$v.log" 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && tail -5 "$OUT/$v.log" && exit $rc
  tail -1 "$OUT/$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['roofline']['kernel_ms'])"
  RIO_LIB_PATH=$LIBP timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_$v" -o run --output-format csv -- \
      python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/pmc_$v.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && tail -5 "$OUT/pmc_$v.log" && exit $rc
  python3 - "$OUT/pmc_$v" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(p)) if "k_snappy_pipe" in r["Kernel_Name"]]
print("  FETCH_SIZE max KiB", max(v), "-> read bytes x2 =", 2 * max(v) * 1024 / 1e9, "GB")
PY
done
