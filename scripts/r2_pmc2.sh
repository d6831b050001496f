#!/bin/bash
# Counter passes (one --pmc set per run) over one bench config, for the in-tree library and any
# variant libraries given (RIO_LIB_PATH). usage: scripts/r2_pmc2.sh <tag> <config> "<lib tags>" set1 [set2 ...]
set -u
TAG=$1; CFG=$2; LIBS=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for lib in $LIBS; do
  if [ "$lib" = "main" ]; then unset RIO_LIB_PATH; else export RIO_LIB_PATH=$PWD/go-sstables_amd/librio_$lib.so; fi
  i=0
  for set in "$@"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d "$OUT/$lib/pmc$i" -o run --output-format csv -- \
        python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/$lib.pmc$i.log" 2>&1
    rc=$?; echo "$lib pass $i rc=$rc"; [ $rc -ne 0 ] && tail -5 "$OUT/$lib.pmc$i.log" && exit $rc
  done
done
echo done
