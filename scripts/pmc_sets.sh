#!/bin/bash
# PMC passes (kernel-trace only) on one bench config, one pass per quoted counter set.
# usage: scripts/pmc_sets.sh <tag> <cfg> "<set1>" ["<set2>" ...]
set -u
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d "$OUT/pmc$i" -o run --output-format csv -- \
      python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/pmc$i.log" && exit $rc
done
echo done
