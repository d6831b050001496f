#!/bin/bash
# Round 3: the device paths built while no GPU run was possible (pytest marker `pending`), then a C2
# bench line and its kernel trace.
# usage: scripts/r3_pending.sh <tag>
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
RIO_TEST_PENDING=1 timeout -k 10 300 python -u -m pytest tests -m "gpu and pending" -v --timeout 120 \
    --timeout-method thread > "$OUT/pending.log" 2>&1
rc=$?; tail -25 "$OUT/pending.log"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > "$OUT/bench_c2.log" 2>&1 || exit $?
grep '^{' "$OUT/bench_c2.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > "$OUT/prof.log" 2>&1 || exit $?
find "$OUT/prof" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$OUT/kernel_stats.csv"
head -12 "$OUT/kernel_stats.csv"
