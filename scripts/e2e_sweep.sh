#!/bin/bash
# End-to-end (host image -> device decode -> host records) rate vs staging copy threads.
set -u
OUT=gpurun_out/e2e; mkdir -p $OUT
for t in ${E2E_THREADS:-0 4 6 12}; do
    RIO_COPY_THREADS=$t timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/t$t.log 2>&1 \
        || { echo "fail $t"; tail -5 $OUT/t$t.log; exit 1; }
    echo "threads=$t $(grep -o '"e2e": {[^}]*}' $OUT/t$t.log)"
done
