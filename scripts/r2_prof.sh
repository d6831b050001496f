#!/bin/bash
# rocprofv3 kernel trace + stats of one bench config (launch count per decode and kernel times)
set -u
OUT=gpurun_out/$1; CFG=${2:-c2}; mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$OUT/prof_$CFG -o run -- python3 /root/repo/bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > /root/repo/$OUT/prof_$CFG.log 2>&1
rc=$?; echo "rocprof $CFG rc=$rc"; find /root/repo/$OUT/prof_$CFG -name "*kernel_stats.csv" | head -1 | xargs -r cut -d, -f1-4 | head -30
