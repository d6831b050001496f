#!/bin/bash
# Round 5 call B: the decoder's memory-stream timing builds, the default bench line (live traffic), the in-process
# multi-device line.
set -u
mkdir -p gpurun_out/r5f
scripts/ab_timing.sh r5f "mem1 mem2 mem3 occ" "c2 c4" 1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r5f/bench_default.log 2>&1; echo bench rc=$?; tail -c 2500 gpurun_out/r5f/bench_default.log
timeout -k 10 300 python bench.py --inproc-devices 0,0 --config c4 --steps 5 > gpurun_out/r5f/inproc_c4.log 2>&1; echo inproc rc=$?; tail -c 1200 gpurun_out/r5f/inproc_c4.log
