#!/bin/bash
# Round 5: the flush store after the step's loads (librio_late, parity subset first) and plain flush stores
# (librio_nt0) against the stock build; the C1 line with the auto walk's chunk-count gate; the in-process
# multi-device line (device 0 listed twice).
set -u
scripts/ab_variant.sh r5i_late late "c2 c4" || exit 1
scripts/ab_timing.sh r5i_nt0 "nt0" "c2 c4" 1 || exit 1
mkdir -p gpurun_out/r5i
timeout -k 10 300 python bench.py --config c1 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none > gpurun_out/r5i/c1.log 2>&1; echo c1 rc=$?; grep '^{' gpurun_out/r5i/c1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['value'], d['stages_ms'])"
timeout -k 10 300 python bench.py --inproc-devices 0,0 --config c4 --steps 5 > gpurun_out/r5i/inproc_c4.log 2>&1; echo inproc rc=$?; tail -c 1500 gpurun_out/r5i/inproc_c4.log
