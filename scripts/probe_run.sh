#!/bin/bash
# GPU call: LDS probe, then GPU tests and a bench line (each step time-limited; stop on a fault).
set -u
OUT=gpurun_out/${1:-probe}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/lds_probe > "$OUT/lds_probe.log" 2>&1 || { echo "probe rc=$?"; exit 1; }
cat "$OUT/lds_probe.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -20 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-e2e > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
