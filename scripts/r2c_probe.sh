#!/bin/bash
# Round-2 session c: GPU tests on the rebuilt tree, then an occupancy probe of the Snappy lane decoder
# (grid 256 = 1 wave per SIMD vs the default 512 = 2 waves per SIMD).
set -u
OUT=gpurun_out/r2c; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_libs.sh c2 2 main g256
