#!/bin/bash
# Round-2 session c: a GPU test subset first (new work), then the whole -m gpu suite.
set -u
OUT=gpurun_out/r2c; mkdir -p "$OUT"; export TMPDIR=/tmp
FIRST=${1:-tests/test_gpu_lzw.py}
timeout -k 10 300 python -u -m pytest $FIRST -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/first.log" 2>&1
rc=$?; tail -30 "$OUT/first.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -15 "$OUT/tests.log"; exit $rc
