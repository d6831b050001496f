#!/bin/bash
# Parity subset (TESTS=...) on librio.so itself, then interleaved bench lines of librio.so against variant builds.
# usage: [TESTS="tests/a.py ..."] scripts/ab_lib_quick.sh <out-tag> "<variant-tags>" [configs]
set -u
TAG=$1; VS=$2; CFGS=${3:-"c2 c3 c4"}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "parity librio.so rc=$rc: $(tail -1 "$OUT/tests.log")"; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_quick.sh "$TAG" "$VS" "$CFGS"
