#!/bin/bash
# round 6, first GPU call: the new tests on librio.so, then the merged-load variant's parity subset and A/B lines
set -u
OUT=gpurun_out/r6a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 scripts/mem_replay cand > $OUT/replay_cand.txt 2>&1; rc=$?; echo "replay rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_batch.py -m gpu -x -v --timeout 400 \
    --timeout-method thread > $OUT/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc: $(tail -1 $OUT/new_tests.log)"; [ $rc -ne 0 ] && exit $rc
TESTS="tests/test_gpu_parity.py tests/test_gpu_snappy_align.py tests/test_gpu_codec_errors.py tests/test_gpu_literal.py" \
    bash scripts/ab_parity_quick.sh r6a "mrg" "c2 c4 c3"
