#!/bin/bash
# Round 5: store policy by record size - the decoder parity subset, then C2 / C4 / C3 lines with live traffic.
set -u
mkdir -p gpurun_out/r5m
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_codec_errors.py \
    tests/test_gpu_literal.py tests/test_gpu_reader_api.py tests/test_gpu_snappy_align.py tests/test_gpu_wide.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5m/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/r5m/tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r5_lines.sh r5m "c2 c4 c3"
