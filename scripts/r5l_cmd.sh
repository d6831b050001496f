#!/bin/bash
# Round 5: the lane walk with 4 chains per lane: its parity tests, then walk A/B (wave walk vs forced lane walk at
# 16 / 32 KiB lane chunks) on C2, C2-ref-random, C1.
set -u
mkdir -p gpurun_out/r5l
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk_lane.py -m gpu > gpurun_out/r5l/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/r5l/tests.log; [ $rc -ne 0 ] && exit $rc
R=1 scripts/ab_env.sh r5l "c2 c2r c1" "RIO_WALK_LANE=0" "RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=16384" "RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=32768" "RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=8192"
