#!/bin/bash
# Round 5 call: lane-walk parity after the pipelining change and its chunk sizes against the wave walk; the paired
# input prefetch variant (parity subset, then A/B); the default bench line (live traffic).
set -u
mkdir -p gpurun_out/r5g
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_walk_lane.py -m gpu > gpurun_out/r5g/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/r5g/tests.log; [ $rc -ne 0 ] && exit $rc
R=1 scripts/ab_env.sh r5g "c2 c2r c3" "RIO_WALK_LANE=0" "RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=8192" "RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=16384" || exit 1
scripts/ab_variant.sh r5g_pair inpair "c2 c3 c4" || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r5g/bench_default.log 2>&1; echo bench rc=$?; tail -c 2500 gpurun_out/r5g/bench_default.log
