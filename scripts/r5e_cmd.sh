#!/bin/bash
# Round 5 validation call A: the lane-walk, registered-image and DiskKeyIndex GPU tests, then the lane walk
# against the wave walk (and lane chunk sizes) on the bench configs, one box.
set -u
mkdir -p gpurun_out/r5e
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_walk_lane.py tests/test_gpu_stream.py tests/test_gpu_disk_index.py -m gpu -k "walk_lane or registered or handed_back or compressed or fixtures_and or baseline or older or repairs" > gpurun_out/r5e/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -5 gpurun_out/r5e/tests.log; [ $rc -ne 0 ] && exit $rc
R=1 scripts/ab_env.sh r5e "c2 c2r c3 c4" "RIO_WALK_LANE=0" "RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=4096" "RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=16384" "RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=65536"
