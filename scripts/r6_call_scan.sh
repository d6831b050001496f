#!/bin/bash
# round 6: the one-workgroup scan (k_scan_one) against k_scan_blocks on the lane-walk corpus test, then the framing suite
set -u
OUT=gpurun_out/r6f; mkdir -p $OUT; export TMPDIR=/tmp
T="tests/test_gpu_walk_lane.py::test_fixtures_and_corpus"
RIO_LIB_PATH=$PWD/go-sstables_amd/librio_scan0.so timeout -k 10 300 python -u -m pytest "$T" -m gpu -x -v --timeout 200 \
    --timeout-method thread > $OUT/scan0.log 2>&1
rc=$?; echo "scan0 rc=$rc: $(tail -1 $OUT/scan0.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest "$T" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/scan1.log 2>&1
rc=$?; echo "scan_one rc=$rc: $(tail -1 $OUT/scan1.log)"; [ $rc -ne 0 ] && exit $rc
TESTS="tests/test_gpu_walk_lane.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_reader_api.py tests/test_gpu_graph.py" \
    bash scripts/ab_lib_quick.sh r6f "scan0" "c1 c1s c2"
