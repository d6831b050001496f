set -u
mkdir -p gpurun_out/r5e
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_walk_lane.py tests/test_gpu_stream.py tests/test_gpu_disk_index.py -m gpu -k "walk_lane or registered or handed_back or compressed or fixtures_and or baseline or older or repairs" > gpurun_out/r5e/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -5 gpurun_out/r5e/tests.log; [ $rc -ne 0 ] && exit $rc
scripts/ab_env.sh r5e "c2 c2r c3 c4" "RIO_WALK_LANE=0" "RIO_WALK_LANE=1" || exit 1
scripts/ab_timing.sh r5d "mem1 mem2 mem3 occ" "c2 c4" 1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r5e/bench_default.log 2>&1; echo bench rc=$?; tail -c 2500 gpurun_out/r5e/bench_default.log
timeout -k 10 300 python bench.py --inproc-devices 0,0 --config c4 --steps 5 > gpurun_out/r5e/inproc_c4.log 2>&1; echo inproc rc=$?; tail -c 1200 gpurun_out/r5e/inproc_c4.log
