set -u
OUT=gpurun_out/v9a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_codec_errors.py tests/test_gpu_batch.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
./scripts/ab_bench.sh v9a c2 base v9 base v9 && ./scripts/ab_bench.sh v9a4 c4 base v9
