set -u
OUT=gpurun_out/${1:-full}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; exit $rc
