# C1 cold pass with and without a code-warming 64-record decode between the eviction and the step (RIO_BENCH_CODE_WARM)
set -u
OUT=gpurun_out/r5ax; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do for w in 0 1; do
  RIO_BENCH_CODE_WARM=$w timeout -k 10 300 python bench.py --config c1 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --traffic none > $OUT/c1_w${w}_$r.log 2>&1 || exit $?
  grep '^{' $OUT/c1_w${w}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1 code_warm=$w', d['value'], d['stages_ms'], d.get('warm'), d.get('verified'))"
done; done
