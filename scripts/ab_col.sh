#!/bin/bash
# The column decoder (RIO_SNAPPY_COL=1) on one box: the Snappy parity suites first, then interleaved
# bench lines against k_snappy_pipe. usage: scripts/ab_col.sh <tag> [configs] [skip-tests]
set -u
TAG=$1; CFGS=${2:-"c2 c3 c4"}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "${3:-}" ]; then
  RIO_SNAPPY_COL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py \
      tests/test_gpu_codec_errors.py tests/test_gpu_literal.py tests/test_gpu_reader_api.py tests/test_gpu_snappy_align.py tests/test_gpu_wide.py -m gpu -x -q \
      --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
  for c in $CFGS; do
    for v in 1 0; do
      RIO_LIB_PATH=$([ $v = 1 ] && echo $PWD/go-sstables_amd/librio.so || echo $PWD/go-sstables_amd/librio_v9.so) timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/b_${c}_col${v}_$r.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $c col=$v rc=$rc"; tail -5 "$OUT/b_${c}_col${v}_$r.log"; exit $rc; }
      grep '^{' "$OUT/b_${c}_col${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c col=$v', d['value'], d['stages_ms'])"
    done
  done
done
# one PMC pass per decoder on C2 (instruction counts; kernel-trace only)
if [ -n "${AB_PMC:-}" ]; then
  for v in 1 0; do
    RIO_SNAPPY_COL=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
        -d "$OUT/pmc_col$v" -o run --output-format csv -- python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/pmc_col$v.log" 2>&1
    rc=$?; echo "pmc col=$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
fi
exit 0
