#!/bin/bash
# Two-wave decoder (RIO_SNAPPY_PAIR=1) against the one-wave decoder on one box: the pair path's parity
# suite on the bounded-wait debug build (a stuck queue prints and ends instead of hanging), one PMC
# pass per decoder on C2 (VALU instructions, waves, busy cycles), then interleaved bench lines.
# usage: scripts/ab_pair2.sh <tag> [configs]
set -u
TAG=$1; CFGS=${2:-"c2 c4"}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
RIO_SNAPPY_PAIR=1 RIO_LIB_PATH=$PWD/go-sstables_amd/librio_pdbg.so timeout -k 10 400 python -u -m pytest \
    tests/test_gpu_parity.py tests/test_gpu_codec_errors.py tests/test_gpu_batch.py -m gpu -x -q --timeout 60 \
    --timeout-method thread > "$OUT/tests_pair.log" 2>&1
rc=$?; tail -3 "$OUT/tests_pair.log"; grep -m3 "stuck\|runaway" "$OUT/tests_pair.log"; [ $rc -ne 0 ] && exit $rc
for p in 0 1; do
  RIO_SNAPPY_PAIR=$p timeout -k 10 120 rocprofv3 --kernel-trace \
      --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
      -d "$OUT/pmc_p$p" -o run --output-format csv -- \
      python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/pmc_p$p.log" 2>&1
  rc=$?; echo "pmc pair=$p rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/pmc_p$p.log"; exit $rc; }
  python scripts/pmc_summary.py "$OUT/pmc_p$p" k_snappy_pipe k_snappy_pair > "$OUT/pmc_p$p.txt"; cat "$OUT/pmc_p$p.txt"
done
for r in 1 2; do
  for c in $CFGS; do
    for p in 0 1; do
      RIO_SNAPPY_PAIR=$p timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/b_${c}_p${p}_$r.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $c pair=$p rc=$rc"; tail -5 "$OUT/b_${c}_p${p}_$r.log"; exit $rc; }
      grep '^{' "$OUT/b_${c}_p${p}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c pair=$p', d['value'], d['stages_ms'])"
    done
  done
done
