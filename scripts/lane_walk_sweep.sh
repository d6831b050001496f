#!/bin/bash
set -u
OUT=gpurun_out/lw; mkdir -p $OUT; export TMPDIR=/tmp
for c in c1s c1; do for lc in 2048 4096 8192; do
  RIO_LIB_PATH=$PWD/go-sstables_amd/librio_nofuse.so RIO_WALK_LANE=1 RIO_LANE_CHUNK_BYTES=$lc timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none > $OUT/${c}_$lc.log 2>&1 || exit 1
  grep '^{' $OUT/${c}_$lc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c lane$lc', d['value'], d['stages_ms'])"
done; done
