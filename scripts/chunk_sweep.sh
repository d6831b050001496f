#!/bin/bash
# Framing chunk size (RIO_CHUNK_BYTES) vs C2 / C3 stage times.
set -u
OUT=gpurun_out/chunk; mkdir -p $OUT
for cfg in c2 c3; do
  for cb in ${CHUNKS:-16384 32768 65536}; do
    RIO_CHUNK_BYTES=$cb timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none \
        > $OUT/${cfg}_$cb.log 2>&1 || { echo "fail $cfg $cb"; tail -5 $OUT/${cfg}_$cb.log; exit 1; }
    echo "$cfg chunk=$cb $(grep -o '"value": [0-9.]*' $OUT/${cfg}_$cb.log) $(grep -o 'stages_ms[^}]*}' $OUT/${cfg}_$cb.log)"
  done
done
