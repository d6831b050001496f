#!/bin/bash
# The driver's N>1 launch shape, rehearsed on a one-GPU box: torchrun with 2 ranks sharing device 0
# (RIO_BENCH_ONE_DEVICE=1), C2 (a file per rank) and C4 (the 8-file set split over the ranks).
set -u
OUT=gpurun_out/${1:-rehearse}; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in c2 c4; do
  RIO_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --config $c > "$OUT/n2_$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; grep '^{' "$OUT/n2_$c.log" | cut -c1-400 || tail -20 "$OUT/n2_$c.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
