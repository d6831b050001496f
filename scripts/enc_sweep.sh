#!/bin/bash
# Encoder launch-shape sweep: LDS kernel lanes per wave (RIO_ENC_LANES), LDS on/off, global grid.
set -u
OUT=gpurun_out/enc_sweep; mkdir -p $OUT
for cfg in ${ENC_CFGS:-"1 4 128" "1 16 128" "1 8 128" "1 4 128" "1 16 128"}; do
    set -- $cfg
    RIO_ENC_LDS=$1 RIO_ENC_LANES=$2 RIO_ENC_GROUPS=$3 timeout -k 10 120 python bench.py --config enc --steps 5 --warmup 1 \
        --no-cpu-baseline > $OUT/c_$1_$2_$3.log 2>&1 || { echo "fail $cfg"; tail -5 $OUT/c_$1_$2_$3.log; exit 1; }
    echo "lds=$1 lanes=$2 groups=$3 $(grep -o '"value": [0-9.]*' $OUT/c_$1_$2_$3.log)"
done
