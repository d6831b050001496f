#!/bin/bash
# SQ counter passes over one bench config's decode kernel (kernel-trace only, one --pmc set per run).
# usage: scripts/r2_pmc.sh <tag> [config]
set -u
TAG=$1; CFG=${2:-c2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d "$OUT/pmc$i" -o run --output-format csv -- \
      python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && tail -5 "$OUT/pmc$i.log" && exit $rc
done
echo done
