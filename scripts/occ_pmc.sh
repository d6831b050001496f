#!/bin/bash
# SQ counters of k_snappy_pipe on C2: the stock build (2 waves per SIMD) against the timing-only 3-wave build
# (librio_occ.so: RIO_EXP_OCC=1, grid 768; WRONG output, same instruction stream). usage: scripts/occ_pmc.sh <tag>
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
S2="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"
for v in base occ; do
  LIBP=$PWD/go-sstables_amd/librio.so; [ $v = occ ] && LIBP=$PWD/go-sstables_amd/librio_occ.so
  i=0
  for set in "$S1" "$S2"; do
    i=$((i+1))
    RIO_LIB_PATH=$LIBP timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d "$OUT/$v/pmc$i" -o run --output-format csv -- \
        python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none > "$OUT/${v}_pmc$i.log" 2>&1
    rc=$?; echo "$v pass $i rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/${v}_pmc$i.log" && exit $rc
  done
  python3 scripts/pmc_summary.py "$OUT/$v" k_snappy_pipe > "$OUT/${v}_summary.txt" 2>&1; echo "== $v"; cat "$OUT/${v}_summary.txt"
done
