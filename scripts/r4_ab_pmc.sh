#!/bin/bash
# parity subset + A/B vs a reference build, then two SQ PMC passes of librio.so on C2
# usage: scripts/r4_ab_pmc.sh <tag> <ref-lib-tag> [configs]
set -u
TAG=$1; REF=$2; CFGS=${3:-"c2 c3 c4"}
bash scripts/ab_libs2.sh $TAG $REF "$CFGS" || exit $?
bash scripts/pmc_sets.sh $TAG/pmc c2 "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES" || exit $?
python3 scripts/pmc_summary.py gpurun_out/$TAG/pmc k_snappy_pipe 2>/dev/null | head -30 || true
