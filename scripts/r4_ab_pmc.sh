#!/bin/bash
# parity subset + A/B vs a reference build, SQ PMC passes of librio.so on C2 (decode and walk), then one
# full C2 bench line (cpu_baseline + e2e)
# usage: scripts/r4_ab_pmc.sh <tag> <ref-lib-tag> [configs]
set -u
TAG=$1; REF=$2; CFGS=${3:-"c2 c3 c4"}
OTHERS="$REF"; for v in ${EXTRA_LIBS:-v4}; do [ -f go-sstables_amd/librio_$v.so ] && OTHERS="$OTHERS $v"; done
bash scripts/ab_libs2.sh $TAG "$OTHERS" "$CFGS" || exit $?
bash scripts/pmc_sets.sh $TAG/pmc c2 "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES" || exit $?
python3 scripts/pmc_summary.py gpurun_out/$TAG/pmc k_snappy_pipe k_walk > gpurun_out/$TAG/pmc_summary.txt 2>&1; cat gpurun_out/$TAG/pmc_summary.txt
timeout -k 10 400 python bench.py --config c2 --steps 20 --warmup 3 > gpurun_out/$TAG/bench_c2_full.log 2>&1 || exit $?
grep '^{' gpurun_out/$TAG/bench_c2_full.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('full c2', d['value'], d['roofline']['frac'], d.get('e2e',{}).get('GiBps_input'), d.get('cpu_baseline',{}).get('value'))"
