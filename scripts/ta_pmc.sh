#!/bin/bash
# Address-path / LDS / issue counters of k_snappy_pipe on C2: the stock build (2 waves per SIMD)
# and the timing-only 3-wave build (librio_occ.so). One --pmc set per pass, kernel trace only, each pass under its
# own timeout; counters the device does not list are dropped from a set before it runs.
# usage: [CFG=c3] [PASSES="1 7"] scripts/ta_pmc.sh <tag> [libs...]   (libs: base occ ...; default "base occ")
set -u
TAG=$1; shift
LIBS=${*:-base occ}
CFG=${CFG:-c2}; PASSES=${PASSES:-1 2 3 4 5 6 7 8}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
have() { grep -qw "$1" "$OUT/counters_list.txt"; }
SETS=(
  "TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE"
  "TA_BUFFER_WRITE_WAVEFRONTS TA_ADDR_STALLED_BY_TC_CYCLES TD_SPI_STALL TD_LOAD_WAVEFRONT"
  "TA_DATA_STALLED_BY_TC_CYCLES TA_ADDR_STALLED_BY_TD_CYCLES TD_STORE_WAVEFRONT TD_ATOMIC_WAVEFRONT"
  "TCP_TOTAL_CACHE_ACCESSES TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES"
  "TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ TCP_GATE_EN1 TCP_TD_TCP_STALL_CYCLES"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
  "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_BRANCH SQ_IFETCH"
)
for v in $LIBS; do
  LIBP=$PWD/go-sstables_amd/librio.so; [ "$v" != base ] && LIBP=$PWD/go-sstables_amd/librio_$v.so
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    case " $PASSES " in *" $i "*) ;; *) continue ;; esac
    ctr=""; for c in $set; do have "$c" && ctr="$ctr $c"; done
    echo "$v pass $i:$ctr" | tee -a "$OUT/passes.txt"
    [ -z "$ctr" ] && continue
    RIO_LIB_PATH=$LIBP timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/$v/pmc$i" -o run --output-format csv -- \
        python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none > "$OUT/${v}_pmc$i.log" 2>&1
    rc=$?; echo "$v pass $i rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/${v}_pmc$i.log" && exit $rc
  done
  python3 scripts/pmc_summary.py "$OUT/$v" k_snappy_pipe k_walk > "$OUT/${v}_summary.txt" 2>&1; echo "== $v"; cat "$OUT/${v}_summary.txt"
done
