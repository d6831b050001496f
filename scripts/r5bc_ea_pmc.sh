#!/bin/bash
# L2 -> fabric (EA) request counters of the decode kernels on C4 and C2 and of the random-load probe
# (scripts/fetch_probe.hip): request sizes, the DRAM path's share, credit stalls, requests in flight (latency by
# Little's law). Two --pmc passes per program, kernel trace only, each under its own timeout.
# usage: scripts/r5bc_ea_pmc.sh <tag>
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_DRAM GRBM_GUI_ACTIVE"
P2="TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ TCC_EA0_WRREQ_64B GRBM_GUI_ACTIVE"
i=0
for set in "$P1" "$P2"; do
  i=$((i+1))
  for c in c4 c2; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set -d "$OUT/${c}_p$i" -o run --output-format csv -- \
      python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none > "$OUT/${c}_p$i.log" 2>&1
    rc=$?; echo "$c pass $i rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/${c}_p$i.log" && exit $rc
  done
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d "$OUT/probe_p$i" -o run --output-format csv -- \
    ./scripts/fetch_probe_bin > "$OUT/probe_p$i.log" 2>&1
  rc=$?; echo "probe pass $i rc=$rc"; [ $rc -ne 0 ] && tail -20 "$OUT/probe_p$i.log" && exit $rc
done
echo done
