#!/bin/bash
# C2 / C4 timing A/B of the plain-store build (nt0), then the windowed host path's timeline
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
bash scripts/ab_time.sh $TAG nt0 "c2 c4" || exit $?
RIO_REPLAY_TRACE=1 timeout -k 10 300 python scripts/e2e_trace.py 64 128 > "$OUT/e2e_trace.log" 2>&1; rc=$?
grep "GiB/s" "$OUT/e2e_trace.log"; exit $rc
