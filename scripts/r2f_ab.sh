#!/bin/bash
# Parity of an experiment library (the whole -m gpu suite, or the files in $SUITE), then an
# interleaved A/B against the main build. usage: scripts/r2f_ab.sh <tag> <lib> <cfgs> <rounds>
set -u
TAG=$1; LIB=$2; CFGS=$3; R=${4:-2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
RIO_LIB_PATH=$PWD/go-sstables_amd/librio_$LIB.so timeout -k 10 600 python -u -m pytest ${SUITE:-tests} -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$OUT/tests_$LIB.log" 2>&1
rc=$?; tail -3 "$OUT/tests_$LIB.log"; [ $rc -ne 0 ] && exit $rc
for c in $CFGS; do
  echo "== $c"
  bash scripts/ab_libs.sh $c $R main $LIB || exit 1
done
