#!/bin/bash
# A/B of the main library against variant libraries on bench configs (decode-stage ms, GiB/s),
# after the decode parity tests of the main library. usage: scripts/r2c_ab.sh "<cfgs>" <rounds> <lib...>
set -u
CFGS=$1; R=$2; shift 2
OUT=gpurun_out/r2c; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_codec_errors.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ab_tests.log" 2>&1
rc=$?; tail -2 "$OUT/ab_tests.log"; [ $rc -ne 0 ] && exit $rc
for c in $CFGS; do echo "== $c"; bash scripts/ab_libs.sh $c $R "$@" || exit 1; done
