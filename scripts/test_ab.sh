#!/bin/bash
# GPU parity tests of the in-tree library, then A/B timing (scripts/ab_bench.sh) of the given builds.
# usage: scripts/test_ab.sh <tag> <config> <lib-tag...>
set -u
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && echo "tests rc=$rc" && exit $rc
./scripts/ab_bench.sh "$TAG" "$CFG" "$@"
