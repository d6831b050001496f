#!/bin/bash
# GPU tests (optional) + bench over several configs. usage: scripts/bench_sweep.sh <tag> <run_tests 0|1> <configs...>
set -u
TAG=$1; TESTS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
        echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"; if fatal $rc; then echo "FATAL $name"; exit $rc; fi; }
if [ "$TESTS" = 1 ]; then run tests 900 python -m pytest tests -m gpu -x -q; fi
for c in "$@"; do run "bench_$c" 600 python bench.py --config "$c" --steps 10 --warmup 2 --no-cpu-baseline --no-e2e; done
