#!/bin/bash
# One gpurun session: smoke -> GPU tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit. A fault / abort / segfault / timeout (exit >= 124 or
# signal) ends the script; an ordinary test failure (exit 1) does not stop the later steps.
# usage: scripts/gpu_run.sh <tag> [pytest-args...]
set -u
TAG=${1:-run}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }

step() {  # step <name> <timeout-s> <cmd...>
    local name=$1 to=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -5 "$OUT/$name.log"
    if fatal $rc; then
        echo "FATAL in $name (rc=$rc): stopping"
        exit $rc
    fi
    return 0
}

step info 60 bash -c 'rocm-smi --showproductname; nproc; grep -m1 "model name" /proc/cpuinfo; free -g | head -2'
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step tests 900 python -m pytest tests -m gpu -x -q "$@"
step bench 600 python bench.py --steps 20 --warmup 3
cat "$OUT/bench.log" | grep '^{' > "$OUT/bench.json" || true
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; || true
echo "done"
