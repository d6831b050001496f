#!/bin/bash
# Round evidence on one GPU box: GPU tests, smoke, the default bench line, the rocprofv3 kernel-trace
# summary of the same command, and the FETCH_SIZE / WRITE_SIZE passes that give the decode kernel's
# HBM traffic (scripts/traffic.py). Every GPU step has its own time limit; a fault, abort or
# timeout ends the script. usage: scripts/profile_round.sh <tag> [config]
set -u
TAG=$1; CFG=${2:-c2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -n "${LINES_ONLY:-}" ]; then  # only the extra bench lines (second call of a round)
    for c in $LINES_ONLY; do
        echo "== bench_$c ($(date +%T))"
        timeout -k 10 600 python bench.py --config $c > "$OUT/bench_$c.log" 2>&1 || { echo "bench_$c failed"; tail -5 "$OUT/bench_$c.log"; exit 1; }
        grep '^{' "$OUT/bench_$c.log" > "$OUT/bench_$c.json" || true
        tail -c 300 "$OUT/bench_$c.json"; echo
    done
    exit 0
fi
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
step() {
    local name=$1 to=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --config "$CFG"
grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --config "$CFG" --no-cpu-baseline --no-e2e --traffic none
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python scripts/kstats.py "$OUT/prof" "$OUT/kernel_launches.json" > /dev/null  # per launch, probe dispatch excluded
step pmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
step pmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
python scripts/traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$CFG" k_snappy_pipe "$OUT/traffic.json"
# C4's decode-kernel traffic (roofline.traffic of the c4 line: profiles/traffic_c4.json)
if [ -z "${SKIP_C4_PMC:-}" ]; then
step pmc_fetch_c4 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch_c4" -o run --output-format csv -- \
    python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
step pmc_write_c4 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write_c4" -o run --output-format csv -- \
    python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
python scripts/traffic.py "$OUT/pmc_fetch_c4" "$OUT/pmc_write_c4" c4 k_snappy_pipe_batch "$OUT/traffic_c4.json"
fi
# the SSTable line (SURVEY config 5) and its kernel trace
step bench_c5 600 python bench.py --config c5
grep '^{' "$OUT/bench_c5.log" > "$OUT/bench_c5.json" || true
step rocprof_c5 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- \
    python bench.py --config c5 --no-cpu-baseline
find "$OUT/prof_c5" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_c5.csv" \;
# the other bench lines (their own metrics): WAL replay, batched DiskKeyIndex.Get, device encode, random records;
# PROFILE_LINES overrides the list (e.g. "c1 c3 c4 c2g" in a second call, keeping each call within gpurun's limit)
for c in ${PROFILE_LINES:-wal idx enc c2r}; do
    step bench_$c 600 python bench.py --config $c
    grep '^{' "$OUT/bench_$c.log" > "$OUT/bench_$c.json" || true
done
echo done
