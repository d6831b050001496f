#!/bin/bash
# round-4 evidence without the (already run) GPU suite: bench lines, rocprofv3 kernel trace, C2 / C4 traffic passes
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step bench 600 python bench.py --config c2
grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --config c2 --no-cpu-baseline --no-e2e --traffic none
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python scripts/kstats.py "$OUT/prof" "$OUT/kernel_launches.json" > /dev/null
step pmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
step pmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
python scripts/traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" c2 k_snappy_pipe "$OUT/traffic.json"
step pmc_fetch_c4 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch_c4" -o run --output-format csv -- \
    python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
step pmc_write_c4 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write_c4" -o run --output-format csv -- \
    python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
python scripts/traffic.py "$OUT/pmc_fetch_c4" "$OUT/pmc_write_c4" c4 k_snappy_pipe_batch "$OUT/traffic_c4.json"
for c in ${PROFILE_LINES:-c3 c4 c1 c2r}; do
    step bench_$c 600 python bench.py --config $c
    grep '^{' "$OUT/bench_$c.log" > "$OUT/bench_$c.json" || true
done
echo done
