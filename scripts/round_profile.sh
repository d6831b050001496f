#!/bin/bash
# Round evidence, call 1: the full GPU suite and smoke, the default bench line (live PMC traffic), its rocprofv3
# kernel trace, and the C2 / C4 FETCH_SIZE / WRITE_SIZE passes (scripts/traffic.py records the source tree).
# usage: scripts/round_profile.sh <tag>   (round 5: r5bj, round 6: r6g ...)
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step gpu_tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-e2e --traffic none
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python scripts/kstats.py "$OUT/prof" "$OUT/kernel_launches.json" > /dev/null
for c in c2 c4; do
    k=k_snappy_pipe; [ $c = c4 ] && k=k_snappy_pipe_batch
    step pmc_fetch_$c 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$c" -o run --output-format csv -- \
        python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
    step pmc_write_$c 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write_$c" -o run --output-format csv -- \
        python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --traffic none
    python scripts/traffic.py "$OUT/pmc_fetch_$c" "$OUT/pmc_write_$c" $c $k "$OUT/traffic_$c.json"
done
echo done
