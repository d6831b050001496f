#!/bin/bash
# Record-parallel Snappy materialisation probe (scripts/blk_probe.hip) on one C4 file, then the parity
# file and the c2 / c3 / c4 lines of the current tree. usage: scripts/r4_blk.sh <tag>
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
# one C4 file (16384 x 64 KiB text-like records), generated on the host as bench.py does
python -c "
import sys; sys.path.insert(0, 'go-sstables_amd')
from recordio import generate
img = generate(16384, 65536, 2, kind=1, seed=1, threads=16)
open('/tmp/c4.rio', 'wb').write(bytes(img))
print('c4 file', len(img))" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/blk_probe.hip -o /tmp/blk_probe || exit 1
step blk_probe 300 /tmp/blk_probe /tmp/c4.rio 5
step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu
for c in ${LINES:-c4 c2 c3}; do
    step bench_$c 600 python bench.py --config $c --no-cpu-baseline --no-e2e
    grep '^{' "$OUT/bench_$c.log" > "$OUT/bench_$c.json" || true
done
echo done
