# Stage / order events released at device scope (librio.so) vs the system-scope default (librio_sysev.so, RIO_EV_SYSTEM=1):
# a parity subset on librio.so, the per-step event cost probe on both, interleaved bench lines.
set -u
OUT=gpurun_out/r5az; mkdir -p $OUT; export TMPDIR=/tmp
TESTS="tests/test_gpu_parity.py tests/test_gpu_threads.py tests/test_gpu_graph.py tests/test_gpu_batch.py tests/test_gpu_walk_lane.py" \
  bash scripts/ab_lib_quick.sh r5az "sysev" "c2 c2r c1 c3" || exit $?
for v in base sysev; do
  LIBP=$PWD/go-sstables_amd/librio.so; [ $v != base ] && LIBP=$PWD/go-sstables_amd/librio_$v.so
  RIO_LIB_PATH=$LIBP timeout -k 10 240 python scripts/event_probe.py 50 > $OUT/probe_$v.txt 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids $OUT/probe_$v.txt
done
