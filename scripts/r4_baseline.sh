set -u
mkdir -p gpurun_out/r4a; export TMPDIR=/tmp
for c in c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r4a/b_$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/r4a/b_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['stages_ms'])"
done
