set -u; mkdir -p gpurun_out/r1c
for g in 128 256 512 1024 2048; do
  RIO_DECODE_GRID=$g timeout -k 10 300 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r1c/g$g.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/r1c/g$g.log') if l.startswith('{')][0]);print($g, d['value'], d['stages_ms'])"
done
