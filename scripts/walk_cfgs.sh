set -u
for c in c2g c2r c4 c1 c2; do
  for v in base w0 base w0; do
    if [ $v = base ]; then L=$PWD/go-sstables_amd/librio.so; else L=$PWD/go-sstables_amd/librio_$v.so; fi
    RIO_LIB_PATH=$L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --traffic none > gpurun_out/wc_${c}_${v}.log 2>&1 || exit 1
    echo $c $v $(grep "^{" gpurun_out/wc_${c}_${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stages_ms']['walk'])")
  done
done
