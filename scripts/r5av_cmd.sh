set -u
OUT=gpurun_out/r5av_far_cp; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/fetch_probe_bin > $OUT/probe.txt 2>&1 && cat $OUT/probe.txt &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- ./scripts/fetch_probe_bin > $OUT/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ TCC_HIT TCC_MISS -d $OUT/pmc_req -o run --output-format csv -- ./scripts/fetch_probe_bin > $OUT/pmc_req.log 2>&1 &&
bash scripts/ab_quick.sh r5av_far_cp "fc1 fc2 fc16 fc17 fc19" "c4"
