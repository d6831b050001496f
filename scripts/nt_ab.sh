set -u
./scripts/ab_bench.sh nt c2 base nt1 nt2 nt3 base && \
./scripts/pmc_lib.sh ntpmc c2 "FETCH_SIZE" base nt1 nt2 nt3 && \
./scripts/pmc_lib.sh ntpmcw c2 "WRITE_SIZE" base nt1
