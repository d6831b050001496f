#!/bin/bash
# The CPU test suite (pytest -m "not gpu") against the sanitizer builds: oracle/librio_oracle_asan.so (the C restatement)
# and go-sstables_amd/librio_asan.so (host runtime: rio_capi, rio_writer, rio_replay) with ASan + UBSan, clang's shared
# runtime preloaded into the interpreter. Any report aborts the test process (UBSan without recovery, ASan by default).
# usage (CPU container, no GPU needed): scripts/asan_cpu_suite.sh [log]   ->  profiles/r6/r6_asan_cpu_suite.log
set -eu
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r6/r6_asan_cpu_suite.log}
mkdir -p "$(dirname "$LOG")"
make -s -C oracle asan
make -s -C go-sstables_amd/csrc asan -j8
RT=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export RIO_ORACLE_PATH=$PWD/oracle/librio_oracle_asan.so RIO_LIB_PATH=$PWD/go-sstables_amd/librio_asan.so
# leaks: the interpreter and torch keep allocations to exit; odr: torch and ROCm libraries register the same globals
export ASAN_OPTIONS=detect_leaks=0:detect_odr_violation=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
{
  echo "# ASan + UBSan CPU suite: oracle $RIO_ORACLE_PATH, library $RIO_LIB_PATH, runtime $RT"
  echo "# $(date -u +%FT%TZ) tree $(git rev-parse --short HEAD)"
  LD_PRELOAD=$RT python -m pytest tests -m "not gpu" -q -p no:cacheprovider 2>&1
} | tee "$LOG"
