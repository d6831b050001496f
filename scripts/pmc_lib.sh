#!/bin/bash
# One PMC pass per library (scripts/pmc_sets.sh for an experiment build).
# usage: scripts/pmc_lib.sh <tag> <config> "<counters>" <lib-tag...>
set -u
TAG=$1; CFG=$2; CTR=$3; shift 3
for v in "$@"; do
  if [ "$v" = base ]; then LIBP=$PWD/go-sstables_amd/librio.so; else LIBP=$PWD/go-sstables_amd/librio_$v.so; fi
  RIO_LIB_PATH=$LIBP ./scripts/pmc_sets.sh "$TAG/$v" "$CFG" "$CTR" || exit $?
done
