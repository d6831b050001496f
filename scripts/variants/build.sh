#!/bin/bash
# A/B variants of the Snappy decoder: builds go-sstables_amd/librio_<tag>.so from scripts/variants/<src>.hip
# in place of rio_snappy.hip (RIO_LIB_PATH selects it). usage: scripts/variants/build.sh <tag> <src> [defs]
set -eu
TAG=$1; SRC=$2; DEFS=${3:-}
C=go-sstables_amd/csrc
mkdir -p $C/build_$TAG
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -Iinclude -I$C -I/opt/rocm/include --offload-arch=gfx950 -munsafe-fp-atomics $DEFS \
    -c scripts/variants/$SRC.hip -o $C/build_$TAG/snappy.o
OBJS=$(ls $C/build/*.o | grep -v rio_snappy.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $C/build_$TAG/snappy.o -o go-sstables_amd/librio_$TAG.so -lz -lpthread
echo built go-sstables_amd/librio_$TAG.so
