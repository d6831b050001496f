#!/bin/bash
# C1 (100k x 1 KiB uncompressed, MALL flushed between steps): framing chunk size, two rounds
set -u
for r in 1 2; do bash scripts/chunk_env_sweep.sh "c1" "32768 16384 8192 4096"; done
