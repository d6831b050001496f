#!/bin/bash
# Round 5: the new defaults (late plain flush stores) - parity subset, then against the non-temporal stores build
# (librio_nt1) on C2 / C3 / C4, two rounds; the far-load and store streams on the new tree (timing-only builds).
set -u
scripts/ab_libs2.sh r5j "nt1" "c2 c3 c4" || exit 1
scripts/ab_timing.sh r5j_mem "mem2 mem3" "c2 c4" 1 || exit 1
