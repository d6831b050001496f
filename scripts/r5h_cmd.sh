#!/bin/bash
# Round 5: the full GPU suite and smoke on the tree with the auto walk and the paired input prefetch, then
# A/B: the walk modes (RIO_WALK_LANE 0 / auto) and the input prefetch (librio_nopair.so) on the bench configs.
set -u
bash scripts/r4_tests.sh r5h || exit $?
R=1 scripts/ab_env.sh r5h "c2 c2r c1 c3" "RIO_WALK_LANE=0" "RIO_WALK_LANE=2" || exit 1
scripts/ab_timing.sh r5h_pair "nopair" "c2 c3 c4" 2 || exit 1
