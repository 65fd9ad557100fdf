#!/bin/bash
# r6e: the step path's scratch users -- tile_sort_window at four waves (w4: no VGPR spill) and the class-1
# sort kernel on an 8-workgroup grid (c1g8) -- parity, A/B at 1M@1080p
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6e; mkdir -p $OUT
VARIANTS="w4 c1g8" bash scripts/abn.sh r6e/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; exit $rc
