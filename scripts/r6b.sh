#!/bin/bash
# r6b: the forward's blend bits per entry through one SGPR and a select into lane j's VGPR (bvgpr) instead of
# one 64-bit SGPR mask per quadrant (which spill under the 80-SGPR budget); parity, A/B at 1M, 5M@4K, 500k
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6b; mkdir -p $OUT
VARIANTS="bvgpr" bash scripts/abn.sh r6b/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="bvgpr" bash scripts/abn.sh r6b/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="bvgpr" bash scripts/abn.sh r6b/abn_500k 2 500k_1080p_sh3 > $OUT/abn_500k.txt 2>&1; rc=$?
cat $OUT/abn_500k.txt; exit $rc
