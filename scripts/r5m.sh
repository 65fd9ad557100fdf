#!/bin/bash
# r5m: gauss_live runs of 2 / 4 groups per wave and atomic, now without scratch (r5j's G > 1 builds kept their
# row arrays in scratch memory) against one group per wave; 1M and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5m; mkdir -p $OUT
VARIANTS="live2 live4" bash scripts/abn.sh r5m/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="live2 live4" bash scripts/abn.sh r5m/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
