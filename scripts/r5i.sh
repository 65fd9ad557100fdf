#!/bin/bash
# r5i: gauss_live with 4 groups per wave (default) against 1 and 8; parity of each, interleaved A/B at 1M and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5i; mkdir -p $OUT
VARIANTS="live1 live8" bash scripts/abn.sh r5i/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="live1 live8" bash scripts/abn.sh r5i/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
