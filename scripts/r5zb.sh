#!/bin/bash
# r5zb: what K3's record starts and content-bit zeroing cost (timing build k3norecs: skipped; the atomic backward
# does not read them), 1M and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5zb; mkdir -p $OUT
ABN_SKIP_PARITY=1 VARIANTS="k3norecs" bash scripts/abn.sh r5zb/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="k3norecs" bash scripts/abn.sh r5zb/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
