#!/bin/bash
# r5y: preprocess -- SH rows evaluated band by band from LDS (pbands), and the first SH half staged by
# global_load_lds into a piece-major image (pglds); parity, A/B at 1M and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5y; mkdir -p $OUT
VARIANTS="pbands pglds" bash scripts/abn.sh r5y/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="pbands pglds" bash scripts/abn.sh r5y/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
