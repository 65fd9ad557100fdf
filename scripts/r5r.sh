#!/bin/bash
# r5r: where gauss_bwd's time goes -- a timing build without its deferred SH pass (results wrong, no parity)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5r; mkdir -p $OUT
ABN_SKIP_PARITY=1 VARIANTS="nosh" bash scripts/abn.sh r5r/abn_1m 2 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; exit $rc
