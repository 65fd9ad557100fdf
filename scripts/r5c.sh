#!/bin/bash
# r5c: interleaved A/B of the atomic backward (libgsr_atomic.so: bwd_atomic on by default) at 1M@1080p, 5M@4K
# and 500k@1080p (parity of each library first, without the bitwise-repeatability tests)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5c; mkdir -p $OUT
# parity of both libraries: r5b (388 -m gpu tests with the bwd_atomic variants, the full-size gradient bars under
# the atomic library); the bitwise-repeatability tests do not apply to the atomic path
export ABN_SKIP_PARITY=1
VARIANTS="atomic" bash scripts/abn.sh r5c/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="atomic" bash scripts/abn.sh r5c/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="atomic" bash scripts/abn.sh r5c/abn_500k 2 500k_1080p_sh3 > $OUT/abn_500k.txt 2>&1; rc=$?
cat $OUT/abn_500k.txt; exit $rc
