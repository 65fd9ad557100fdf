#!/bin/bash
# r5l: PMC passes of the final build (atomic backward default) for the three configs; the per-lane-entry
# cost probe of 4x4-block units (libgsr_lanee) against the product forward at 500k@1080p and 1M@1080p
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5l; mkdir -p $OUT
for c in 1m_1080p_sh3 5m_4k_sh3 500k_1080p_sh3; do
  bash scripts/pmc_session.sh "r5l/pmc_$c" scripts/pmc_all.txt $c > $OUT/pmc_$c.txt 2>&1; rc=$?
  echo "pmc $c rc=$rc"; cat $OUT/pmc_$c.txt; [ $rc -eq 0 ] || exit $rc
done
VARIANTS="lanee" bash scripts/abn.sh r5l/abn_lanee_500k 3 500k_1080p_sh3 > $OUT/abn_lanee_500k.txt 2>&1; rc=$?
cat $OUT/abn_lanee_500k.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="lanee" bash scripts/abn.sh r5l/abn_lanee_1m 2 1m_1080p_sh3 > $OUT/abn_lanee_1m.txt 2>&1; rc=$?
cat $OUT/abn_lanee_1m.txt; exit $rc
