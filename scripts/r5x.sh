#!/bin/bash
# r5x: PMC passes of the final build (blend mask, gauss_live groups) for the three configs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5x; mkdir -p $OUT
for c in 1m_1080p_sh3 5m_4k_sh3 500k_1080p_sh3; do
  bash scripts/pmc_session.sh "r5x/pmc_$c" scripts/pmc_all.txt $c > $OUT/pmc_$c.txt 2>&1; rc=$?
  echo "pmc $c rc=$rc"; tail -n 4 $OUT/pmc_$c.txt; [ $rc -eq 0 ] || exit $rc
done
