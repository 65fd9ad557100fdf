#!/bin/bash
# r5h: gauss_live one lane per Gaussian; parity, then interleaved env A/B of bwd_atomic at 1M@1080p and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5h; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=3 CFG=1m_1080p_sh3 bash scripts/ab_env.sh r5h/ab_atomic_1m "GSR_BWD_ATOMIC=0" "GSR_BWD_ATOMIC=1" > $OUT/ab_atomic_1m.txt 2>&1; rc=$?
cat $OUT/ab_atomic_1m.txt; [ $rc -eq 0 ] || exit $rc
REPS=1 CFG=5m_4k_sh3 bash scripts/ab_env.sh r5h/ab_atomic_5m "GSR_BWD_ATOMIC=0" "GSR_BWD_ATOMIC=1" > $OUT/ab_atomic_5m.txt 2>&1; rc=$?
cat $OUT/ab_atomic_5m.txt; exit $rc
