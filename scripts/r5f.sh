#!/bin/bash
# r5f: the atomic backward follows its forward's mark; bitwise tests pinned to the record path; both backward
# paths at full size; interleaved env A/B of bwd_atomic at 1M@1080p and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5f; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=3 CFG=1m_1080p_sh3 bash scripts/ab_env.sh r5f/ab_atomic_1m "GSR_BWD_ATOMIC=0" "GSR_BWD_ATOMIC=1" > $OUT/ab_atomic_1m.txt 2>&1; rc=$?
cat $OUT/ab_atomic_1m.txt; [ $rc -eq 0 ] || exit $rc
REPS=2 CFG=5m_4k_sh3 bash scripts/ab_env.sh r5f/ab_atomic_5m "GSR_BWD_ATOMIC=0" "GSR_BWD_ATOMIC=1" > $OUT/ab_atomic_5m.txt 2>&1; rc=$?
cat $OUT/ab_atomic_5m.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 600 --timeout-method thread > $OUT/pytest_full.log 2>&1; rc=$?
echo "fullsize rc=$rc"; grep -E "PASS|FAIL|Error|atomic vs record" $OUT/pytest_full.log | tail -n 40; exit $rc
