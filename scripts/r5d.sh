#!/bin/bash
# r5d: near-first binning (parity, full-size bitwise, A/B at 5M@4K and 1M@1080p) and the atomic backward A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5d; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 600 --timeout-method thread > $OUT/pytest_full.log 2>&1; rc=$?
echo "fullsize rc=$rc"; grep -E "near-first|PASS|FAIL|Error" $OUT/pytest_full.log | tail -n 40; [ $rc -eq 0 ] || exit $rc
REPS=2 CFG=5m_4k_sh3 bash scripts/ab_env.sh r5d/ab_near_5m "" "GSR_NEAR_MASS=0" > $OUT/ab_near_5m.txt 2>&1; rc=$?
cat $OUT/ab_near_5m.txt; [ $rc -eq 0 ] || exit $rc
REPS=3 CFG=1m_1080p_sh3 bash scripts/ab_env.sh r5d/ab_near_1m "" "GSR_NEAR_MASS=0" > $OUT/ab_near_1m.txt 2>&1; rc=$?
cat $OUT/ab_near_1m.txt; [ $rc -eq 0 ] || exit $rc
export ABN_SKIP_PARITY=1
VARIANTS="atomic" bash scripts/abn.sh r5d/abn_atomic_1m 3 1m_1080p_sh3 > $OUT/abn_atomic_1m.txt 2>&1; rc=$?
cat $OUT/abn_atomic_1m.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="atomic" bash scripts/abn.sh r5d/abn_atomic_5m 2 5m_4k_sh3 > $OUT/abn_atomic_5m.txt 2>&1; rc=$?
cat $OUT/abn_atomic_5m.txt; exit $rc
