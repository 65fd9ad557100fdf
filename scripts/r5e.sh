#!/bin/bash
# r5e: near-first gate (mean list >= 2048) + atomic backward v2 (gauss_live moves the sums to list order; the
# forward zeroes only the rows that can be touched): parity, full-size gradient bars under the atomic library,
# interleaved A/B at 1M@1080p and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5e; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
GSR_LIBRARY=$PWD/gaussian_splatting_amd/lib/libgsr_atomic.so timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 600 --timeout-method thread -k "fullsize_backward or integers_identical" > $OUT/pytest_full_atomic.log 2>&1; rc=$?
echo "fullsize atomic rc=$rc"; grep -E "PASS|FAIL|Error" $OUT/pytest_full_atomic.log | tail -n 12; [ $rc -eq 0 ] || exit $rc
export ABN_SKIP_PARITY=1
VARIANTS="atomic" bash scripts/abn.sh r5e/abn_atomic_1m 3 1m_1080p_sh3 > $OUT/abn_atomic_1m.txt 2>&1; rc=$?
cat $OUT/abn_atomic_1m.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="atomic" bash scripts/abn.sh r5e/abn_atomic_5m 2 5m_4k_sh3 > $OUT/abn_atomic_5m.txt 2>&1; rc=$?
cat $OUT/abn_atomic_5m.txt; exit $rc
