#!/bin/bash
# r5b: the atomic backward (bwd_atomic) -- parity on the default library (options suite incl. the new
# variant), the atomic library as default against the oracle (small + full-size gradient bars), then
# interleaved A/B at 1M@1080p and 5M@4K.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
export ABN_PARITY_K="not deterministic and not capacity_forward and not sort_prefix_and_redo"
GSR_LIBRARY=$PWD/gaussian_splatting_amd/lib/libgsr_atomic.so timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 600 --timeout-method thread -k "fullsize_backward" > $OUT/pytest_full_atomic.log 2>&1; rc=$?
echo "fullsize atomic rc=$rc"; grep -E "PASS|FAIL|Error|\] " $OUT/pytest_full_atomic.log | tail -n 12; [ $rc -eq 0 ] || exit $rc
VARIANTS="atomic" bash scripts/abn.sh r5b/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="atomic" bash scripts/abn.sh r5b/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
