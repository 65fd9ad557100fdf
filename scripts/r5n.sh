#!/bin/bash
# r5n: gauss_bwd without scratch (dL/dmean3D kept in a register); the view-vector pin for the combined SH
# layout too (libgsr_gbpin: 165 -> 103 VGPRs); parity of both, interleaved A/B at 1M and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5n; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
GSR_LIBRARY=$PWD/gaussian_splatting_amd/lib/libgsr_gbpin.so timeout -k 10 300 python -u -m pytest tests/test_separate_sh.py tests/test_gpu_train_iteration.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gbpin_sep.log 2>&1; rc=$?
echo "gbpin separate_sh rc=$rc"; tail -n 2 $OUT/pytest_gbpin_sep.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="gbpin live8" bash scripts/abn.sh r5n/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="gbpin live8" bash scripts/abn.sh r5n/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
