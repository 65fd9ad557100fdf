#!/bin/bash
# r5zc: K3 skips the record path's inputs after an atomic-backward forward (a record-path backward of such a
# buffer runs rec_prep first); GPU suite + full size on it, A/B against K3 always writing them (k3always)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5zc; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="k3always" bash scripts/abn.sh r5zc/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="k3always" bash scripts/abn.sh r5zc/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_full.log 2>&1; rc=$?
echo "fullsize rc=$rc"; tail -n 1 $OUT/pytest_full.log; exit $rc
