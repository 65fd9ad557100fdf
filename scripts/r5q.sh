#!/bin/bash
# r5q: gauss_bwd list kernel on a 2048-block strided grid (gbs) instead of the worst-case grid, and with the view-vector pin (gbspin)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5q; mkdir -p $OUT
for v in gbs gbspin; do
  GSR_LIBRARY=$PWD/gaussian_splatting_amd/lib/libgsr_$v.so timeout -k 10 300 python -u -m pytest tests/test_separate_sh.py tests/test_gpu_train_iteration.py tests/test_gpu_options.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -n 1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
VARIANTS="gbs gbspin" bash scripts/abn.sh r5q/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="gbs gbspin" bash scripts/abn.sh r5q/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
