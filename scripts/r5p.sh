#!/bin/bash
# r5p: gauss_bwd list kernel with 32 entries per wave (e32), and with the view-vector pin as well (e32pin:
# 103 VGPRs, four waves per SIMD); parity of each, interleaved A/B at 1M and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5p; mkdir -p $OUT
for v in e32 e32pin; do
  GSR_LIBRARY=$PWD/gaussian_splatting_amd/lib/libgsr_$v.so timeout -k 10 300 python -u -m pytest tests/test_separate_sh.py tests/test_gpu_train_iteration.py tests/test_gpu_options.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -n 1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
VARIANTS="e32 e32pin" bash scripts/abn.sh r5p/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="e32 e32pin" bash scripts/abn.sh r5p/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
