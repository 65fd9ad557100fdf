#!/bin/bash
# r5u: blend mask with the ORs deferred past the next batch's loads; parity (GPU suite + full size) and
# interleaved A/B at 1M, 5M@4K and 500k
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5u; mkdir -p $OUT
L=$PWD/gaussian_splatting_amd/lib/libgsr_blend.so
GSR_LIBRARY=$L timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest_blend.log 2>&1; rc=$?
echo "blend tests rc=$rc"; tail -n 1 $OUT/pytest_blend.log; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="blend" bash scripts/abn.sh r5u/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="blend" bash scripts/abn.sh r5u/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="blend" bash scripts/abn.sh r5u/abn_500k 2 500k_1080p_sh3 > $OUT/abn_500k.txt 2>&1; rc=$?
cat $OUT/abn_500k.txt; [ $rc -eq 0 ] || exit $rc
GSR_LIBRARY=$L timeout -k 10 800 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_full_blend.log 2>&1; rc=$?
echo "blend fullsize rc=$rc"; tail -n 1 $OUT/pytest_full_blend.log; exit $rc
