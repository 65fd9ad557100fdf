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
REPS=2 CFG=1m_1080p_sh3 bash scripts/ab_env.sh r5d/ab_near_1m "" "GSR_NEAR_MASS=0" "GSR_NEAR_MASS=20" > $OUT/ab_near_1m.txt 2>&1; rc=$?
cat $OUT/ab_near_1m.txt; [ $rc -eq 0 ] || exit $rc
export ABN_SKIP_PARITY=1
VARIANTS="atomic" bash scripts/abn.sh r5d/abn_atomic_1m 2 1m_1080p_sh3 > $OUT/abn_atomic_1m.txt 2>&1; rc=$?
cat $OUT/abn_atomic_1m.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="atomic" bash scripts/abn.sh r5d/abn_atomic_5m 2 5m_4k_sh3 > $OUT/abn_atomic_5m.txt 2>&1; rc=$?
cat $OUT/abn_atomic_5m.txt; [ $rc -eq 0 ] || exit $rc
# verdict r4 item 6: the GSR_CELL=2 build on the large-image test (it failed with 'invalid argument' in r4al)
GSR_LIBRARY=$PWD/gaussian_splatting_amd/lib/libgsr_cell2.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k large_image > $OUT/pytest_cell2_large_image.log 2>&1; rc=$?
echo "cell2 large_image rc=$rc: $(tail -n 1 $OUT/pytest_cell2_large_image.log)"; [ $rc -eq 0 ] || exit $rc
# bench.py --gpus 2 launching its own ranks on one GPU (gloo): the three --exchange auto candidates
GSR_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/launch2.json 2> $OUT/launch2.err; rc=$?
echo "launch2 rc=$rc"; cat $OUT/launch2.json; exit $rc
