#!/bin/bash
# r5j: gauss_live with one counter atomic per run of G groups (G = 8 default, 1, 4); the cost of the atomic
# flush's touched ORs (attr8) and accumulator adds (attr16) in render_bwd (timing-only builds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5j; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="live1 live4" bash scripts/abn.sh r5j/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="attr8 attr16" bash scripts/abn.sh r5j/abn_attr_1m 2 1m_1080p_sh3 > $OUT/abn_attr_1m.txt 2>&1; rc=$?
cat $OUT/abn_attr_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="live1 live4" bash scripts/abn.sh r5j/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
