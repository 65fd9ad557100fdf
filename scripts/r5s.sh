#!/bin/bash
# r5s: software-pipelined LDS reads of the staged entries (the next entry's rows read before the current one
# is evaluated) in render_fwd (fpf) and render_bwd (bpf); parity, interleaved A/B at 1M and 5M@4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5s; mkdir -p $OUT
ABN_PARITY_K="not census" VARIANTS="fpf bpf hoist" bash scripts/abn.sh r5s/abn_1m 3 1m_1080p_sh3 > $OUT/abn_1m.txt 2>&1; rc=$?
cat $OUT/abn_1m.txt; [ $rc -eq 0 ] || exit $rc
ABN_SKIP_PARITY=1 VARIANTS="fpf bpf hoist" bash scripts/abn.sh r5s/abn_5m 2 5m_4k_sh3 > $OUT/abn_5m.txt 2>&1; rc=$?
cat $OUT/abn_5m.txt; exit $rc
