#!/bin/bash
# r5o: bench.py --gpus 2 (its own ranks, gloo on one GPU) on the final build; where the backward's zero fill
# of the dense outputs lands (GSR_ZERO_FILL 3 = in render_bwd's launch, 2 = its own kernel before it, 1 = a
# side stream): stage attribution at 1M
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5o; mkdir -p $OUT
bash scripts/gpu_session.sh r5o launch2; rc=$?; [ $rc -eq 0 ] || exit $rc
REPS=2 CFG=1m_1080p_sh3 bash scripts/ab_env.sh r5o/ab_fill "GSR_ZERO_FILL=3" "GSR_ZERO_FILL=2" "GSR_ZERO_FILL=1" > $OUT/ab_fill.txt 2>&1; rc=$?
cat $OUT/ab_fill.txt; exit $rc
