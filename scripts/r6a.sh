#!/bin/bash
# r6a: the final build of the round -- GPU suite, smoke, full size, default bench (with the CPU baseline),
# kernel statistics per config, the N=2 rehearsal, PMC passes at 1M@1080p
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_session.sh r6a tests smoke full bench prof cfg:500k_1080p_sh3 cfg:5m_4k_sh3 launch2 || exit $?
bash scripts/pmc_session.sh "r6a/pmc_1m_1080p_sh3" scripts/pmc_all.txt 1m_1080p_sh3 > gpurun_out/r6a/pmc_1m.txt 2>&1; rc=$?
echo "pmc rc=$rc"; tail -n 4 gpurun_out/r6a/pmc_1m.txt; exit $rc
