#!/bin/bash
# render_bwd traffic attribution: FETCH_SIZE / WRITE_SIZE passes of the
# production library and of the GSR_ATTR measurement builds (libgsr_attr{1,2,4}.so).
# Usage: scripts/pmc_attr.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
for v in "" attr1 attr2 attr4; do
  lib=$ROOT/gaussian_splatting_amd/lib/libgsr${v:+_$v}.so
  GSR_LIBRARY=$lib bash scripts/pmc_session.sh "$1/pmc_${v:-base}" scripts/pmc_fw.txt || exit $?
done
