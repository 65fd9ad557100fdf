#!/bin/bash
# Interleaved A/B of library variants: ROUNDS rounds of (every libgsr*.so in turn: bench stage times),
# so clock / box drift hits every variant alike.  Parity of each variant: tests/test_gpu_parity.py once.
# Usage: scripts/abn.sh TAG ROUNDS [CONFIG] [EXTRA BENCH FLAGS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; R=${2:-2}; CFG=${3:-1m_1080p_sh3}; XF=${4:-}; mkdir -p "$OUT"
# VARIANTS="a b" restricts the side libraries to libgsr_a.so libgsr_b.so (default: every libgsr_*.so)
if [ -n "${VARIANTS:-}" ]; then
  LIBS="$ROOT/gaussian_splatting_amd/lib/libgsr.so $(for v in $VARIANTS; do echo $ROOT/gaussian_splatting_amd/lib/libgsr_$v.so; done)"
else
  LIBS="$ROOT/gaussian_splatting_amd/lib/libgsr.so $(ls $ROOT/gaussian_splatting_amd/lib/libgsr_*.so 2>/dev/null)"
fi
for lib in $LIBS; do
  [ "${ABN_SKIP_PARITY:-0}" = "1" ] && break  # (parity established by an earlier run of the same libraries)
  v=$(basename $lib .so)
  # ABN_PARITY_K: a pytest -k expression for the parity run (e.g. to leave out the bitwise-repeatability
  # tests for a variant whose backward is not bitwise reproducible)
  GSR_LIBRARY=$lib timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x ${ABN_PARITY_K:+-k "$ABN_PARITY_K"} > "$OUT/pytest_$v.log" 2>&1; rc=$?
  echo "$v parity rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 $R); do
  for lib in $LIBS; do
    v=$(basename $lib .so)
    GSR_LIBRARY=$lib timeout -k 10 300 python bench.py --config $CFG $XF --no-cpu-baseline --no-census --steps 40 > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err"; rc=$?
    [ $rc -eq 0 ] || { tail -3 "$OUT/bench_${v}_$r.err"; exit $rc; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); s=d['stage_ms']; print('$r $v', round(d['ms_per_step'],4), ' '.join(f'{k}={v*1e3:.1f}' for k,v in s.items()))"
  done
done
