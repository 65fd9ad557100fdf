#!/bin/bash
# Interleaved A/B of library builds: bench.py under each library in turn, ROUNDS rounds, per config.
# Usage: scripts/ab_libs.sh TAG ROUNDS "CONFIGS" LIB... (LIB: a path under gaussian_splatting_amd/lib, "base",
# or "env:NAME=VALUE[,NAME=VALUE...]" -- the default library under those environment settings, e.g. a GSR_ option)
# Each run's JSON line goes to gpurun_out/TAG/<config>_<lib>_<round>.json; a summary (median ms/step and
# render-stage times per library) is printed at the end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=$1; ROUNDS=$2; CONFIGS=$3; shift 3
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for cfg in $CONFIGS; do
  for r in $(seq 1 "$ROUNDS"); do
    for lib in "$@"; do
      name=$(basename "$lib" .so)
      if [ "$lib" = base ]; then env_lib=""
      elif [ "${lib#env:}" != "$lib" ]; then env_lib=$(echo "${lib#env:}" | tr ',' ' '); name=$(echo "${lib#env:}" | sed 's#[^,]*/##g' | tr ',=' '-.')
      else env_lib="GSR_LIBRARY=$ROOT/$lib"; fi
      env $env_lib timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --no-census --steps 30 \
        > "$OUT/${cfg}_${name}_$r.json" 2> "$OUT/${cfg}_${name}_$r.err"; rc=$?
      echo "$cfg $name round $r rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
python3 - "$OUT" <<'PY'
import glob, json, os, statistics, sys, collections
out = sys.argv[1]
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "*.json"))):
    base = os.path.basename(f)[:-5]
    cfg, rest = base.split("_", 1)[0], base
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    key = base.rsplit("_", 1)[0]
    rows[key].append((d["ms_per_step"], d["stage_ms"]))
for key, v in sorted(rows.items()):
    ms = [x[0] for x in v]
    st = {k: statistics.median([x[1].get(k, 0) for x in v]) for k in v[0][1]}
    print(f"{key:40s} ms/step median {statistics.median(ms):.4f} (min {min(ms):.4f} max {max(ms):.4f}) "
          + " ".join(f"{k} {st[k]*1e3:.1f}" for k in ("render_fwd", "render_bwd", "tile_sort", "bin_count", "bin_scatter", "gauss_bwd", "gauss_reduce")))
PY
