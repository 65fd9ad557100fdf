#!/bin/bash
# Back-to-back bench processes (1M@1080p), each line: ms/step and the host-side timings of the run
# (bench.py "host": Python call times and the library's own forward / backward / count-wait times),
# to catch the occasional slow process.
# Usage: scripts/host_probe.sh TAG RUNS [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; R=${2:-8}; shift 2; mkdir -p "$OUT"
for i in $(seq 1 $R); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-census --steps 60 "$@" > "$OUT/b$i.json" 2> "$OUT/b$i.err" || exit $?
  python - "$OUT/b$i.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); h = d["host"]
f = lambda k: f"{h[k]['mean']:.3f}/{h[k]['max']:.3f}" if h.get(k) and h[k].get('mean') is not None else "-"
print(f"{d['ms_per_step']:.4f} ms/step | wall {f('step_wall_ms')} | fwd call {f('forward_call_ms')} lib {f('lib_forward_ms')}"
      f" wait {f('lib_count_wait_ms')} | bwd call {f('backward_call_ms')} lib {f('lib_backward_ms')} | gc {h['python_gc_collections']}")
PY
done
