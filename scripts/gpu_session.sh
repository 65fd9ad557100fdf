#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.  Stops at the
# first crash / timeout (exit codes other than 0 = pass and 1 = test failures).
# Usage: scripts/gpu_session.sh TAG [forcebuild] [tests] [smoke] [full] [bench] [prof] [pmc] [cfg:C] ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "host: $(hostname) cpus=$(nproc)" > "$OUT/host.txt"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
for stage in "$@"; do
  case $stage in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "not fullsize" > "$OUT/pytest.log" 2>&1; rc=$?
      echo "tests rc=$rc"; tail -5 "$OUT/pytest.log"; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc ;;
    full)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread -k "fullsize" > "$OUT/pytest_full.log" 2>&1; rc=$?
      echo "full rc=$rc"; tail -5 "$OUT/pytest_full.log"; ok $rc || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
      echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; [ $rc -eq 0 ] || exit $rc ;;
    cpuonly)  # BASELINE configs[0]: the pure-PyTorch fallback forward on this host, no GPU touched
      timeout -k 10 600 python bench.py --cpu-only --config 10k_256_sh0 > "$OUT/cpu_only_10k_256_sh0.json" 2> "$OUT/cpu_only.err"; rc=$?
      echo "cpuonly rc=$rc"; cat "$OUT/cpu_only_10k_256_sh0.json"; [ $rc -eq 0 ] || exit $rc ;;
    benchquick)
      timeout -k 10 600 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
      echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; [ $rc -eq 0 ] || exit $rc ;;
    variants)
      for lib in gaussian_splatting_amd/lib/libgsr_*.so; do
        v=$(basename $lib .so)
        GSR_LIBRARY=$ROOT/$lib timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > "$OUT/pytest_$v.log" 2>&1; rc=$?
        echo "variant $v tests rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; ok $rc || exit $rc
        GSR_LIBRARY=$ROOT/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"; rc=$?
        echo "variant $v rc=$rc"; python -c "import json,sys; d=json.load(open('$OUT/bench_$v.json')); print(' ', d['ms_per_step'], d['stage_ms'])"; [ $rc -eq 0 ] || exit $rc
      done ;;
    cfg:*)  # bench + kernel stats of one config: cfg:<config>
      c=${stage#cfg:}
      timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"; rc=$?
      echo "bench $c rc=$rc"; cat "$OUT/bench_$c.json"; [ $rc -eq 0 ] || exit $rc
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o run -- \
        python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-census > "$OUT/prof_$c.log" 2>&1); rc=$?
      echo "prof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmccfg:*)  # PMC passes of one config: pmccfg:<config>
      c=${stage#pmccfg:}
      bash scripts/pmc_session.sh "$TAG/pmc_$c" scripts/pmc_all.txt $c; rc=$?
      echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    launch2)  # bench.py --gpus 2 launching its own ranks (child torch.distributed.run), on one GPU with gloo
      GSR_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 \
        > "$OUT/launch2.json" 2> "$OUT/launch2.err"; rc=$?
      echo "launch2 rc=$rc"; cat "$OUT/launch2.json"; tail -3 "$OUT/launch2.err"; [ $rc -eq 0 ] || exit $rc ;;
    stamps)  # per-workgroup timelines of the binning and render kernels (needs libgsr_stamps.so, built beforehand)
      GSR_LIBRARY=$ROOT/gaussian_splatting_amd/lib/libgsr_stamps.so timeout -k 10 300 python tools/stamps.py > "$OUT/stamps.json" 2> "$OUT/stamps.err"; rc=$?
      echo "stamps rc=$rc"; tail -c 3000 "$OUT/stamps.json"; [ $rc -eq 0 ] || exit $rc ;;
    forcebuild)  # rebuild libgsr.so from the sources on this box (ignoring the pushed library) and check its id
      { sha256sum gaussian_splatting_amd/lib/libgsr.so; cat gaussian_splatting_amd/lib/libgsr.so.inputs; } > "$OUT/build_force.log" 2>&1
      timeout -k 10 900 python -m gaussian_splatting_amd.build --force --jobs 16 >> "$OUT/build_force.log" 2>&1; rc=$?
      { sha256sum gaussian_splatting_amd/lib/libgsr.so; python -c "from gaussian_splatting_amd import _lib, build; \
print('gsr_build_id', _lib.build_id(), 'tree', build.input_hash())"; } >> "$OUT/build_force.log" 2>&1
      echo "forcebuild rc=$rc"; cat "$OUT/build_force.log"; [ $rc -eq 0 ] || exit $rc ;;
    calib)  # FETCH_SIZE / WRITE_SIZE against known byte counts per access shape (tools/fetch_calib.hip), one pass each
      for ctr in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/calib_$ctr" -o run -- \
          "$ROOT/tools/fetch_calib" > "$OUT/calib_$ctr.log" 2>&1); rc=$?
        echo "calib $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done
      python tools/fetch_calib.py "$OUT/calib_FETCH_SIZE" "$OUT/calib_WRITE_SIZE" "$OUT/calib_FETCH_SIZE.log" \
        --json "$OUT/fetch_calib.json" | tee "$OUT/fetch_calib.md" ;;
    abn:*)  # interleaved A/B of the side libraries: abn:<rounds>[:<config>]
      spec=${stage#abn:}; r=${spec%%:*}; c=1m_1080p_sh3; [ "$spec" != "$r" ] && c=${spec#*:}
      bash scripts/abn.sh "$TAG/abn_$c" $r $c > "$OUT/abn_$c.txt" 2>&1; rc=$?
      echo "abn $c rc=$rc"; cat "$OUT/abn_$c.txt"; [ $rc -eq 0 ] || exit $rc ;;
    cpus)  # the CPU set the baselines run on
      python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP', os.environ.get('OMP_NUM_THREADS'))" | tee "$OUT/cpus.txt" ;;
    rehearse2)  # N=2 on one GPU (gloo collectives): the multi-rank bench path, both exchanges
      for ex in auto views dense allreduce; do
        GSR_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --exchange $ex \
          > "$OUT/rehearse2_$ex.json" 2> "$OUT/rehearse2_$ex.err"; rc=$?
        echo "rehearse2 $ex rc=$rc"; cat "$OUT/rehearse2_$ex.json"; [ $rc -eq 0 ] || exit $rc
      done ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-census > "$OUT/prof.log" 2>&1); rc=$?
      echo "prof rc=$rc"; tail -3 "$OUT/prof.log"; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      for ctr in "FETCH_SIZE" "WRITE_SIZE"; do
        (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_$ctr" -o run -- \
          python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-census > "$OUT/pmc_$ctr.log" 2>&1); rc=$?
        echo "pmc $ctr rc=$rc"; tail -2 "$OUT/pmc_$ctr.log"; [ $rc -eq 0 ] || exit $rc
      done ;;
  esac
done
