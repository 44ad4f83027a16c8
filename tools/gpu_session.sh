#!/bin/bash
# One GPU-box session: smoke, parity tests, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/timeout stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-s1}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = rc, $2 = step
  local rc=$1
  echo "[$2] rc=$rc" | tee -a "$OUT/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc in $2, stopping"; exit "$rc"; fi
}
rocm-smi --showproductname > "$OUT/gpu.txt" 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
stop_if_fatal $? smoke
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1
  stop_if_fatal $? pytest
fi
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 600 python tools/sweep.py $SWEEP > "$OUT/sweep.log" 2>&1
  stop_if_fatal $? sweep
fi
if [ -n "${SWEEP2:-}" ]; then
  timeout -k 10 600 python tools/sweep.py $SWEEP2 > "$OUT/sweep2.log" 2>&1
  stop_if_fatal $? sweep2
fi
if [ -n "${SWEEP3:-}" ]; then
  timeout -k 10 600 python tools/sweep.py $SWEEP3 > "$OUT/sweep3.log" 2>&1
  stop_if_fatal $? sweep3
fi
timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 3 --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
stop_if_fatal $? bench
if [ "${RUN_PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --sharded-extra none --cold-reps 0 > "$OUT/prof.log" 2>&1
  stop_if_fatal $? rocprof
fi
if [ "${RUN_PMC:-0}" = 1 ]; then
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $ctr | cut -d' ' -f1)
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_$tag" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sharded-extra none --cold-reps 0 --f1-companion 0 \
        > "$OUT/pmc_$tag.log" 2>&1
    stop_if_fatal $? "pmc $tag"
  done
  python tools/pmc_traffic.py --kernel "cheb_step_kernel<4, true" "$OUT"/pmc_* --out "$OUT/traffic.json" \
      > "$OUT/traffic.log" 2>&1
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --sharded-extra none --traffic-json "$OUT/traffic.json" \
      --out "$OUT/bench_traffic.json" > "$OUT/bench_traffic.log" 2>&1
  stop_if_fatal $? bench_traffic
fi
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 900 bash -c "$EXTRA" > "$OUT/extra.log" 2>&1
  stop_if_fatal $? extra
fi
echo done
