#!/bin/bash
# r03: bench line + rocprofv3 kernel trace of the same bench command (N=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-r03bench}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {
  echo "[$2] rc=$1" | tee -a "$OUT/steps.log"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "fatal rc in $2, stopping"; exit "$1"; fi
}
if [ "${FULLSIZE:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_fullsize.py -m gpu -v --timeout 600 --timeout-method thread \
      -p no:cacheprovider -rf > "$OUT/gpu_fullsize.log" 2>&1
  stop_if_fatal $? pytest_fullsize
fi
timeout -k 10 600 python -u bench.py --steps ${STEPS:-20} --warmup 3 --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
stop_if_fatal $? bench
if [ "${RUN_PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$$ -o run -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --sharded-extra none --cold-reps 0 > "$OUT/prof.log" 2>&1
  rc=$?
  mkdir -p "$OUT/prof"
  cp /tmp/prof_$$/run_kernel_stats.csv "$OUT/prof/" 2>/dev/null || find /tmp/prof_$$ -name '*kernel_stats.csv' -exec cp {} "$OUT/prof/" \;
  rm -rf /tmp/prof_$$
  stop_if_fatal $rc rocprof
fi
echo done
