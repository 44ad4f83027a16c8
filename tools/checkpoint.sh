#!/bin/bash
# One GPU checkpoint of the current tree (run on the GPU box): the main GPU test suite, smoke(), the
# default bench line and a headline-only rocprofv3 kernel trace.  Each step has its own time limit;
# the first failure ends the run.
#   bash tools/checkpoint.sh <out-name> [steps: tests,smoke,bench,prof]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=$1
steps=${2:-tests,smoke,bench,prof}
OUT=gpurun_out/$name
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in ${steps//,/ }; do
  case $s in
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
             > "$OUT/tests.log" 2>&1 || { echo "tests failed rc=$?"; tail -30 "$OUT/tests.log"; exit 1; } ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
             || { echo "smoke failed rc=$?"; tail -30 "$OUT/smoke.log"; exit 1; } ;;
    bench) timeout -k 10 900 python -u bench.py --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 \
             || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.log"; exit 1; } ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- \
            python3 bench.py --no-cpu-baseline --sharded-extra none --cold-reps 0 --f1-companion 0 \
            --connected-companion 0 --pubmed-companion 0 --replicas 0 --out "$OUT/headline.json" > "$OUT/prof.log" 2>&1 \
             || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
          cp "$(find /tmp/prof_$name -name '*kernel_stats.csv' | head -1)" "$OUT/headline_kernel_stats.csv" ;;
  esac
  echo "[$s] done"
done
