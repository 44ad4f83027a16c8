#!/bin/bash
# r03: smoke + the GPU suite (main files, then the full-size ones), each under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-r03tests}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {
  echo "[$2] rc=$1" | tee -a "$OUT/steps.log"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "fatal rc in $2, stopping"; exit "$1"; fi
}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
stop_if_fatal $? smoke
timeout -k 10 900 python -u -m pytest tests -m gpu -q --ignore=tests/test_fullsize.py --timeout 300 --timeout-method thread \
    --maxfail=20 -p no:cacheprovider -rf > "$OUT/gpu_tests.log" 2>&1
stop_if_fatal $? pytest_main
if [ "${FULLSIZE:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_fullsize.py -m gpu -v --timeout 600 --timeout-method thread \
      -p no:cacheprovider -rf > "$OUT/gpu_fullsize.log" 2>&1
  stop_if_fatal $? pytest_fullsize
fi
echo done
