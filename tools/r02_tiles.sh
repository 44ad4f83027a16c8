#!/bin/bash
# Hybrid-step session: parity tests, then the Reddit-size probe; each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-r02_tiles}
mkdir -p "$OUT"
step() {  # $1 = tag, $2 = seconds, rest = command
  local tag=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$tag.log" 2>&1
  local rc=$?
  echo "[$tag] rc=$rc" | tee -a "$OUT/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc in $tag, stopping"; exit "$rc"; fi
  return 0
}
if [ -n "${TESTS:-1}" ]; then
  step tests 400 python -u -m pytest ${TEST_ARGS:-tests/test_tiles.py} -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -rf
  grep -q " passed" "$OUT/tests.log" && ! grep -q "FAILED\|ERROR" "$OUT/tests.log" || { echo "tests not green, stopping"; exit 1; }
fi
step probe 600 python -u tools/tiles_probe.py --config ${CONFIG:-reddit-f41} --sets "${SETS:-tiles=0;tiles=1,tile_th=64,tile_max=128}" --reps ${REPS:-5}
echo done
