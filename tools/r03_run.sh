#!/bin/bash
# One GPU-box step list for round 3: each step under its own time limit; a GPU
# fault, abort or time-limit kill (rc other than 0/1) ends the session.
#   STEPS="tests:<pytest args>|bench:<bench args>|cmd:<command>" (| separated)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-r03}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
IFS='|' read -ra LIST <<< "${STEPS:-}"
for st in "${LIST[@]}"; do
  i=$((i + 1))
  kind=${st%%:*}
  arg=${st#*:}
  case $kind in
    tests) timeout -k 10 ${TLIM:-900} python -u -m pytest $arg -m gpu -v -s --timeout 600 --timeout-method thread \
             -p no:cacheprovider -rf > "$OUT/step$i.log" 2>&1 ;;
    bench) timeout -k 10 ${BLIM:-600} python -u bench.py $arg --out "$OUT/bench$i.json" > "$OUT/step$i.log" 2>&1 ;;
    cmd) timeout -k 10 ${CLIM:-600} bash -c "$arg" > "$OUT/step$i.log" 2>&1 ;;
  esac
  rc=$?
  echo "[step$i $kind] rc=$rc" | tee -a "$OUT/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc in step$i, stopping"; exit "$rc"; fi
done
echo done
