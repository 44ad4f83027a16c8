#!/bin/bash
# GPU test session: each pytest group under its own time limit; a GPU fault,
# abort or time-limit kill (rc other than 0/1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-r02_tests}
mkdir -p "$OUT"
run() {  # $1 = tag, $2 = seconds, rest = pytest args
  local tag=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python -u -m pytest "$@" -v -s --timeout 600 --timeout-method thread -p no:cacheprovider \
      -rf > "$OUT/$tag.log" 2>&1
  local rc=$?
  echo "[$tag] rc=$rc" | tee -a "$OUT/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc in $tag, stopping"; exit "$rc"; fi
}
for grp in ${TEST_GROUPS:-main fullsize}; do
  case $grp in
    main) run main 700 tests -m gpu --ignore=tests/test_fullsize.py ;;
    fullsize) run fullsize 700 tests/test_fullsize.py -m gpu ;;
    *) run "$(echo "$grp" | tr '/.:' '___')" 600 $grp -m gpu ;;
  esac
done
echo done
