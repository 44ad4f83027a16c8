#!/bin/bash
# One GPU-box session, parameterised (replaces the per-session r0*_s*.sh scripts):
#   SESSION=<name> tools/session.sh <step> [<step> ...]
# Steps (each under its own time limit; a crash, abort or timeout ends the session):
#   smoke          __graft_entry__.smoke()
#   tests          pytest -m gpu, every file but the full-size one
#   fullsize       pytest tests/test_fullsize.py -m gpu
#   bench          python bench.py (the driver's default N = 1 line) -> bench.json
#   headline_prof  rocprofv3 --kernel-trace --stats of the N = 1 headline workload ALONE
#                  (no companions / extras): its kernel summary reproduces the line's roofline
#   pmc            FETCH_SIZE / WRITE_SIZE / L2 hit passes of the headline alone -> traffic.json
#   sweep:<args>   python tools/sweep.py <args> (spaces as '+'), WATS_HIP_LIB from $LIB if set
#   rehearse:<N>   tools/rehearse.sh: the N-rank bench with every rank on device 0 (IPC exchange)
#   py:<script>    python <script> (spaces as '+')
# Output: gpurun_out/$SESSION/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
HEADLINE="--no-cpu-baseline --sharded-extra none --cold-reps 0 --f1-companion 0 --connected-companion 0 --pubmed-companion 0"
n=0
stop_if_fatal() {  # $1 = rc, $2 = step
  echo "[$2] rc=$1 $(date +%T)" | tee -a "$OUT/steps.log"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "fatal rc $1 in $2, stopping"; exit "$1"; fi
}
for step in "$@"; do
  n=$((n + 1))
  case "$step" in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      stop_if_fatal $? smoke ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --ignore=tests/test_fullsize.py --timeout 300 \
          --timeout-method thread --maxfail=20 -p no:cacheprovider -rf > "$OUT/gpu_tests.log" 2>&1
      stop_if_fatal $? tests ;;
    fullsize)
      timeout -k 10 900 python -u -m pytest tests/test_fullsize.py -m gpu -v --timeout 600 --timeout-method thread \
          -p no:cacheprovider -rf > "$OUT/gpu_fullsize.log" 2>&1
      stop_if_fatal $? fullsize ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps ${STEPS:-20} --warmup 3 --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
      stop_if_fatal $? bench ;;
    headline_prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$$ -o run -- \
          python3 -u bench.py --steps ${STEPS:-20} --warmup 3 $HEADLINE --out "$OUT/headline.json" \
          > "$OUT/headline_prof.log" 2>&1
      rc=$?
      mkdir -p "$OUT/headline_prof"
      find /tmp/prof_$$ -name '*kernel_stats.csv' -exec cp {} "$OUT/headline_prof/" \;
      find /tmp/prof_$$ -name '*kernel_trace.csv' -exec cp {} "$OUT/headline_prof/" \;
      rm -rf /tmp/prof_$$
      stop_if_fatal $rc headline_prof ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
        tag=$(echo $ctr | cut -d' ' -f1)
        timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_$tag" -o run -- \
            python3 bench.py --steps 2 --warmup 1 $HEADLINE > "$OUT/pmc_$tag.log" 2>&1
        stop_if_fatal $? "pmc $tag"
      done
      python3 tools/pmc_traffic.py --kernel "${PMC_KERNEL:-cheb_team4_kernel}" "$OUT"/pmc_* \
          --out "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1
      rm -rf "$OUT"/pmc_FETCH_SIZE "$OUT"/pmc_WRITE_SIZE "$OUT"/pmc_TCC_HIT_sum ;;
    sweep:*)
      args=$(echo "${step#sweep:}" | tr '+' ' ')
      WATS_HIP_LIB=${LIB:-} timeout -k 10 600 python -u tools/sweep.py $args > "$OUT/sweep$n.log" 2>&1
      stop_if_fatal $? "sweep$n" ;;
    rehearse:*)
      N=${step#rehearse:} SESSION=${SESSION:-session}/rehearse bash tools/rehearse.sh
      stop_if_fatal $? "$step" ;;
    py:*)
      args=$(echo "${step#py:}" | tr '+' ' ')
      timeout -k 10 600 python -u $args > "$OUT/py$n.log" 2>&1
      stop_if_fatal $? "py$n" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
