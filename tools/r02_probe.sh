#!/bin/bash
# Round-2 profiling session: rocprofv3 kernel trace + PMC passes of the step
# kernels the verdict names (Reddit-size F=41 run as F=44, 8M R-MAT hub teams).
# Usage: SESSION=r02_s1 PARTS="trace reddit rmat8m" bash tools/r02_probe.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-r02}
mkdir -p "$OUT"
export TMPDIR=/tmp
PARTS=${PARTS:-trace reddit rmat8m}
fatal() { echo "[$1] rc=$2" | tee -a "$OUT/steps.log"; if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then exit "$2"; fi; }
for part in $PARTS; do
  case $part in
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/trace_reddit" -o run -- \
        python3 tools/sweep.py --config reddit-f41 --grid "iter=192;chunk_iter=128" --K 16 --reps 5 > "$OUT/trace_reddit.log" 2>&1
      fatal trace_reddit $?
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/trace_rmat8m" -o run -- \
        python3 tools/sweep.py --config rmat-8m --grid "hub_iter=16" --K 32 --reps 3 > "$OUT/trace_rmat8m.log" 2>&1
      fatal trace_rmat8m $?
      ;;
    reddit)
      SESSION=${SESSION:-r02}/pmc_reddit CONFIG=reddit-f41 GRID="iter=192;chunk_iter=128" KERNEL="cheb_step_kernel<4" \
        timeout -k 10 1000 bash tools/pmc_deep.sh > "$OUT/pmc_reddit.log" 2>&1
      fatal pmc_reddit $?
      ;;
    rmat8m)
      SESSION=${SESSION:-r02}/pmc_rmat8m CONFIG=rmat-8m GRID="hub_iter=16" KERNEL="cheb_hub1_kernel" PMC_K=4 \
        timeout -k 10 1000 bash tools/pmc_deep.sh > "$OUT/pmc_rmat8m.log" 2>&1
      fatal pmc_rmat8m $?
      ;;
    *)
      if [ -n "${EXTRA:-}" ]; then timeout -k 10 900 bash -c "$EXTRA" > "$OUT/extra.log" 2>&1; fatal extra $?; fi
      ;;
  esac
done
echo done
