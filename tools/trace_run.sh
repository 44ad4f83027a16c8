#!/bin/bash
# Kernel trace of one command on the GPU box, summarised there (the rocpd
# database of a Reddit-size run is too large to copy back):
#   bash tools/trace_run.sh <out-name> <timeout-s> <program> [args...]
# writes gpurun_out/<out-name>/{cmd.log, stats.csv (per kernel and grid),
# seq.txt (every chain kernel in launch order: name grid_x grid_y ns)}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=$1; tlim=$2; shift 2
OUT=gpurun_out/$name
mkdir -p "$OUT"
export TMPDIR=/tmp
DB=/tmp/trace_$name
rm -rf "$DB"
timeout -k 10 "$tlim" rocprofv3 --kernel-trace -d "$DB" -o run -- "$@" > "$OUT/cmd.log" 2>&1
rc=$?
echo "[trace] rc=$rc" >> "$OUT/cmd.log"
if [ -f "$DB/run_results.db" ]; then
  python tools/rocpd_stats.py "$DB/run_results.db" --by-grid --csv "$OUT/stats.csv"
  python tools/rocpd_stats.py "$DB/run_results.db" --seq --like cheb_ > "$OUT/seq.txt"
  python tools/rocpd_stats.py "$DB/run_results.db" --seq --like tiles_ >> "$OUT/seq.txt"
fi
rm -rf "$DB"
exit $rc
