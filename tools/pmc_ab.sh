#!/bin/bash
# PMC passes over tools/sweep.py for a knob grid whose points run DIFFERENT kernels (one run
# counts both, e.g. GRID="team=1,0": cheb_team4_kernel and cheb_step_kernel), then per-kernel
# means (tools/pmc_summary.py).  One pass per counter group (rocprofv3 does not split passes).
#   SESSION=name CONFIG=ogbn-arxiv GRID="team=1,0" bash tools/pmc_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-pmc_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
CONFIG=${CONFIG:-ogbn-arxiv}
GRID=${GRID:-team=1,0}
i=0
for grp in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_WAIT_INST_ANY SQ_INSTS_VMEM" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$PWD/$OUT/pmc_$i" -o run -- \
      python3 tools/sweep.py --config "$CONFIG" --grid "$GRID" --reps 5 --warm-s 0.2 > "$OUT/pmc_$i.log" 2>&1
  rc=$?
  echo "[pmc $i: $grp] rc=$rc $(date +%T)"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py "$OUT"/pmc_* --match cheb_ --out "$OUT/pmc_summary.json" > /dev/null
echo "summary: $OUT/pmc_summary.json"
