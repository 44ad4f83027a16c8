#!/bin/bash
# PMC passes on the step kernel of one sweep config (each counter group in its
# own rocprofv3 pass; an unavailable counter only fails its own pass).
# Usage: SESSION=s11 CONFIG=reddit GRID="iter=16;block_iter=8;chunk_iter=16" bash tools/pmc_probe.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L 2>&1 | grep -E "^[A-Za-z]" | cut -c1-120 > "$OUT/counters.txt" || true
CONFIG=${CONFIG:-reddit}
GRID=${GRID:-iter=16;block_iter=8;chunk_iter=16}
i=0
DEFAULT_GROUPS=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM"
  "TA_BUSY_avr TA_TA_BUSY_sum" "GRBM_GUI_ACTIVE GRBM_COUNT")
# GROUPS="A B|C D" overrides the counter groups ('|' separates passes)
if [ -n "${GROUPS_OVERRIDE:-}" ]; then IFS='|' read -r -a PASSES <<< "$GROUPS_OVERRIDE"; else PASSES=("${DEFAULT_GROUPS[@]}"); fi
for grp in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$PWD/$OUT/pmc_${CONFIG}_$i" -o run -- \
      python3 tools/sweep.py --config $CONFIG --grid "$GRID" --K ${PMC_K:-4} --reps 2 > "$OUT/pmc_${CONFIG}_$i.log" 2>&1
  rc=$?
  echo "[$grp] rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc $rc"; exit $rc; fi
  python3 tools/pmc_traffic.py --kernel ${KERNEL:-cheb_step_kernel} "$OUT/pmc_${CONFIG}_$i" --out "$OUT/pmc_${CONFIG}_$i.json" > /dev/null 2>&1 || true
  rm -rf "$OUT/pmc_${CONFIG}_$i"
done
echo done
