#!/bin/bash
# PMC passes of the hybrid step (tile kernel + tail step kernel) on Reddit-size F=41,
# each counter group in its own rocprofv3 pass under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-pmc_tiles}
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"
        "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
        "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum"
        "TCP_PENDING_STALL_CYCLES_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum")
i=0
for grp in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_tiles_$i -o run -- \
      python3 tools/tiles_probe.py --config reddit-f41 --sets "${SETS:-tiles=-1}" --reps 1 > "$OUT/pass_$i.log" 2>&1
  rc=$?
  grep -E "Counter_Name|cheb_|tiles_combine" /tmp/pmc_tiles_$i/run_counter_collection.csv > "$OUT/pass_${i}_counters.csv" || true
  echo "[pass $i: $grp] rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc $rc"; exit $rc; fi
done
python3 tools/pmc_summary.py /tmp/pmc_tiles_* --match "wg::" --out "$OUT/pmc_summary.json" > /dev/null
echo done
