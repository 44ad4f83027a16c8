#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group, each under its own time
# limit) of any command on the GPU box:
#   bash tools/pmc_run.sh <out-name> <program> [args...]
# writes gpurun_out/<out-name>/{pass_i.log, steps.log, pmc_summary.json}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=$1; shift
OUT=gpurun_out/$name
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"
        "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
        "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum"
        "TCP_PENDING_STALL_CYCLES_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum")
# PMC_PASSES="A B C;D E" replaces the default groups (';' between passes)
if [ -n "${PMC_PASSES:-}" ]; then IFS=';' read -r -a PASSES <<< "$PMC_PASSES"; fi
i=0
for grp in "${PASSES[@]}"; do
  i=$((i+1))
  rm -rf /tmp/pmc_${name}_$i
  timeout -s KILL ${PLIM:-240} rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_${name}_$i -o run -- "$@" > "$OUT/pass_$i.log" 2>&1
  rc=$?
  echo "[pass $i: $grp] rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc $rc"; exit $rc; fi
done
python3 tools/pmc_summary.py /tmp/pmc_${name}_* --match "wg::" --out "$OUT/pmc_summary.json" > /dev/null
rm -rf /tmp/pmc_${name}_*
echo done
