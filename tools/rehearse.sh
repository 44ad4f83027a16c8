#!/bin/bash
# One-GPU rehearsal of the driver's N > 1 bench: N ranks share device 0 (gloo process
# group, IPC halo exchange; RCCL refuses two ranks per device), same bench.py flags
# otherwise.  N <= 8 (the box allows 16 GPU processes).
#   N=4 SESSION=name [EXCH=ipc|sdma|ipc,sdma] bash tools/rehearse.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${N:-2}
OUT=gpurun_out/${SESSION:-rehearse}
mkdir -p "$OUT"
export TMPDIR=/tmp
# a heartbeat under gpurun_out/ while the ranks generate their graphs (they print nothing meanwhile)
( while sleep 30; do echo "[hb N=$N] $(date +%T)" >> "$OUT/hb.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
WATS_BENCH_DEVICE=0 WATS_BENCH_PG=gloo timeout -k 10 ${TLIM:-500} python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port ${PORT:-29533} bench.py --gpus "$N" \
    --steps ${STEPS:-5} --warmup 1 --exchange ${EXCH:-ipc} --sharded-extra "${EXTRA:-none}" \
    --out "$OUT/bench$N.json" > "$OUT/rehearse$N.log" 2>&1
rc=$?
echo "[rehearse N=$N] rc=$rc" | tee -a "$OUT/steps.log"
exit $rc
