#!/bin/bash
# Fabric traffic of the step kernels of the three bandwidth legs: the same
# five PMC passes over each workload, every pass its own rocprofv3 run under its own time limit, so
# FETCH_SIZE and WRITE_SIZE come from the same dispatch set as the request counters (pmc_summary.py
# records the dispatch count of every counter).
#   bash tools/pmc_legs.sh <out-name>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=$1
export PMC_PASSES="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum;\
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum;\
TCC_EA0_RDREQ_DRAM_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE"
export PLIM=${PLIM:-240}
legs=${LEGS:-arxiv,rmat8m,reddit41}
for leg in ${legs//,/ }; do
  case $leg in
    arxiv) bash tools/pmc_run.sh "$name/arxiv" python3 tools/knob_ab.py --config ogbn-arxiv --sets "fold=1" --rounds 1 --reps 6 || exit $? ;;
    rmat8m) bash tools/pmc_run.sh "$name/rmat8m" python3 tools/sweep.py --config rmat-8m --grid "hub_iter=16" --reps 1 --warm-s 0 || exit $? ;;
    reddit41) bash tools/pmc_run.sh "$name/reddit41" python3 tools/sweep.py --config reddit-f41 --grid "tile_th=96" --reps 1 --warm-s 0 || exit $? ;;
    # rank 0's shard of the 8-way Reddit-size F = 41 split, stepped alone (the fused hybrid launch, round 6)
    shard8) bash tools/pmc_run.sh "$name/shard8" python3 tools/shard_probe.py --config reddit --world 8 --F 48 --reps 3 || exit $? ;;
  esac
done
