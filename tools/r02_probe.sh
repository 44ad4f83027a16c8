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
    sweeps)
      # gather-only probe (knob probe) and cache-line row padding (knob fpad) on the two wide workloads
      timeout -k 10 300 python3 tools/sweep.py --config ogbn-arxiv --grid "probe=0,1,0,1" --K 16 --reps 20 \
        > "$OUT/sweep_arxiv_probe.log" 2>&1
      fatal sweep_arxiv_probe $?
      timeout -k 10 400 python3 tools/sweep.py --config reddit-f41 --grid "fpad=4,8,4,8;probe=0,1" --K 16 --reps 5 \
        > "$OUT/sweep_reddit_fpad_probe.log" 2>&1
      fatal sweep_reddit $?
      ;;
    pmcprobe)
      # PMC of the arxiv gather-only probe: requests, latency, L2 hits (compare profiles/r01/s38_pmc_deep.json)
      SESSION=${SESSION:-r02}/pmc_arxiv_probe CONFIG=ogbn-arxiv GRID="probe=1" KERNEL="cheb_step_kernel<4" PMC_K=16 \
        timeout -k 10 900 bash tools/pmc_deep.sh > "$OUT/pmc_arxiv_probe.log" 2>&1
      fatal pmc_arxiv_probe $?
      ;;
    parity)
      timeout -k 10 400 python3 tools/parity_distribution.py --out "$OUT/parity_distribution.json" > "$OUT/parity.log" 2>&1
      fatal parity $?
      ;;
    bench)
      timeout -k 10 500 python3 bench.py --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
      fatal bench $?
      ;;
    benchprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --sharded-extra none --cold-reps 0 \
        --connected-companion 0 > "$OUT/prof.log" 2>&1
      fatal benchprof $?
      ;;
    tracetiles)
      # the hybrid step (tiles.hip) on Reddit-size F=41 with its defaults: tile kernel + tail step kernel
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/trace_tiles -o run -- \
        python3 tools/tiles_probe.py --config reddit-f41 --sets "tiles=-1" --reps 5 > "$OUT/trace_tiles.log" 2>&1
      fatal trace_tiles $?
      cp /tmp/trace_tiles/run_kernel_stats.csv "$OUT/trace_tiles_kernel_stats.csv"
      ;;
    rehearse2)
      WATS_BENCH_PG=gloo WATS_BENCH_DEVICE=0 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
        --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29611 bench.py --gpus 2 --exchange ipc \
        --sharded-extra reddit --out "$OUT/rehearse2.json" > "$OUT/rehearse2.log" 2>&1
      fatal rehearse2 $?
      ;;
    *)
      if [ -n "${EXTRA:-}" ]; then timeout -k 10 900 bash -c "$EXTRA" > "$OUT/extra.log" 2>&1; fatal extra $?; fi
      ;;
  esac
done
echo done
