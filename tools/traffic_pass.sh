# FETCH_SIZE / WRITE_SIZE (+ L2 hit) passes of the bench's step kernel, each in its own rocprofv3 run
# (MI355X_MICROARCH.md "HBM": FETCH_SIZE counts half the bytes of wide reads on gfx950 -> doubled by
# tools/pmc_traffic.py); then the bench line with that per-launch traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-traffic}
mkdir -p "$OUT"
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_$tag" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sharded-extra none --cold-reps 0 --f1-companion 0 \
      --connected-companion 0 --pubmed-companion 0 > "$OUT/pmc_$tag.log" 2>&1
  rc=$?; echo "[pmc $tag] rc=$rc" | tee -a "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_traffic.py --kernel "cheb_step_kernel<4, true" "$OUT"/pmc_* --out "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1
rm -rf "$OUT"/pmc_FETCH_SIZE "$OUT"/pmc_WRITE_SIZE "$OUT"/pmc_TCC_HIT_sum
echo done
