# shard probes: per-rank step of the Reddit-size shards (F = 1 LDS windows; F = 48 gather kernel, the F = 41
# headline's width) at 1 / 2 / 4 / 8 ranks
mkdir -p gpurun_out/r02_s11
for w in 1 2 4 8; do
  timeout -k 10 200 python tools/shard_probe.py --config reddit --world $w >> gpurun_out/r02_s11/shard_probe_reddit_f1.log 2>&1 || exit $?
  timeout -k 10 200 python tools/shard_probe.py --config reddit --world $w --F 48 >> gpurun_out/r02_s11/shard_probe_reddit_f48.log 2>&1 || exit $?
done
