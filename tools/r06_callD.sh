set -u
export TMPDIR=/tmp
O=gpurun_out/r06s6
mkdir -p $O
LEGS=shard8 bash tools/pmc_legs.sh r06s6 || exit $?
rm -rf /tmp/kt_shard8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_shard8 -o run -- python3 tools/shard_probe.py --config reddit --world 8 --F 48 --reps 5 > $O/kt_shard8.log 2>&1 || exit $?
cp "$(find /tmp/kt_shard8 -name '*kernel_stats.csv' | head -1)" $O/kt_shard8_kernel_stats.csv
tail -3 $O/kt_shard8.log
