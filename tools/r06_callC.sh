set -u
export TMPDIR=/tmp
O=gpurun_out/r06s5
mkdir -p $O
LEGS=reddit41,shard8 bash tools/pmc_legs.sh r06s5 || exit $?
for leg in reddit41 shard8; do
  case $leg in
    reddit41) cmd="python3 tools/sweep.py --config reddit-f41 --grid tile_th=96 --reps 3 --warm-s 0" ;;
    shard8) cmd="python3 tools/shard_probe.py --config reddit --world 8 --F 41 --reps 5" ;;
  esac
  rm -rf /tmp/kt_$leg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$leg -o run -- $cmd > $O/kt_$leg.log 2>&1 || exit $?
  cp "$(find /tmp/kt_$leg -name '*kernel_stats.csv' | head -1)" $O/kt_${leg}_kernel_stats.csv
done
WATS_HIP_LIB=$PWD/efficient-gnn_amd/wats_hip/libwats_hip_probes.so timeout -k 10 300 python3 -u tools/tier_probe.py --config reddit --world 8 --F 41 --delays 0,30,60 > $O/tier8.log 2>&1 || exit $?
tail -5 $O/tier8.log
