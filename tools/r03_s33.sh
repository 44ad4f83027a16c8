set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s33
for v in "" u8 u2; do
  WATS_HIP_LIB=$PWD/efficient-gnn_amd/wats_hip/libwats_hip${v:+_$v}.so timeout -k 10 300 python tools/shard_probe.py --config reddit --world 8 --F 48 --grid "waves=4;waves=8;waves=16" > gpurun_out/r03s33/v_${v:-base}.log 2>&1 || exit $?
done
