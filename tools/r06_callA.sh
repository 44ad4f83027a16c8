set -u
mkdir -p gpurun_out/r06s3
timeout -k 10 500 python -u -m pytest tests/test_tiles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s3/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06s3/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/knob_ab.py --config ogbn-arxiv --sets "closed_side=0;closed_side=1" --rounds 3 --reps 20 > gpurun_out/r06s3/closed_side_ab.log 2>&1 || exit $?
cat gpurun_out/r06s3/closed_side_ab.log | cut -c1-220
WATS_HIP_LIB=$PWD/efficient-gnn_amd/wats_hip/libwats_hip_probes.so timeout -k 10 300 python -u tools/knob_ab.py --config ogbn-arxiv --sets "probe_ns=0,probe_h2=0;probe_ns=3,probe_h2=0;probe_ns=0,probe_h2=-1;probe_ns=0,probe_h2=-2;probe_ns=0,probe_h2=-3;probe_ns=0,probe_h2=-4" --rounds 2 --reps 20 > gpurun_out/r06s3/floor_probes.log 2>&1 || exit $?
cat gpurun_out/r06s3/floor_probes.log | cut -c1-220
